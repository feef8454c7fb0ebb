// vs_kernels.h — host-side launchers for the HIP kernels in vs_kernels.hip.
// Internal to the library; the public boundary is include/vsearch.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vsk {

// Query slots of the MFMA scan's buffers (most queries one launch handles:
// 8 waves x 32 at dim <= 768, 8 x 16 at dim 1024 / 1536; mfma_queries()).
constexpr uint32_t kMfmaQueries = 256;
// Largest k of the batched MFMA scan (candidate path); larger k uses the
// GEMV scan per query. The sorted-list pass (small collections, k <= 16)
// keeps kMfmaListMaxK keys per query in LDS.
constexpr uint32_t kMfmaMaxK = 128;
constexpr uint32_t kMfmaListMaxK = 16;
// Largest k of the list scans (GEMV register lists: 16 entries per lane) and
// of the one-workgroup merge; larger k takes the large-k path below.
constexpr uint32_t kMaxK = 1024;
// Large-k path (k > kMaxK; Qdrant serves any limit, rag/vector-service/
// main.go:252): per query, launch_gemv_scores writes every row's score image
// (the result key's high word: order-preserving, 0 = masked) and counts the
// first radix digit; launch_rsel finds the k-th largest 64-bit key by radix
// select (6 digits of 11/11/10 bits over the high word then the row word;
// a digit pass is skipped once the threshold's bucket holds exactly what is
// left to take) and compacts the k keys >= it; launch_sort_keys_desc sorts
// them. Exact, stream-ordered, no host round trip.
constexpr int kRselBits0 = 11;
constexpr int kRselBins = 1 << kRselBits0;
struct RselState {
  unsigned long long prefix;  // key bits fixed so far (the top plen bits)
  unsigned long long thr;     // when done: every key >= thr is selected
  uint32_t plen;              // bits fixed
  uint32_t krem;              // keys still to take inside the prefix bucket
  uint32_t done;
  uint32_t count;             // compaction cursor
};
hipError_t launch_gemv_scores(const void* X, bool bf16, uint32_t dim, uint32_t n_rows,
                              const float* q, const uint64_t* allow, uint32_t* sc, uint32_t* hist,
                              hipStream_t st);
// hist (kRselBins u32, the first digit's counts from launch_gemv_scores) is
// left zeroed; `keff` = min(k, unmasked rows) keys land in sel (unordered).
// The same selection in two launches (r03): hist1 = kRselBins u32 and ctr =
// 3 u32 (zero between calls, left zero), cand = n_rows keys of scratch; keff
// keys land in sel (unordered), hist is left zeroed.
hipError_t launch_rsel_fused(const uint32_t* sc, uint32_t n_rows, uint32_t row_base,
                             uint32_t keff, uint32_t* hist, uint32_t* hist1, uint32_t* ctr,
                             uint64_t* sel, uint64_t* cand, hipStream_t st);
hipError_t launch_rsel(const uint32_t* sc, uint32_t n_rows, uint32_t row_base, uint32_t keff,
                       uint32_t* hist, RselState* state, uint64_t* sel, hipStream_t st);
// Descending sort of n 64-bit keys (rocPRIM radix sort); temp / temp_bytes
// from sort_keys_temp_bytes(n).
size_t sort_keys_temp_bytes(uint64_t n);
hipError_t launch_sort_keys_desc(const uint64_t* in, uint64_t* out, uint64_t n, void* temp,
                                 size_t temp_bytes, hipStream_t st);
// Merge for any k (the large-k form of launch_merge): the L lists of each
// query concatenated, sorted (rocPRIM segmented radix sort), repeated keys
// dropped, the first k kept (0-padded). scratch: merge_large_scratch bytes.
size_t merge_large_scratch(uint32_t L, uint32_t nq, uint32_t kin);
hipError_t launch_merge_large(const uint64_t* lists, uint32_t L, uint64_t lstride,
                              uint64_t qstride, uint32_t nq, uint32_t kin, uint32_t k,
                              uint64_t* out, void* scratch, size_t scratch_bytes, hipStream_t st);
// MFMA passes: workgroups per launch (<= CUs), most candidate slots per
// (workgroup, query), sample-pass tiles per workgroup, and the select
// kernel's LDS buffer (candidates are streamed through it in chunks).
constexpr uint32_t kMfmaMaxLists = 256;
constexpr uint32_t kMfmaMaxCandCap = 1024;
constexpr uint32_t kMfmaMaxSampleTiles = 64;
constexpr uint32_t kMfmaSelBuf = 8192;

// Preprocess n fp32 vectors (n x dim, device) and store them as the
// collection dtype into dst rows: dst_rows[i] if non-null, else dst0 + i;
// also_bf16 (nullable) receives a bf16 copy at the same rows.
hipError_t launch_preprocess(const float* in, uint32_t n, uint32_t dim,
                             bool cosine, bool bf16, void* dst,
                             const uint64_t* dst_rows, uint64_t dst0,
                             hipStream_t st, uint16_t* also_bf16 = nullptr);

// Search-side query preprocess (Qdrant cosine normalise when `cosine`):
// qp (nullable) = fp32 queries, rounded to bf16 values when round_qp;
// qb (nullable) = bf16 copy. Bit-identical to launch_preprocess's values.
hipError_t launch_query_prep(const float* in, uint32_t n, uint32_t dim, bool cosine,
                             bool round_qp, float* qp, uint16_t* qb, hipStream_t st);

// Generate n synthetic unit rows with global numbers grow0 .. grow0+n-1 and
// store them into dst rows dst0 .. (bf16 or fp32), or as fp32 when f32_out.
// Global numbers advance by gstride per row (a shard of a row-striped
// collection holds every gstride-th global row).
hipError_t launch_generate(uint64_t seed, uint64_t grow0, uint64_t n,
                           uint32_t dim, bool bf16, void* dst, uint64_t dst0,
                           hipStream_t st, uint64_t gstride = 1);

// Single-query scan (GEMV) with per-wave register top-k. Writes one sorted
// key list of length k per workgroup to out[nlists][k]; returns nlists.
// `q` is dim fp32 on the device (already preprocessed / bf16-rounded).
hipError_t launch_gemv(const void* X, bool bf16, uint32_t dim, uint32_t n_rows,
                       uint32_t row_base, const float* q, uint32_t k,
                       uint64_t* out, uint32_t max_lists, uint32_t* nlists,
                       hipStream_t st, const uint64_t* allow = nullptr,
                       const uint32_t* rows = nullptr);
// With `rows` (device, n_rows entries of local row indices) the scan gathers
// those rows only (a selective filter) and `allow` is ignored.
// Filter bitmap -> the allowed local rows (< n_rows), ascending. `rows`
// holds popcount(allow) entries; `scratch` compact_scratch_words(n_rows) u32.
hipError_t launch_compact_rows(const uint64_t* allow, uint32_t n_rows, uint32_t* rows,
                               uint32_t* scratch, hipStream_t st);
uint32_t compact_scratch_words(uint32_t n_rows);
// One-launch search of a small collection for one raw (unpreprocessed)
// query: query prep + scan + merge in one workgroup, writing the k final keys
// to out[0, k). Bit-identical to launch_query_prep + launch_gemv +
// launch_merge. Only where gemv_small_ok (dim in the GEMV table up to 1536,
// rows <= kGemvSmallMaxRows, k <= kGemvSmallMaxK); unfiltered.
// With `part` (kGemvSmallMaxParts * kGemvSmallMaxK keys) and `counter` (one
// u32, zero between launches; the kernel leaves it zero), the rows are spread
// over gemv_small_parts() workgroups and the last one to finish merges; both
// buffers belong to one stream (concurrent launches need their own).
// With `flag`, `out` is mapped pinned host memory (k keys) and the kernel
// stores `seq` to *flag (mapped host memory) after the keys are visible to
// the host, which may then read them without waiting for the stream.
// With `q_host` (dim <= kGemvSmallArgDim) the raw query is read from host
// memory at launch and travels in the kernel arguments (q_raw unused).
constexpr uint32_t kGemvSmallArgDim = 768;  // 3 KiB of fp32 in the argument segment
constexpr uint32_t kGemvSmallMaxRows = 256;  // 32 rows per wave
constexpr uint32_t kGemvSmallMaxK = 16;  // the workgroup merge is serial in k
constexpr uint32_t kGemvSmallMaxParts = 16;
bool gemv_small_ok(uint32_t dim, uint32_t n_rows, uint32_t k);
uint32_t gemv_small_parts(uint32_t dim, bool bf16, uint32_t n_rows);
hipError_t launch_gemv_small(const void* X, bool bf16, uint32_t dim, uint32_t n_rows,
                             uint32_t row_base, const float* q_raw, bool cosine, uint32_t k,
                             uint64_t* out, hipStream_t st, uint64_t* part = nullptr,
                             uint32_t* counter = nullptr, uint64_t* flag = nullptr,
                             uint64_t seq = 0, const float* q_host = nullptr);

// One query in one launch (r03): the raw fp32 query q_raw (device) is
// preprocessed by every workgroup (as launch_query_prep), the scan writes
// per-workgroup lists to `lists` (gemv_max_lists(dim, bf16, n_rows, k)
// entries of k keys), and the last workgroup merges them into dst[0, k) --
// the same keys as query prep + launch_gemv + launch_merge, bit for bit.
// `counter`: one u32, zero between launches (the kernel leaves it zero), of
// this stream only; NULL = no merge (the lists are left for launch_merge).
// q_host (no merge, dim <= kGemvSmallArgDim): the raw query is read from host
// memory at launch and travels in the kernel arguments (q_raw unused). With `flag` (dst and flag mapped pinned host memory)
// `seq` is stored to *flag once dst is host-visible. gemv_one_ok: the GEMV
// table's dims up to 1024 and k <= 128 (register lists merged per workgroup).
bool gemv_one_ok(uint32_t dim, uint32_t k);
hipError_t launch_gemv_one(const void* X, bool bf16, uint32_t dim, uint32_t n_rows,
                           uint32_t row_base, const float* q_raw, bool cosine,
                           const uint64_t* allow, uint32_t k, uint64_t* lists, uint32_t max_lists,
                           uint32_t* counter, uint64_t* dst, hipStream_t st,
                           uint64_t* flag = nullptr, uint64_t seq = 0,
                           uint32_t* nlists = nullptr, const float* q_host = nullptr);

// Upper bound on the lists launch_gemv writes for these sizes.
uint32_t gemv_max_lists(uint32_t dim, bool bf16, uint32_t n_rows, uint32_t k);
// Single query on the int8 copy (r05): the int8 rows X8 (the
// batched prefilter's copy: tile bounds `meta`, scale `glob`) are scanned for
// every row's bracket L <= s <= U, then the rows whose U reaches a lower bound
// on the k-th score are rescored on the GEMV's own arithmetic from X: the keys
// equal launch_gemv_one's bit for bit. Two launches; `q_raw` is the raw query
// (prepped in the kernels as the one-launch GEMV does). dim 768 / 1024, k <=
// 128. scratch >= gemv_q8_scratch_bytes; ctr = 2 u32, zero between launches
// (left zero). dst receives k keys (mapped host memory with `flag`: seq is
// stored there once they are visible). stats (nullable, tests): [0] += rows
// rescored, [1] += workgroup lists replaced by all their rows. part: 1 = the
// scan launch, 2 = the finishing launch, 3 = both (the engine brackets them
// with separate timing events).
bool gemv_q8_ok(uint32_t dim, uint32_t k);
uint32_t gemv_q8_lists(uint32_t n_rows);
size_t gemv_q8_scratch_bytes(uint32_t n_rows, uint32_t k);
hipError_t launch_gemv_q8(int part, const void* X, bool bf16, const int8_t* X8, const float* meta,
                          const float* glob, uint32_t dim, uint32_t n_rows, uint32_t row_base,
                          const float* q_raw, bool cosine, const uint64_t* allow, uint32_t k,
                          void* scratch, size_t scratch_bytes, uint32_t* ctr, uint64_t* dst,
                          hipStream_t st, uint64_t* flag = nullptr, uint64_t seq = 0,
                          uint32_t* stats = nullptr,
                          uint64_t* clk = nullptr);  // (tools) [finish wg][8] stage clocks

// Batched scan on MFMA with fused top-k: bf16 rows on
// v_mfma_f32_16x16x32_bf16, or fp32 rows (f32) on v_mfma_f32_16x16x4_f32.
// X and Q are the collection's dtype; Q is kMfmaQueries x dim (zero-padded),
// nq_valid <= mfma_queries(dim, f32), k <= kMfmaMaxK; one workgroup per CU
// streams a contiguous row range (nlists workgroups).
//  * sample pass: first max_tiles 32-row tiles of every workgroup; each
//    tile's (masked) maximum score per query -> tmax[kMfmaQueries][m], m =
//    nlists * max_tiles (-inf past a workgroup's last tile);
//    launch_sample_bound then gives per query the k-th largest of those
//    maxima: k distinct rows reach it, so it lower-bounds the k-th score;
//  * main pass: every row; a lane whose 8 scores of a tile reach the
//    per-query lower bound init_score[q] appends them as one slab
//    (8 f32, the accumulator layout) and the tile's first global row to the
//    query's buffer: slabs[nlists][kMfmaQueries][cap][8],
//    slab_tile[nlists][kMfmaQueries][cap] (cap % 4 == 0, cap >= 4 k:
//    quarter j of a buffer is lane j's, counts in slabs
//    cand_cnt[nlists][256][4]); a full quarter keeps its cap / 4 best slabs
//    (exact for k <= cap / 4, never overflows); cand_max (nullable, same
//    shape): each quarter's largest admitted score (vs::score_ord, 0 = no
//    slab), which lets the select read only the few quarters that can hold
//    a top-k key (r04);
//    launch_select_slabs picks the top k;
//  * lists pass (k <= kMfmaListMaxK): the main pass with per-query sorted
//    lists in LDS (any input) -> lists[nlists][kMfmaQueries][k]; collections
//    of fewer than 8 tiles per workgroup, where the sample bound has too
//    few tiles to be worth a pass.
// `allow` (nullable, all passes): filter pre-mask, bit r of allow[r / 64]
// admits local row r; masked rows are never candidates, maxima or results.
bool mfma_supported(uint32_t dim, bool f32);
uint32_t mfma_queries(uint32_t dim, bool f32);  // queries per launch at this dim
hipError_t launch_mfma_sample(const void* X, bool f32, uint32_t dim, uint32_t n_rows,
                              uint32_t row_base, const void* Q, uint32_t nq_valid,
                              uint32_t k, uint32_t max_tiles, float* tmax, uint32_t max_lists,
                              uint32_t* nlists, hipStream_t st, const uint64_t* allow = nullptr,
                              const uint32_t* run_if = nullptr);
// bound[q] = the k-th largest of tmax[q][0, m) (radix select; -inf if m < k).
hipError_t launch_sample_bound(const float* tmax, uint32_t m, uint32_t nq, uint32_t k,
                               float* bound, hipStream_t st, const uint32_t* run_if = nullptr);
hipError_t launch_mfma_cand(const void* X, bool f32, uint32_t dim, uint32_t n_rows,
                            uint32_t row_base, const void* Q, uint32_t nq_valid, uint32_t k,
                            const float* init_score, float* slabs,
                            uint32_t* slab_tile, uint32_t cand_cap,
                            uint32_t* cand_cnt, uint32_t max_lists, uint32_t* nlists,
                            hipStream_t st, const uint64_t* allow = nullptr,
                            uint32_t* cand_max = nullptr, const uint32_t* run_if = nullptr);
hipError_t launch_mfma_lists(const void* X, bool f32, uint32_t dim, uint32_t n_rows,
                             uint32_t row_base, const void* Q, uint32_t nq_valid,
                             uint32_t k, const float* init_score, uint64_t* lists,
                             uint32_t max_lists,
                             uint32_t* nlists, hipStream_t st, const uint64_t* allow = nullptr);
// Top-k of the main pass's slab buffers (see launch_mfma_cand) for queries
// 0 .. nq-1 -> out[nq][k], sorted, 0-padded; the main pass leaves masked rows
// in its slabs, so the select applies the same pre-mask `allow` (local rows =
// global - row_base).
hipError_t launch_select_slabs(const float* slabs, const uint32_t* slab_tile,
                               const uint32_t* cand_cnt, uint32_t nwg, uint32_t cap, uint32_t nq,
                               uint32_t k, uint64_t* out, hipStream_t st, uint32_t row_base = 0,
                               const uint64_t* allow = nullptr,
                               const uint32_t* cand_max = nullptr,
                               const uint32_t* run_if = nullptr);
// run_if (nullable, both launches above): the launch does nothing unless
// *run_if != 0 -- the bf16 pass standing behind the int8 prefilter.

// int8 prefilter (r04, DESIGN.md §5 "int8 prefilter"): bf16 collections
// keep an int8 copy X8 (x ~ S * x8, one scale S per collection) and per
// 32-row tile {dt, nt} = the largest |x - S x8| and |x| of its rows, rounded
// up; glob = {absmax, dmax, nmax, S}. The main pass runs on
// v_mfma_i32_16x16x64_i8 (twice the bf16 rate, half the bytes) against int8
// queries Q8 with per-query {sqS, a, c, sigma} (q8par) and admits every row
// whose upper bound on its fp32 score reaches the sample bound;
// launch_select_q8 bounds, rescores the survivors from the bf16 rows and
// writes the top k; `allow` (nullable) is the pre-mask, as the bf16 pass's.
// A full quarter keeps counting (its count then passes its capacity) and its
// largest dot stays exact; the select recomputes such a quarter's rows from
// the int8 copy X8 with the queries' images Q8 and streams more survivors
// than its buffer through a running top k (r05; r04 handed the batch to a
// gated bf16 pass instead). Exact: the answer is the bf16 pass's.
// dims with an int8 pass: bf16 rows 768 / 1024, fp32 rows 768 (r04)
bool q8_supported(uint32_t dim, bool f32);
hipError_t launch_mfma_cand_q8(const void* X8, uint32_t dim, uint32_t n_rows, uint32_t row_base,
                               const void* Q8, uint32_t nq_valid, uint32_t k,
                               const float* init_score, const float* q8par, const float* q8glob,
                               float* slabs, uint32_t* slab_tile, uint32_t cand_cap,
                               uint32_t* cand_cnt, uint32_t* cand_max, uint32_t max_lists,
                               uint32_t* nlists, uint32_t* gate, hipStream_t st,
                               const uint64_t* allow = nullptr, const uint32_t* run_if = nullptr);
// cand_max (same shape as cand_cnt): each quarter's largest appended dot
// (int32; INT_MIN when empty), so the select reads only the quarters that
// can hold a top-k row.
// X / Q: the collection's rows and the pass's queries in its dtype (bf16, or
// fp32 when f32: survivors rescored on the f32 pass's 16x16x4 chain).
struct SpecVerifyArgs;  // below
hipError_t launch_select_q8(const float* slabs, const uint32_t* slab_tile, const uint32_t* cand_cnt,
                            const uint32_t* cand_max, uint32_t nwg, uint32_t cap, uint32_t nq,
                            uint32_t k, uint64_t* out,
                            uint32_t row_base, const void* X, const void* qb, bool f32, uint32_t dim,
                            const float* q8par, const float* q8glob, const float* meta,
                            const float* bound, const void* X8, const void* Q8,
                            const uint64_t* allow, uint32_t n_rows, hipStream_t st,
                            uint32_t* stats = nullptr,  // (tools) += slabs read, survivors, slow paths
                            uint64_t* clk = nullptr,    // (tools) [nq][16] stage wall clocks
                            const uint32_t* run_if = nullptr,   // stand down unless *run_if
                            // (r06 ablation) the batch's check or record by the select's
                            // last workgroup (instead of launch_q8_verify_record after it)
                            const SpecVerifyArgs* verify = nullptr);
// Store side (vs_q8.hip; X: bf16 rows, or fp32 rows when f32): glob[0] = max
// |x| over n values (atomic max; zero it first); glob[3] = S = glob[0] / 127
// (1 when 0).
hipError_t launch_q8_absmax(const void* X, bool f32, uint64_t n, float* glob, hipStream_t st);
hipError_t launch_q8_set_scale(float* glob, hipStream_t st);
// Requantise whole 32-row tiles (tiles[i] if non-null, else t0 + i; rows past
// n_rows are written as zeros) with the scale glob[3]: X8, meta[tile] = {dt,
// nt}, and glob[1], glob[2] raised to the tiles' maxima.
hipError_t launch_q8_quantize(const void* X, bool f32, uint32_t n_rows, uint32_t dim,
                              const uint32_t* tiles, uint32_t t0, uint32_t ntiles, int8_t* X8,
                              float* meta, float* glob, hipStream_t st);
// Speculative bound, device state after a collection's int8
// bounds {absmax, dmax, nmax, S} in the same allocation (q8_glob):
//   Q8SpecStat at byte 16: cumulative counters, zeroed when the copy is made;
//   Q8SpecK[kQ8SpecK] at byte 48: per k, zeroed by every store-side write.
// ratio: the k-th exact score per unit |q| a speculative batch of this k (or
// a smaller one) starts from, 0 = unset. It is REPLACED by every batch that
// verifies or is answered on the sample path: 0.97 x a low quantile (the
// 1 + n/64-th smallest) of that batch's ratios, so up to n/64 outlier queries
// (a k-th far under the others') never lower it (r06). backoff: the cool-down
// the next failed check sets (0, 1, 2, 4 ... 64 batches on the sample path
// over consecutive failures; 0 again after a verified batch), handed to the
// host through its advice words (launch_q8_verify_record).
// loose: set by a sample-path batch when ratio x |q| falls under more than a
// quarter of its queries' sample bounds -- a single ratio cannot follow the
// queries' own k-th scores (clustered rows), so speculating would admit more
// rows than the sample pass does; no speculative batch runs while it is set.
// since: speculative batches since the last sample-path one; every
// kQ8SpecProbe-th runs the sample path instead, which re-judges `loose`.
struct Q8SpecStat {
  unsigned long long tries;    // speculative batches run
  unsigned long long fails;    // of those, failed their check: the sample path re-answered
  unsigned long long skipped;  // sent to the sample path by the device (ratio unset,
                               // loose or a probe; host-side skips: Collection)
  unsigned long long spare;
};
struct Q8SpecK {
  float ratio;
  uint32_t backoff, loose, since, pad[4];
};
constexpr uint32_t kQ8SpecK = kMfmaMaxK + 1;
constexpr size_t kQ8SpecStatOff = 16, kQ8SpecKOff = 48;
constexpr size_t kQ8GlobBytes = kQ8SpecKOff + (size_t)kQ8SpecK * sizeof(Q8SpecK);
constexpr uint32_t kQ8SpecMaxBackoff = 64;
constexpr uint32_t kQ8SpecProbe = 64;
inline Q8SpecStat* q8_spec_stat(float* glob) {
  return (Q8SpecStat*)((char*)glob + kQ8SpecStatOff);
}
inline Q8SpecK* q8_spec_k(float* glob) { return (Q8SpecK*)((char*)glob + kQ8SpecKOff); }
// The batch's control words (after q8par's kMfmaQueries x 4 floats): [0] the
// verdict (the sample path runs unless 0), [1] a forced ratio (tests), [2] go
// (the speculative launches run unless 0).
constexpr uint32_t kGateVerdict = 0, kGateForced = 1, kGateGo = 2;

// (r06) What the int8 select's last workgroup needs to check / record a batch
// (vs_spec_dev.h). vq: one float4 per query (r, |q|, bound, ok) handed over by
// every workgroup; ticket: one u32, zero between launches (the last workgroup
// leaves it zero).
struct SpecVerifyArgs {
  uint32_t check;  // 1: check a speculative batch; 0: record a sample-path one
  uint32_t dim;
  const float* bound;
  const float* q8par;
  const float* glob;
  uint32_t* gate;
  Q8SpecK* sk;
  Q8SpecStat* stat;
  uint32_t* advice;
  float4* vq;
  uint32_t* ticket;
};
// The int8-query buffer's layout (engine scratch, kMfmaQueries slots): q8par
// (4 floats a query), then the gate words (64 B), the verify hand-over vq (one
// float4 a query) and its ticket.
constexpr size_t kQ8ParBytes = (size_t)kMfmaQueries * 16 + 64 + (size_t)kMfmaQueries * 16 + 64;

// Queries (bf16, or fp32 when f32; nq x dim) -> int8 rows Q8 and q8par[q] =
// {sq * S, |sq q8|, |q - sq q8|, sigma}, norms rounded up.
// Also zeroes gate[kGateVerdict] ahead of the int8 pass.
// Speculative form (spec_k non-null): also bound[q] = *ratio x |q|, and the
// batch's go / verdict words: go = 1, verdict = 0 when *ratio is set and
// (unless force) spec_k is neither loose nor due a probe; else go = 0,
// verdict = 1 (the sample path answers).
hipError_t launch_q8_query(const void* q, bool f32, uint32_t nq, uint32_t dim, const float* glob,
                           int8_t* q8, float* q8par, uint32_t* gate, hipStream_t st,
                           const float* ratio = nullptr, float* bound = nullptr,
                           Q8SpecK* spec_k = nullptr, Q8SpecStat* stat = nullptr,
                           bool force = false);
constexpr uint32_t kQueryPrepFusedMaxDim = 1536;  // = 64 x vs_qprep_dev.h kQPrepMax
// (r06) The speculative form of launch_q8_query fused with launch_query_prep
// (dim <= kQueryPrepFusedMaxDim): the raw fp32 queries `in` -> qp / qbf exactly as
// launch_query_prep(in, nq, dim, cosine, round_qp, qp, qbf) writes them, and
// the int8 images, bounds and go / verdict words exactly as launch_q8_query
// over qp (f32) or qbf -- one launch.
hipError_t launch_q8_prep_query(const float* in, bool cosine, bool round_qp, float* qp,
                                uint16_t* qbf, bool f32, uint32_t nq, uint32_t dim,
                                const float* glob, int8_t* q8, float* q8par, uint32_t* gate,
                                hipStream_t st, const float* ratio, float* bound, Q8SpecK* spec_k,
                                Q8SpecStat* stat, bool force);
// After a batch's select (one workgroup; nq <= kMfmaQueries). check (a
// speculative batch): a query whose k-th exact score is under its bound -
// sigma nmax fails it; any failure sets gate[kGateVerdict] (the sample path
// re-answers the batch), counts it and starts a cool-down (spec_k->backoff); a
// verified batch clears the back-off. A verified batch, or any batch with
// check off (the sample path's answer: `bound` then holds its sample bounds,
// which also re-judge spec_k->loose), replaces spec_k->ratio (see Q8SpecK).
// advice (nullable; coherent mapped host memory, this k's word of the
// collection's 2 x kQ8SpecK): the record stores loose (1: the host enqueues
// the sample path alone), a failed check stores the cool-down's length at
// advice[kQ8SpecK] (the host counts it off). run_if: stand down unless *run_if.
hipError_t launch_q8_verify_record(const uint64_t* keys, uint32_t nq, uint32_t k, uint32_t dim,
                                   const float* bound, const float* q8par, const float* glob,
                                   bool check, uint32_t* gate, Q8SpecK* spec_k, Q8SpecStat* stat,
                                   uint32_t* advice, hipStream_t st,
                                   const uint32_t* run_if = nullptr);
// launch_sample_bound (nq_bound queries) and launch_q8_query (nq queries) as
// one launch: the int8 path's per-batch prep, one dispatch fewer (r04).
hipError_t launch_sample_bound_q8(const float* tmax, uint32_t m, uint32_t nq_bound, uint32_t k,
                                  float* bound, const void* q, bool f32, uint32_t nq,
                                  uint32_t dim, const float* glob, int8_t* q8, float* q8par,
                                  uint32_t* gate, hipStream_t st, const uint32_t* run_if = nullptr);
// Radix passes of the sample bound (VS_BOUND_PASSES, read once; default 2).
int sample_bound_passes();
// Sample tiles per workgroup, and the main pass's candidate capacity per
// (workgroup, query) sized from the expected survivors of the sample bound.
uint32_t mfma_sample_tiles(uint32_t n_rows, uint32_t dim = 768, bool f32 = false);
// (scale: expected survivors relative to the bf16 pass's; the int8 pass
// admits ~4x as many rows, its upper bounds being looser than exact scores)
uint32_t mfma_cand_cap(uint32_t n_rows, uint32_t k, uint32_t sample_tiles, double scale = 1.0);
uint32_t mfma_max_lists(uint32_t n_rows);
uint32_t mfma_tiles_per_wg(uint32_t n_rows);
void mfma_grid(uint32_t n_rows, uint32_t* nwg, uint32_t* rows_per_wg);

// Merge L sorted key lists per query -> out [nq][k] (global top-k by key).
// List l of query q starts at lists[l * lstride + q * qstride], kin entries.
// With `flag` (nq == 1; out and flag in mapped pinned host memory) every
// writer fences at system scope, then `seq` is stored to *flag: the host may
// read out once it sees seq (as launch_gemv_small's completion word).
hipError_t launch_merge(const uint64_t* lists, uint32_t L, uint64_t lstride,
                        uint64_t qstride, uint32_t nq, uint32_t kin, uint32_t k,
                        uint64_t* out, hipStream_t st, uint64_t* flag = nullptr,
                        uint64_t seq = 0);

// Convert fp32 queries (nq x dim) to bf16 (after preprocessing).
hipError_t launch_to_bf16(const float* in, uint64_t n, uint16_t* out,
                          hipStream_t st);
// fp32 -> fp32 with bf16 rounding (values exactly representable in bf16).
hipError_t launch_round_bf16(const float* in, uint64_t n, float* out,
                             hipStream_t st);

// Snapshot checksum of nbytes at p (vs::snap_word summed) -> *d_out (device).
hipError_t launch_checksum(const void* p, uint64_t nbytes, uint64_t* d_out, hipStream_t st);
// The same over one shard of a row-striped collection: rows x row_bytes
// (row_bytes % 8 == 0), local row l = global row l * stride + offset.
hipError_t launch_checksum_rows(const void* p, uint64_t rows, uint32_t row_bytes, uint64_t stride,
                                uint64_t offset, uint64_t* d_out, hipStream_t st);
// Shard keys (local rows) -> global rows base + local * stride + offset.
hipError_t launch_remap_keys(uint64_t* keys, uint64_t n, uint32_t stride, uint32_t offset,
                             uint32_t base, hipStream_t st);

int device_cu_count();

}  // namespace vsk
