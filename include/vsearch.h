/*
 * vsearch.h — C-ABI of the MI355X exact top-k vector search engine.
 *
 * This is the drop-in boundary for GoRilla-RAG's rag/vector-service. In the
 * reference, vector-service is a Go HTTP shim over a Qdrant server reached by
 * gRPC. Its engine calls are exactly five:
 *
 *   Collections.Get      rag/vector-service/main.go:91   -> vs_collection_info
 *   Collections.Create   rag/vector-service/main.go:102  -> vs_collection_create
 *   Qdrant.HealthCheck   rag/vector-service/main.go:126  -> vs_health
 *   Points.Upsert        rag/vector-service/main.go:209  -> vs_upsert
 *   Points.Search        rag/vector-service/main.go:249  -> vs_search
 *
 * The gRPC client globals they go through (main.go:44-51, created at
 * main.go:56-65) are replaced by one engine handle from vs_open.
 *
 * Conventions
 *  - Plain C types only: no HIP, torch or Go types in any signature.
 *  - Every function returns VS_OK (0) or a negative vs_status. The message of
 *    the last failure on the calling thread is available from vs_last_error().
 *  - The caller owns every buffer it passes. The library copies inputs before
 *    returning and never keeps a caller pointer (this satisfies cgo's pointer
 *    passing rules for Go slices).
 *  - The engine deals in dense row numbers only. Point UUIDs and payloads stay
 *    on the caller's side, exactly as the Go service keeps
 *    them outside the engine.
 *  - Thread safety: every entry point may be called concurrently. Collections
 *    are guarded by reader/writer locks (upsert = writer, search = reader).
 *
 * Search semantics (what Qdrant's exact search returns for SearchPoints with
 * no filter/offset/threshold, rag/vector-service/main.go:249-254):
 *  - COSINE: both the stored rows and the query are L2-normalised
 *    ("cosine preprocess"); the score is the dot product of the normalised
 *    vectors. A vector whose squared norm is < FLT_EPSILON, or within 1e-6 of
 *    1, is left unchanged.
 *  - DOT: plain inner product, no preprocessing.
 *  - Results are ordered by score descending; equal scores are ordered by row
 *    ascending (the reference leaves tie order unspecified; this fixes it).
 *  - min(k, rows) results are returned per query.
 *  - BF16 collections store the preprocessed row rounded to bfloat16
 *    (round-to-nearest-even); queries are preprocessed in fp32 then rounded
 *    to bf16; products are accumulated in fp32.
 */
#ifndef VSEARCH_H_
#define VSEARCH_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VSEARCH_ABI_VERSION 1

typedef struct vs_engine vs_engine;

typedef enum vs_status {
  VS_OK = 0,
  VS_ERR_INVALID_ARG = -1,  /* bad argument (maps to HTTP 400 in the service) */
  VS_ERR_NOT_FOUND = -2,    /* unknown collection (mirrors codes.NotFound, main.go:96) */
  VS_ERR_DIM_MISMATCH = -3, /* vector length != collection dim */
  VS_ERR_OOM = -4,          /* device or host allocation failed */
  VS_ERR_DEVICE = -5,       /* HIP runtime error, or no usable GPU */
  VS_ERR_EXISTS = -6,       /* collection already exists */
  VS_ERR_INTERNAL = -7,
  VS_ERR_IO = -8            /* snapshot file unreadable, unwritable or corrupt */
} vs_status;

/* Mirrors qdrant.Distance (main.go:108 uses Distance_Cosine). */
typedef enum vs_metric { VS_METRIC_COSINE = 0, VS_METRIC_DOT = 1 } vs_metric;

/* Storage element type of a collection. */
typedef enum vs_dtype { VS_DTYPE_F32 = 0, VS_DTYPE_BF16 = 1 } vs_dtype;

typedef struct vs_config {
  int32_t device; /* HIP device ordinal this engine owns; -1 = current device */
  uint32_t flags; /* VS_FLAG_* */
} vs_config;

/* Record HIP events around every scan launch (read with vs_timing). */
#define VS_FLAG_TIMING 1u
/* ... and around every merge / select launch too. Each event record costs a
 * few microseconds of device idle between launches, so the benchmark times
 * scans only. */
#define VS_FLAG_TIMING_MERGE 2u
/* With VS_FLAG_TIMING: bracket only one scan launch in 4 (batches) or in 16
 * (one query: every 4th cost a single-query step 1.5%), the 4th / 16th after a
 * vs_timing reset first: a sampled average that keeps the event gaps out of
 * the other steps and the first scan after a synchronize out of the sample. */
#define VS_FLAG_TIMING_SAMPLE 4u
/* vs_open_multi only: place every collection WHOLE on one of the engine's
 * devices (the one with the fewest bytes reserved by capacity hints, then
 * the fewest collections) instead of row-striping it over all shards. Each
 * call then goes to that device alone, so calls for collections on
 * different devices run concurrently and no collective is needed: the
 * layout for several independent collections that each fit one HBM (config
 * C5: 3 x 5M x 1024 bf16 = 10 GB each; the reference serves three
 * collections from concurrent handlers, main.go:77, :80-119). Row-striping
 * stays the layout for one collection larger than one device. */
#define VS_FLAG_PLACE_COLLECTIONS 8u
/* With VS_FLAG_PLACE_COLLECTIONS: one device engine (its own store, search
 * contexts and streams) per entry of `devices`, even where ordinals repeat,
 * so {0, 0} holds two placement slots on device 0. Collections placed on the
 * second slot take the cross-device path of vs_search_keys (query and key
 * copies ordered by events on the caller's stream) on a one-GPU host, where
 * it is otherwise only reachable with two GPUs. Ignored without placement:
 * RCCL holds one rank per device. */
#define VS_FLAG_ENGINE_PER_SHARD 16u
/* No int8 prefilter copies (r04) for this engine's collections: batched
 * searches of bf16 collections then always run the bf16 MFMA pass. By
 * default a bf16 collection (dim 768) that takes the batched candidate pass
 * keeps an int8 copy of its rows (+50% of its HBM) and answers batches from
 * an int8 MFMA pass whose candidates are rescored exactly from the bf16 rows:
 * the same keys as the bf16 pass ("int8 prefilter"). */
#define VS_FLAG_NO_PREFILTER 32u
/* (r06) No speculative bound for this engine's batched int8
 * searches: every batch runs the sample pass for its bound. Same keys either
 * way; the environment's VS_Q8_SPEC=0 does this for every engine. */
#define VS_FLAG_NO_SPECULATIVE 64u

/* ---- engine lifetime ---------------------------------------------------- */

/* Replaces grpc.DialContext + New{Collections,Points,Qdrant}Client
 * (rag/vector-service/main.go:56-65). Fails with VS_ERR_DEVICE when no HIP
 * device is usable: there is no CPU fallback. */
int vs_open(const vs_config* cfg, vs_engine** out);
void vs_close(vs_engine* eng);

/* ---- multi-GPU engine ------------------------------------
 * One process drives several devices, one engine handle for all of them
 * (the reference keeps one client handle per process, main.go:44-65).
 * Shard s lives on HIP device devices[s] (NULL: device s); a device may
 * hold several shards. Every collection of such an engine is row-striped:
 * global row g is stored by shard g % n_shards as its local row
 * g / n_shards, so appends (upsert, generate) spread evenly. Every entry
 * point below serves it unchanged: a search scans all shards, merges the
 * shards of each device on that device, all-gathers one [nq][k] key list per
 * device over RCCL (one communicator from ncclCommInitAll) and merges them on
 * the first device, whose stream and memory the device-pointer forms use.
 * row_base must be 0 (stripes, not blocks; a placed collection, see
 * VS_FLAG_PLACE_COLLECTIONS, takes any). Snapshots of a sharded
 * collection hold its rows in global order: the file is the same as that of
 * the collection on one device. n_shards == 1 is vs_open on devices[0]. */
typedef struct vs_config_multi {
  const int32_t* devices; /* n_shards HIP ordinals (may repeat); NULL = 0 .. n_shards-1 */
  uint32_t n_shards;
  uint32_t flags; /* VS_FLAG_* */
} vs_config_multi;

int vs_open_multi(const vs_config_multi* cfg, vs_engine** out);

/* Shards and distinct devices of an engine (1 and 1 for vs_open). */
int vs_engine_layout(vs_engine* eng, uint32_t* n_shards, uint32_t* n_devices);

/* The HIP device ordinal holding the whole collection, or -1 when it is
 * row-striped over several devices. Callers that schedule per device (the
 * service's batcher) key their queues on it. */
int vs_collection_placement(vs_engine* eng, const char* name, int32_t* device);

/* Number of visible HIP devices (0 when none). Never fails. */
int vs_device_count(void);

/* ---- collections ---------------------------------------------------------- */

/* Replaces Collections.Create (main.go:102-112). `capacity_hint` pre-reserves
 * rows in HBM (0 = grow on demand). `row_base` is the global number of this
 * collection's row 0: a shard of a row-sharded collection stores global rows
 * [row_base, row_base + rows). Single-GPU callers pass 0. */
int vs_collection_create(vs_engine* eng, const char* name, uint32_t dim,
                         int metric, int dtype, uint64_t capacity_hint,
                         uint64_t row_base);

/* Replaces Collections.Get (main.go:91). Any out pointer may be NULL. */
int vs_collection_info(vs_engine* eng, const char* name, uint32_t* dim,
                       uint64_t* rows, int* metric, int* dtype);

/* Frees the collection's device memory. */
int vs_collection_drop(vs_engine* eng, const char* name);

/* HBM bytes of the collection's int8 prefilter copy (summed over shards; 0 =
 * none: its batched searches run the bf16 pass). See VS_FLAG_NO_PREFILTER. */
int vs_collection_prefilter_bytes(vs_engine* eng, const char* name, uint64_t* bytes);

/* (r06, diagnostics; no reference counterpart) Counters of the speculative
 * bound of the collection's batched int8 searches, summed over
 * shards, after every search enqueued so far on its devices has finished:
 * out[0] speculative batches run, out[1] of those that failed their check (the
 * sample path re-answered them: `spec_fallbacks`), out[2] batches a cool-down
 * or an unset ratio sent to the sample path, out[3] 0. All zero without an
 * int8 copy. Counted since the copy was (re)built. */
int vs_collection_spec_stats(vs_engine* eng, const char* name, uint64_t out[4]);

/* ---- store side ----------------------------------------------------------- */

/* Replaces Points.Upsert(wait=true) (main.go:208-213): writes `n` vectors
 * (n x dim fp32, row-major; `dim` must equal the collection's, else
 * VS_ERR_DIM_MISMATCH) into local rows `rows[i]`. A row below the
 * collection's current row count is overwritten; rows at or above it are
 * appended and must form exactly the range [rows, rows + m) (no holes).
 * Duplicate rows in one call: the last occurrence wins. The vectors are
 * preprocessed on the device (COSINE) and stored as the collection dtype.
 * Returns after the data is resident. */
int vs_upsert(vs_engine* eng, const char* coll, uint64_t n, uint32_t dim,
              const uint64_t* rows, const float* vecs);

/* Appends `n` synthetic unit-norm rows generated on the device by the
 * counter-based generator of DESIGN.md §4 (seed, global row numbers
 * row_base + rows ... ). Used for benchmarks: no host data is moved. */
int vs_generate(vs_engine* eng, const char* coll, uint64_t n, uint64_t seed);

/* Writes n synthetic unit vectors (generator rows row0 .. row0+n-1 of `seed`)
 * as fp32 into the device buffer d_out (n x dim), ordered on `stream`. Used to
 * build benchmark queries on the device. */
int vs_generate_vectors(vs_engine* eng, uint64_t seed, uint64_t row0, uint64_t n,
                        uint32_t dim, float* d_out, void* stream);

/* Copies stored (preprocessed) rows [first, first + n) back to the host as
 * fp32 (bf16 rows are widened exactly). For verification. */
int vs_read_rows(vs_engine* eng, const char* coll, uint64_t first, uint64_t n,
                 float* out);

/* ---- search side ---------------------------------------------------------- */

/* Replaces Points.Search (main.go:249-254), batched: `nq` queries of `dim`
 * fp32 each (`dim` must equal the collection's, else VS_ERR_DIM_MISMATCH).
 * For query i, out_scores[i*k + j] / out_rows[i*k + j] hold the j-th best (score desc, row asc) for j < out_count[i] = min(k, rows).
 * Rows are global (row_base added). Blocking. Any k >= 1 (Qdrant's limit
 * is unbounded, main.go:252): k <= 1024 keeps the scans' register lists;
 * larger k scores every row once and selects the k-th key by a radix select
 * on the device (DESIGN.md §5 "Large k"). The output arrays are nq x k, so a
 * caller passes k <= rows where rows is large. */
int vs_search(vs_engine* eng, const char* coll, const float* queries,
              uint32_t nq, uint32_t dim, uint32_t k, float* out_scores,
              uint64_t* out_rows, uint32_t* out_count);

/* vs_search with a payload filter pre-mask: only local
 * rows r with bit (allow[r / 64] >> (r % 64)) & 1 set can be returned;
 * out_count[i] = min(k, allowed rows). `allow_words` >= ceil(rows / 64); bits
 * past the last row are ignored. Batched (MFMA) searches apply the bitmap
 * inside the scan kernels (rows are read but never become candidates), so
 * they cost what an unfiltered search does. GEMV-path searches (one query,
 * fp32, or k > 128) with at most 1/8 of the rows allowed scan only the
 * allowed rows, gathered through a compacted row list built on the device.
 * The reference accepts `filter` and ignores it (main.go:30 vs :249-254); the
 * service mirror applies it only when configured to. */
int vs_search_filtered(vs_engine* eng, const char* coll, const float* queries, uint32_t nq,
                       uint32_t dim, uint32_t k, const uint64_t* allow, uint64_t allow_words,
                       float* out_scores, uint64_t* out_rows, uint32_t* out_count);

/* Device-resident filters: a filter the caller will reuse (the service caches
 * one per canonical `filter` object) is uploaded once: the bitmap, its
 * popcount and, when at most 1/8 of the rows are allowed, the compacted row
 * list stay in HBM, so vs_search_filter_id ships no bitmap and builds no list
 * per call. A filter is bound to the collection and its row count at
 * creation: a search after rows were added fails with VS_ERR_INVALID_ARG
 * (rebuild it). Bits are rows, not payloads: a caller whose payloads changed
 * must rebuild it too. Ids are never reused within an engine. */
int vs_filter_create(vs_engine* eng, const char* coll, const uint64_t* allow,
                     uint64_t allow_words, uint64_t* filter_id);
int vs_filter_drop(vs_engine* eng, uint64_t filter_id);
/* vs_search_filtered with a filter made by vs_filter_create. */
int vs_search_filter_id(vs_engine* eng, const char* coll, const float* queries, uint32_t nq,
                        uint32_t dim, uint32_t k, uint64_t filter_id, float* out_scores,
                        uint64_t* out_rows, uint32_t* out_count);

/* Device-pointer form for sharded callers. `d_queries` (nq x dim fp32) and
 * `d_keys` (nq x k uint64) are device pointers on this engine's device;
 * `stream` is a hipStream_t (NULL = the null stream). The work is ordered
 * after prior work on `stream`, and later work on `stream` sees the result.
 * Each result is a 64-bit key (see below); unused slots hold 0.
 * The stream and the pointers must come from the HIP runtime this library
 * is linked to: in a process that maps two libamdhip64 runtimes (e.g.
 * torch's bundled copy next to /opt/rocm's) this call and every other one
 * taking caller device pointers (vs_merge_keys, vs_gather_merge_keys,
 * vs_decode_keys, vs_generate_vectors) fail with VS_ERR_DEVICE rather than
 * run unordered with the caller's work. vs_runtime_check() runs that test
 * alone (no device needed): VS_OK, or VS_ERR_DEVICE naming both runtimes. */
int vs_runtime_check(void);
int vs_search_keys(vs_engine* eng, const char* coll, const float* d_queries,
                   uint32_t nq, uint32_t dim, uint32_t k, uint64_t* d_keys,
                   void* stream);

/* Merges `n_lists` per-shard key lists into the global top-k on the device:
 * d_lists is [n_lists][nq][k_in] (e.g. the result of an all-gather of
 * vs_search_keys outputs); d_out_keys is [nq][k]. Each list is sorted
 * descending without repeats, 0-padded (as vs_search_keys writes it). A key
 * found in more than one list (overlapping or replicated shards) is returned
 * once; slots past the number of distinct non-zero keys hold 0. */
int vs_merge_keys(vs_engine* eng, const uint64_t* d_lists, uint32_t n_lists,
                  uint32_t nq, uint32_t k_in, uint32_t k, uint64_t* d_out_keys,
                  void* stream);

/* ---- one process per GPU (row shards across processes) --------------------
 *
 * Each process opens its own single-device engine (vs_open) over its shard
 * of rows (vs_collection_create with row_base = the shard's first global
 * row). One rank makes an RCCL unique id; every rank receives those bytes
 * over any host transport (the launcher's store, a socket, an env var) and
 * calls vs_comm_init with the same id, its rank and the rank count (a
 * collective call: it returns once all ranks joined). vs_gather_merge_keys
 * then turns each rank's vs_search_keys output into the global top-k on
 * every rank: ONE RCCL all-gather of the ranks' [nq][k_in] lists over xGMI
 * and the vs_merge_keys merge, both on `stream`, with nothing between them
 * (no event or cross-stream wait; every rank must make the same sequence of
 * calls with the same nq / k_in / k). Replaces a framework all-gather +
 * vs_merge_keys pair (the form shard.py uses with gloo). Not available on a
 * vs_open_multi engine, which holds its own communicator. */
#define VS_COMM_ID_BYTES 128
int vs_comm_unique_id(unsigned char id[VS_COMM_ID_BYTES]);
int vs_comm_init(vs_engine* eng, uint32_t n_ranks, uint32_t rank,
                 const unsigned char id[VS_COMM_ID_BYTES]);
/* d_local [nq][k_in] and d_out_keys [nq][k] on this engine's device. */
int vs_gather_merge_keys(vs_engine* eng, const uint64_t* d_local, uint32_t nq,
                         uint32_t k_in, uint32_t k, uint64_t* d_out_keys,
                         void* stream);

/* Decodes device keys into host scores/rows/counts (blocking D2H). */
int vs_decode_keys(vs_engine* eng, const uint64_t* d_keys, uint32_t nq,
                   uint32_t k, float* out_scores, uint64_t* out_rows,
                   uint32_t* out_count, void* stream);

/* Result key layout (host helpers below are the reference definition):
 *   key = ord(score) << 32 | (0xFFFFFFFF - row)
 * where ord() maps fp32 bits to an order-preserving uint32 (-0.0 is encoded
 * as +0.0). Larger key =
 * better result (higher score; lower row on equal score). 0 = empty slot. */
static inline uint64_t vs_key_encode(float score, uint32_t row) {
  union { float f; uint32_t u; } c; c.f = score == 0.0f ? 0.0f : score;
  uint32_t o = (c.u & 0x80000000u) ? ~c.u : (c.u | 0x80000000u);
  return ((uint64_t)o << 32) | (uint32_t)(0xFFFFFFFFu - row);
}
static inline float vs_key_score(uint64_t key) {
  uint32_t o = (uint32_t)(key >> 32);
  union { float f; uint32_t u; } c;
  c.u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
  return c.f;
}
static inline uint32_t vs_key_row(uint64_t key) {
  return 0xFFFFFFFFu - (uint32_t)key;
}

/* ---- snapshot / restore --------------------------------- */

/* Replaces Qdrant's persistent volume (docker-compose.yml:9-10,14-15): the
 * HBM-resident store is otherwise volatile. vs_snapshot writes a collection's
 * rows, exactly as stored (preprocessed, fp32 or bf16), to `path`:
 * a 128-byte header (magic "VSNAP01\0", version, dim, metric, dtype,
 * element bytes, rows, row_base, data bytes, checksum of the data, checksum
 * of the header) followed by rows x dim elements, row-major, little-endian.
 * The checksum is vs_checksum's, computed on the device. Concurrent searches
 * proceed; upserts wait. */
int vs_snapshot(vs_engine* eng, const char* coll, const char* path);

/* Creates collection `coll` (which must not exist) from a snapshot file,
 * bit-exact, with capacity for its rows. The data checksum is recomputed on
 * the device after the upload; on any mismatch or I/O error the collection
 * is not created and VS_ERR_IO is returned. `row_base` is taken from the file. */
int vs_restore(vs_engine* eng, const char* coll, const char* path);

/* Checksum of a collection's stored rows (rows x dim elements as stored):
 * sum over little-endian 64-bit words w_i of splitmix64(w_i ^ i * 0x9E37..15)
 * mod 2^64 (vs_common.h snap_word; oracle/vsearch_oracle.c restates it). */
int vs_checksum(vs_engine* eng, const char* coll, uint64_t* out);

/* ---- health / errors / timing -------------------------------------------- */

/* Replaces Qdrant.HealthCheck (main.go:126). Writes a NUL-terminated JSON
 * object {"status":"healthy"|"degraded","engine":"vsearch-hip",...}. */
int vs_health(vs_engine* eng, char* buf, size_t len);

/* Thread-local message of the last failure ("" if none). */
const char* vs_last_error(void);

/* Copies the calling thread's last error message into buf (NUL-terminated,
 * truncated to len - 1 bytes) and returns its full length. For bindings
 * whose calls may migrate between OS threads (cgo): a wrapper that makes
 * the failing call and this copy inside ONE foreign call reads the message
 * of that call, not of whatever ran on the thread in between. */
size_t vs_copy_last_error(char* buf, size_t len);

/* Provenance: the first 16 hex digits of the sha256 over the sources this
 * library was linked from (build.py tree_hash(): every source under csrc,
 * the headers under include, and build.py). Never fails. */
const char* vs_build_id(void);

/* With VS_FLAG_TIMING (and VS_FLAG_TIMING_MERGE): average device duration
 * (ms) of scan (and merge) kernel launches recorded since the last reset, and
 * their counts. Blocks until the
 * recorded work is done. reset != 0 clears the accumulators afterwards. */
int vs_timing(vs_engine* eng, double* scan_ms_avg, uint64_t* scan_count,
              double* merge_ms_avg, uint64_t* merge_count, int reset);

#ifdef __cplusplus
}
#endif

#endif /* VSEARCH_H_ */
