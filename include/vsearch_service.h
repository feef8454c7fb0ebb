/*
 * vsearch_service.h — host-side mirror of rag/vector-service's HTTP handlers
 * over the engine C-ABI (include/vsearch.h).
 *
 * The reference service is Go (rag/vector-service/main.go); no Go toolchain
 * exists in this build image, so the handler logic is restated in C++ with
 * the same routes, JSON shapes, status codes and error texts:
 *
 *   GET  /health       healthHandler       main.go:121-136
 *   GET  /collections  collectionsHandler  main.go:138-147
 *   POST /upsert       upsertHandler       main.go:149-225
 *   POST /search       searchHandler       main.go:227-278
 *
 * served in-process by vsvc_handle, or over TCP by vsvc_http_start (the
 * reference's http.ListenAndServe, main.go:75-77).
 *
 * Point UUIDs and payloads live here (a UUID -> row map and a row-indexed
 * payload store per collection); the engine sees dense rows only. A Go
 * deployment binds the same engine C-ABI through cgo and
 * keeps this logic in Go; this library is the drop-in for hosts without Go
 * and the executable specification the parity tests run against.
 */
#ifndef VSEARCH_SERVICE_H_
#define VSEARCH_SERVICE_H_

#include <stddef.h>
#include <stdint.h>

#include "vsearch.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vsvc vsvc;

/* Creates the service over `eng` (not owned). `config_json` may be NULL for
 * the reference defaults (initializeCollections, main.go:80-119: collections
 * regulatory_docs, merchant_docs, kyc_docs, dim 768, Cosine, fp32) or
 * {"collections":[{"name":"..","dim":768,"metric":"Cosine"|"Dot",
 *  "dtype":"f32"|"bf16"}...],
 *  "batching":{"enabled":true,"max_batch":256,"max_wait_us":0,"workers":2,
 *              "lead_us":300,"caller_runs":true},
 *  "filter":"ignore"|"match"}.
 * "filter":"ignore" (default) keeps the reference's behaviour: the request's
 * `filter` is decoded and dropped (main.go:30 vs :249-254). "match" applies
 * it as a pre-mask (a point is eligible when its payload holds every filter
 * key with an equal JSON value); each distinct filter is cached as a
 * device-resident filter (vs_filter_create) until the next upsert, and
 * searched with vs_search_filter_id. Existing collections are reused.
 * Batching (on by default) coalesces concurrent /search requests into one
 * engine call per collection (and per filter, for filtered requests)
 * (csrc/service/batcher.h); each request still gets exactly its own top k.
 * With 2 workers two calls are in flight (the second enqueued while the
 * first runs, its batch formed lead_us before the first is expected to end);
 * a request meeting an idle batcher runs on its own thread (caller_runs). */
int vsvc_open(vs_engine* eng, const char* config_json, vsvc** out);
void vsvc_close(vsvc* svc);

/* Bulk load for benchmarks and large corpora: appends n
 * synthetic unit rows generated on the device (vs_generate, `seed`) to an
 * EMPTY collection, with synthetic version-4 UUIDs (a per-collection tag and
 * the row number, invertible, so no per-row host state is kept) and empty
 * payloads. /search returns those ids; /upsert with one of them overwrites
 * that row; new ids append after the bulk rows. VS_ERR_EXISTS if the
 * collection already holds points. */
int vsvc_bulk_generate(vsvc* svc, const char* coll, uint64_t n, uint64_t seed);
/* Snapshot / restore of the whole service: for every
 * collection, <dir>/<name>.vsnap (vs_snapshot: the rows) and
 * <dir>/<name>.points.json (UUIDs, payloads, bulk range). vsvc_restore loads
 * every collection that has both files into a service whose collections are
 * still empty (VS_ERR_EXISTS otherwise); a corrupt file leaves that
 * collection empty and returns VS_ERR_IO. `dir` must exist. */
int vsvc_snapshot(vsvc* svc, const char* dir);
int vsvc_restore(vsvc* svc, const char* dir);
/* The point id (canonical UUID, 36 chars + NUL) of `row` of `coll`. */
int vsvc_point_id(vsvc* svc, const char* coll, uint64_t row, char* buf, size_t len);

/* Batcher counters as JSON (*out malloc'd; free with vsvc_free):
 * {"batching":{...},"requests":n,"engine_calls":n,"largest_call":n,
 *  "calls_by_log2_nq":[nq=1, 2-3, 4-7, ..., 256-511, 512+]}. */
int vsvc_stats(vsvc* svc, char** out);

/* Closed-loop load generator: `clients` threads each send
 * /search bodies shaped like rag/retrieval-service's searchVectorDB
 * (main.go:221-226: {"collection","filter","query","top_k"}) back to back,
 * for `seconds`: through vsvc_handle in-process, or, with "http":"host:port",
 * as HTTP/1.1 POSTs over TCP to a listener (vsvc_http_start or any server
 * with the reference's routes; `svc` may then be NULL), each client on its
 * own keep-alive connection ("keepalive":false opens one per request).
 * spec_json: {"collections":["..",..],"dim":768,"clients":64,"seconds":5,
 * "k_min":3,"k_max":50,"queries":256,"seed":1,"http":"127.0.0.1:8082",
 * "keepalive":true}. *report (malloc'd) gets
 * {"requests","errors","seconds","qps","lat_ms":{"p50","p90","p99","max"},
 *  "first_error","transport":"inproc"|"http"}. Returns VS_OK or
 * VS_ERR_INVALID_ARG for a bad spec. */
int vsvc_loadgen(vsvc* svc, const char* spec_json, char** report);

/* The reference's http.ListenAndServe(":"+PORT, mux) (main.go:70-77): an
 * HTTP/1.1 listener on `addr` ("host:port", ":port" for every IPv4
 * address; port 0 picks a free one, see vsvc_http_port) that hands every
 * request to vsvc_handle and answers as net/http does: keep-alive and
 * pipelining, Content-Length or chunked request bodies, Expect:
 * 100-continue, HEAD, routing on the URL path without its query, 400 for a
 * malformed request or a missing Host header, 431 past 1 MiB of headers,
 * 501 for a transfer coding other than chunked, 505 for HTTP/2+ request
 * lines. One thread per connection (net/http: one goroutine); concurrent
 * /search requests meet in the batcher. Returns VS_OK, VS_ERR_INVALID_ARG
 * (bad address) or VS_ERR_IO (socket / bind / listen failed). */
typedef struct vsvc_http vsvc_http;
int vsvc_http_start(vsvc* svc, const char* addr, vsvc_http** out);
/* The bound TCP port. */
int vsvc_http_port(const vsvc_http* h);
/* Stops accepting, closes every connection after its in-flight request and
 * joins the threads. Call before vsvc_close. */
void vsvc_http_stop(vsvc_http* h);

/* Serves one HTTP request. Sets *status, *body (malloc'd, NUL-terminated;
 * free with vsvc_free) and *content_type (static string). Safe to call from
 * many threads at once. Returns VS_OK, or a negative vs_status if the
 * arguments are unusable. */
int vsvc_handle(vsvc* svc, const char* method, const char* path, const char* body,
                size_t body_len, int* status, char** resp, size_t* resp_len,
                const char** content_type);
void vsvc_free(char* p);

/* Pure helpers exposed for tests (no engine needed). */
/* Re-encodes a JSON document the way Go's json.Encoder writes a decoded
 * interface{} (sorted keys, shortest floats, HTML escaping, trailing '\n').
 * Returns 0, or -1 with *out = the syntax error text. */
int vsvc_reencode(const char* json, size_t len, char** out);
/* Validates a /search or /upsert body exactly as the handler's decode step
 * does, without touching the engine. Returns the HTTP status the handler
 * would answer for a malformed body (400) or 0 when the body decodes;
 * *msg (malloc'd) gets the error text or "". */
int vsvc_validate(const char* path, const char* body, size_t len, char** msg);

#ifdef __cplusplus
}
#endif

#endif /* VSEARCH_SERVICE_H_ */
