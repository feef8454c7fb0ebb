// Package vsearch binds the MI355X exact top-k search engine (include/vsearch.h)
// for rag/vector-service. It replaces the github.com/qdrant/go-client stubs
// the reference dials (rag/vector-service/main.go:14, :44-51, :56-65): the
// five engine calls of the reference map to Info, Create, Health, Upsert and
// Search. The engine deals in dense row numbers; UUIDs and payloads stay in
// the caller (see ../vector-service).
//
// Memory rules: Go slices are passed to C directly. The library copies every
// input before it returns and never keeps a pointer, which is what cgo's
// pointer-passing rules require. Every function is safe for concurrent use.
package vsearch

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../gorilla-rag---agentic-rag-with-mcp-using-golang-microservices_amd/lib -lvsearch -Wl,-rpath,${SRCDIR}/../../gorilla-rag---agentic-rag-with-mcp-using-golang-microservices_amd/lib
#include <stdlib.h>
#include "vsearch.h"

// vs_last_error() is thread-local, and a goroutine may resume on another OS
// thread between two cgo calls. So every entry point is called through a
// wrapper that, on failure, copies the message into the caller's buffer
// inside the SAME C call (vs_copy_last_error); Go never makes a second call
// to fetch it.
typedef struct { char msg[512]; } vsg_err;
static int vsg_fin(int rc, vsg_err* e) {
	if (rc != 0) vs_copy_last_error(e->msg, sizeof e->msg);
	return rc;
}
static int vsg_open(const vs_config* c, vs_engine** h, vsg_err* e) { return vsg_fin(vs_open(c, h), e); }
static int vsg_open_multi(const vs_config_multi* c, vs_engine** h, vsg_err* e) {
	return vsg_fin(vs_open_multi(c, h), e);
}
static int vsg_engine_layout(vs_engine* h, uint32_t* s, uint32_t* d, vsg_err* e) {
	return vsg_fin(vs_engine_layout(h, s, d), e);
}
static int vsg_collection_placement(vs_engine* h, const char* n, int32_t* d, vsg_err* e) {
	return vsg_fin(vs_collection_placement(h, n, d), e);
}
static int vsg_collection_prefilter_bytes(vs_engine* h, const char* n, uint64_t* b, vsg_err* e) {
	return vsg_fin(vs_collection_prefilter_bytes(h, n, b), e);
}
static int vsg_collection_spec_stats(vs_engine* h, const char* n, uint64_t* o, vsg_err* e) {
	return vsg_fin(vs_collection_spec_stats(h, n, o), e);
}
static int vsg_collection_info(vs_engine* h, const char* n, uint32_t* d, uint64_t* r, vsg_err* e) {
	return vsg_fin(vs_collection_info(h, n, d, r, NULL, NULL), e);
}
static int vsg_collection_create(vs_engine* h, const char* n, uint32_t d, int m, int t, uint64_t cap,
                                 vsg_err* e) {
	return vsg_fin(vs_collection_create(h, n, d, m, t, cap, 0), e);
}
static int vsg_collection_drop(vs_engine* h, const char* n, vsg_err* e) {
	return vsg_fin(vs_collection_drop(h, n), e);
}
static int vsg_upsert(vs_engine* h, const char* n, uint64_t cnt, uint32_t d, const uint64_t* r,
                      const float* v, vsg_err* e) {
	return vsg_fin(vs_upsert(h, n, cnt, d, r, v), e);
}
static int vsg_generate(vs_engine* h, const char* n, uint64_t cnt, uint64_t seed, vsg_err* e) {
	return vsg_fin(vs_generate(h, n, cnt, seed), e);
}
static int vsg_search(vs_engine* h, const char* n, const float* q, uint32_t nq, uint32_t d, uint32_t k,
                      float* s, uint64_t* r, uint32_t* c, vsg_err* e) {
	return vsg_fin(vs_search(h, n, q, nq, d, k, s, r, c), e);
}
static int vsg_search_filtered(vs_engine* h, const char* n, const float* q, uint32_t nq, uint32_t d,
                               uint32_t k, const uint64_t* a, uint64_t aw, float* s, uint64_t* r,
                               uint32_t* c, vsg_err* e) {
	return vsg_fin(vs_search_filtered(h, n, q, nq, d, k, a, aw, s, r, c), e);
}
static int vsg_search_filter_id(vs_engine* h, const char* n, const float* q, uint32_t nq, uint32_t d,
                                uint32_t k, uint64_t fid, float* s, uint64_t* r, uint32_t* c,
                                vsg_err* e) {
	return vsg_fin(vs_search_filter_id(h, n, q, nq, d, k, fid, s, r, c), e);
}
static int vsg_filter_create(vs_engine* h, const char* n, const uint64_t* a, uint64_t aw,
                             uint64_t* id, vsg_err* e) {
	return vsg_fin(vs_filter_create(h, n, a, aw, id), e);
}
static int vsg_filter_drop(vs_engine* h, uint64_t id, vsg_err* e) {
	return vsg_fin(vs_filter_drop(h, id), e);
}
static int vsg_snapshot(vs_engine* h, const char* n, const char* p, vsg_err* e) {
	return vsg_fin(vs_snapshot(h, n, p), e);
}
static int vsg_restore(vs_engine* h, const char* n, const char* p, vsg_err* e) {
	return vsg_fin(vs_restore(h, n, p), e);
}
static int vsg_health(vs_engine* h, char* b, size_t len, vsg_err* e) {
	return vsg_fin(vs_health(h, b, len), e);
}
static int vsg_comm_unique_id(unsigned char* id, vsg_err* e) {
	return vsg_fin(vs_comm_unique_id(id), e);
}
static int vsg_comm_init(vs_engine* h, uint32_t n, uint32_t r, const unsigned char* id, vsg_err* e) {
	return vsg_fin(vs_comm_init(h, n, r, id), e);
}
static int vsg_gather_merge_keys(vs_engine* h, const uint64_t* l, uint32_t nq, uint32_t ki,
                                 uint32_t k, uint64_t* o, void* st, vsg_err* e) {
	return vsg_fin(vs_gather_merge_keys(h, l, nq, ki, k, o, st), e);
}
static int vsg_runtime_check(vsg_err* e) { return vsg_fin(vs_runtime_check(), e); }
*/
import "C"

import (
	"errors"
	"fmt"
	"unsafe"
)

// Metric and dtype of a collection (qdrant.Distance_Cosine is main.go:108).
const (
	MetricCosine = int(C.VS_METRIC_COSINE)
	MetricDot    = int(C.VS_METRIC_DOT)
	DtypeF32     = int(C.VS_DTYPE_F32)
	DtypeBF16    = int(C.VS_DTYPE_BF16)
)

// Status codes of the C-ABI.
var (
	ErrInvalidArg  = errors.New("invalid argument")
	ErrNotFound    = errors.New("not found")
	ErrDimMismatch = errors.New("dimension mismatch")
	ErrOOM         = errors.New("out of memory")
	ErrDevice      = errors.New("device error")
	ErrExists      = errors.New("already exists")
	ErrInternal    = errors.New("internal error")
	ErrIO          = errors.New("i/o error")
)

// Error carries the status and the library's message (copied by vs_copy_last_error
// inside the failing call's own wrapper).
type Error struct {
	Code int
	Msg  string
}

func (e *Error) Error() string { return e.Msg }

// Unwrap lets errors.Is(err, vsearch.ErrNotFound) replace the reference's
// status.Code(err) == codes.NotFound test (main.go:96).
func (e *Error) Unwrap() error {
	switch e.Code {
	case int(C.VS_ERR_INVALID_ARG):
		return ErrInvalidArg
	case int(C.VS_ERR_NOT_FOUND):
		return ErrNotFound
	case int(C.VS_ERR_DIM_MISMATCH):
		return ErrDimMismatch
	case int(C.VS_ERR_OOM):
		return ErrOOM
	case int(C.VS_ERR_DEVICE):
		return ErrDevice
	case int(C.VS_ERR_EXISTS):
		return ErrExists
	case int(C.VS_ERR_IO):
		return ErrIO
	}
	return ErrInternal
}

// check turns a wrapper's status into an error. The message was copied into
// e by the same C call that failed (see the vsg_* wrappers above).
func check(rc C.int, e *C.vsg_err) error {
	if rc == 0 {
		return nil
	}
	return &Error{Code: int(rc), Msg: C.GoString(&e.msg[0])}
}

// Engine is one engine handle: one GPU (Open) or row shards over several
// (OpenShards).
type Engine struct{ h *C.vs_engine }

// Open binds the engine to one HIP device (-1: the current one). It replaces
// grpc.DialContext + the New*Client calls (main.go:56-65).
func Open(device int) (*Engine, error) {
	cfg := C.vs_config{device: C.int32_t(device)}
	var h *C.vs_engine
	var e C.vsg_err
	if err := check(C.vsg_open(&cfg, &h, &e), &e); err != nil {
		return nil, err
	}
	return &Engine{h}, nil
}

// OpenPlaced opens one engine over several devices that places every
// collection whole on one of them (VS_FLAG_PLACE_COLLECTIONS): calls for
// collections on different devices run concurrently, with no collective.
func OpenPlaced(devices []int) (*Engine, error) {
	return openMulti(devices, C.VS_FLAG_PLACE_COLLECTIONS)
}

// Placement reports the HIP device holding the whole collection, or -1 when
// it is row-striped over several.
func (e *Engine) Placement(name string) (int, error) {
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	var d C.int32_t
	var ce C.vsg_err
	err := check(C.vsg_collection_placement(e.h, cs, &d, &ce), &ce)
	return int(d), err
}

// PrefilterBytes is the HBM held by the collection's int8 prefilter copy
// (0: none). See VS_FLAG_NO_PREFILTER.
func (e *Engine) PrefilterBytes(name string) (uint64, error) {
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	var b C.uint64_t
	var ce C.vsg_err
	err := check(C.vsg_collection_prefilter_bytes(e.h, cs, &b, &ce), &ce)
	return uint64(b), err
}

// SpecStats reports the collection's speculative-bound counters
// (vs_collection_spec_stats): batches tried, of those re-answered on the
// sample path after a failed check (fallbacks), and batches kept on the
// sample path (skipped). Diagnostics; the reference has no counterpart.
func (e *Engine) SpecStats(name string) (tries, fallbacks, skipped uint64, err error) {
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	var o [4]C.uint64_t
	var ce C.vsg_err
	err = check(C.vsg_collection_spec_stats(e.h, cs, &o[0], &ce), &ce)
	return uint64(o[0]), uint64(o[1]), uint64(o[2]), err
}

// OpenShards opens one engine over row shards: shard s on HIP device
// devices[s] (a device may repeat). Collections are then row-striped over
// the shards and each search ends in one RCCL all-gather; every other call
// is unchanged.
func OpenShards(devices []int) (*Engine, error) { return openMulti(devices, 0) }

func openMulti(devices []int, flags C.uint32_t) (*Engine, error) {
	if len(devices) == 0 {
		return nil, fmt.Errorf("vsearch: no devices: %w", ErrInvalidArg)
	}
	devs := (*C.int32_t)(C.malloc(C.size_t(len(devices)) * 4))
	defer C.free(unsafe.Pointer(devs))
	ds := unsafe.Slice(devs, len(devices))
	for i, d := range devices {
		ds[i] = C.int32_t(d)
	}
	cfg := C.vs_config_multi{devices: devs, n_shards: C.uint32_t(len(devices)), flags: flags}
	var h *C.vs_engine
	var e C.vsg_err
	if err := check(C.vsg_open_multi(&cfg, &h, &e), &e); err != nil {
		return nil, err
	}
	return &Engine{h}, nil
}

// Close releases the device memory of every collection.
func (e *Engine) Close() {
	if e.h != nil {
		C.vs_close(e.h)
		e.h = nil
	}
}

// Layout reports the engine's shards and distinct devices.
func (e *Engine) Layout() (shards, devices int, err error) {
	var s, d C.uint32_t
	var ce C.vsg_err
	err = check(C.vsg_engine_layout(e.h, &s, &d, &ce), &ce)
	return int(s), int(d), err
}

// Info mirrors collectionsClient.Get (main.go:91).
func (e *Engine) Info(name string) (dim uint32, rows uint64, err error) {
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	var d C.uint32_t
	var r C.uint64_t
	var ce C.vsg_err
	err = check(C.vsg_collection_info(e.h, cs, &d, &r, &ce), &ce)
	return uint32(d), uint64(r), err
}

// Create mirrors collectionsClient.Create (main.go:102-112).
func (e *Engine) Create(name string, dim uint32, metric, dtype int, capacity uint64) error {
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	var ce C.vsg_err
	return check(C.vsg_collection_create(e.h, cs, C.uint32_t(dim), C.int(metric), C.int(dtype),
		C.uint64_t(capacity), &ce), &ce)
}

// Drop frees a collection.
func (e *Engine) Drop(name string) error {
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	var ce C.vsg_err
	return check(C.vsg_collection_drop(e.h, cs, &ce), &ce)
}

// Upsert writes len(rows) vectors (vecs is len(rows)*dim float32, row-major)
// into rows; rows at or past the row count append (contiguously). It mirrors
// pointsClient.Upsert(wait=true) (main.go:208-213): it returns once the data
// is resident.
func (e *Engine) Upsert(name string, dim uint32, rows []uint64, vecs []float32) error {
	if len(rows) == 0 {
		return nil
	}
	if len(vecs) != len(rows)*int(dim) {
		return fmt.Errorf("vsearch: %d vectors of dim %d need %d floats, got %d: %w",
			len(rows), dim, len(rows)*int(dim), len(vecs), ErrInvalidArg)
	}
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	var ce C.vsg_err
	return check(C.vsg_upsert(e.h, cs, C.uint64_t(len(rows)), C.uint32_t(dim),
		(*C.uint64_t)(unsafe.Pointer(&rows[0])), (*C.float)(unsafe.Pointer(&vecs[0])), &ce), &ce)
}

// Generate appends n synthetic unit rows made on the device (benchmarks).
func (e *Engine) Generate(name string, n, seed uint64) error {
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	var ce C.vsg_err
	return check(C.vsg_generate(e.h, cs, C.uint64_t(n), C.uint64_t(seed), &ce), &ce)
}

// Hits of one query: rows and scores, best first.
type Hits struct {
	Rows   []uint64
	Scores []float32
}

// SearchBatch searches nq = len(queries)/dim queries at once (the batched
// MFMA path from 2 queries on) and returns each query's top k. It mirrors
// pointsClient.Search (main.go:249-254) for many queries in one call.
func (e *Engine) SearchBatch(name string, queries []float32, dim, k uint32) ([]Hits, error) {
	return e.search(name, queries, dim, k, nil, 0)
}

// Search is SearchBatch for one query.
func (e *Engine) Search(name string, query []float32, k uint32) ([]uint64, []float32, error) {
	h, err := e.search(name, query, uint32(len(query)), k, nil, 0)
	if err != nil {
		return nil, nil, err
	}
	return h[0].Rows, h[0].Scores, nil
}

// SearchFiltered restricts a search to the rows whose bit is set in allow
// (bit r of word r/64); the reference parses SearchRequest.Filter
// (main.go:30) but never applies it.
func (e *Engine) SearchFiltered(name string, queries []float32, dim, k uint32,
	allow []uint64) ([]Hits, error) {
	if len(allow) == 0 {
		return nil, fmt.Errorf("vsearch: empty filter bitmap: %w", ErrInvalidArg)
	}
	return e.search(name, queries, dim, k, allow, 0)
}

// FilterCreate uploads a filter bitmap once; SearchFilterID then ships no
// bitmap per call.
func (e *Engine) FilterCreate(name string, allow []uint64) (uint64, error) {
	if len(allow) == 0 {
		return 0, fmt.Errorf("vsearch: empty filter bitmap: %w", ErrInvalidArg)
	}
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	var id C.uint64_t
	var ce C.vsg_err
	err := check(C.vsg_filter_create(e.h, cs, (*C.uint64_t)(unsafe.Pointer(&allow[0])),
		C.uint64_t(len(allow)), &id, &ce), &ce)
	return uint64(id), err
}

// FilterDrop frees a resident filter.
func (e *Engine) FilterDrop(id uint64) error {
	var ce C.vsg_err
	return check(C.vsg_filter_drop(e.h, C.uint64_t(id), &ce), &ce)
}

// SearchFilterID searches with a resident filter (stale after an upsert
// that added rows: rebuild it).
func (e *Engine) SearchFilterID(name string, queries []float32, dim, k uint32,
	id uint64) ([]Hits, error) {
	return e.search(name, queries, dim, k, nil, id)
}

func (e *Engine) search(name string, queries []float32, dim, k uint32, allow []uint64,
	fid uint64) ([]Hits, error) {
	if dim == 0 || len(queries) == 0 || len(queries)%int(dim) != 0 {
		return nil, fmt.Errorf("vsearch: %d floats are not whole queries of dim %d: %w",
			len(queries), dim, ErrInvalidArg)
	}
	if k == 0 {
		return nil, fmt.Errorf("vsearch: k must be at least 1: %w", ErrInvalidArg)
	}
	nq := len(queries) / int(dim)
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	rows := make([]uint64, nq*int(k))
	scores := make([]float32, nq*int(k))
	count := make([]uint32, nq)
	q := (*C.float)(unsafe.Pointer(&queries[0]))
	pr := (*C.uint64_t)(unsafe.Pointer(&rows[0]))
	ps := (*C.float)(unsafe.Pointer(&scores[0]))
	pc := (*C.uint32_t)(unsafe.Pointer(&count[0]))
	var rc C.int
	var ce C.vsg_err
	switch {
	case fid != 0:
		rc = C.vsg_search_filter_id(e.h, cs, q, C.uint32_t(nq), C.uint32_t(dim), C.uint32_t(k),
			C.uint64_t(fid), ps, pr, pc, &ce)
	case allow != nil:
		rc = C.vsg_search_filtered(e.h, cs, q, C.uint32_t(nq), C.uint32_t(dim), C.uint32_t(k),
			(*C.uint64_t)(unsafe.Pointer(&allow[0])), C.uint64_t(len(allow)), ps, pr, pc, &ce)
	default:
		rc = C.vsg_search(e.h, cs, q, C.uint32_t(nq), C.uint32_t(dim), C.uint32_t(k), ps, pr, pc, &ce)
	}
	if err := check(rc, &ce); err != nil {
		return nil, err
	}
	out := make([]Hits, nq)
	for i := range out {
		lo, n := i*int(k), int(count[i])
		out[i] = Hits{Rows: rows[lo : lo+n], Scores: scores[lo : lo+n]}
	}
	return out, nil
}

// Snapshot writes a collection's stored rows to path (replaces Qdrant's
// persistent volume, docker-compose.yml:9-10,14-15); searches proceed meanwhile.
func (e *Engine) Snapshot(name, path string) error {
	cn, cp := C.CString(name), C.CString(path)
	defer C.free(unsafe.Pointer(cn))
	defer C.free(unsafe.Pointer(cp))
	var ce C.vsg_err
	return check(C.vsg_snapshot(e.h, cn, cp, &ce), &ce)
}

// Restore creates a collection from a snapshot (bit-exact, checksum-verified).
func (e *Engine) Restore(name, path string) error {
	cn, cp := C.CString(name), C.CString(path)
	defer C.free(unsafe.Pointer(cn))
	defer C.free(unsafe.Pointer(cp))
	var ce C.vsg_err
	return check(C.vsg_restore(e.h, cn, cp, &ce), &ce)
}

// Health mirrors systemClient.HealthCheck (main.go:126): the engine's JSON
// status object ({"status":"healthy"|"degraded","engine":"vsearch-hip",...}).
func (e *Engine) Health() (string, error) {
	buf := (*C.char)(C.malloc(4096))
	defer C.free(unsafe.Pointer(buf))
	var ce C.vsg_err
	err := check(C.vsg_health(e.h, buf, 4096, &ce), &ce)
	return C.GoString(buf), err
}

// RuntimeCheck reports whether this process maps exactly one HIP runtime
// (vs_runtime_check). A process that also loads another libamdhip64 (e.g. a
// framework's bundled copy) has two sets of streams with no ordering between
// them; the device-pointer calls (GatherMergeKeys, ...) then refuse to run.
func RuntimeCheck() error {
	var ce C.vsg_err
	return check(C.vsg_runtime_check(&ce), &ce)
}

// CommUniqueID makes the RCCL id of a one-process-per-GPU deployment: call it
// on one rank and hand the bytes to every rank (any host transport).
func CommUniqueID() ([]byte, error) {
	id := make([]byte, C.VS_COMM_ID_BYTES)
	var ce C.vsg_err
	err := check(C.vsg_comm_unique_id((*C.uchar)(unsafe.Pointer(&id[0])), &ce), &ce)
	return id, err
}

// CommInit joins this engine (one GPU, one row shard opened with a row_base)
// to the ranks' communicator; every rank calls it with the same id.
func (e *Engine) CommInit(nRanks, rank int, id []byte) error {
	if len(id) != int(C.VS_COMM_ID_BYTES) {
		return fmt.Errorf("vsearch: comm id must be %d bytes: %w", int(C.VS_COMM_ID_BYTES), ErrInvalidArg)
	}
	var ce C.vsg_err
	return check(C.vsg_comm_init(e.h, C.uint32_t(nRanks), C.uint32_t(rank),
		(*C.uchar)(unsafe.Pointer(&id[0])), &ce), &ce)
}

// GatherMergeKeys exchanges every rank's [nq][kIn] device keys (the output of
// vs_search_keys) with one RCCL all-gather and merges them into the global
// [nq][k] keys, both on `stream` (a hipStream_t; nil = the null stream).
// dLocal and dOut are device pointers, which cgo passes as plain addresses.
func (e *Engine) GatherMergeKeys(dLocal, dOut unsafe.Pointer, nq, kIn, k uint32,
	stream unsafe.Pointer) error {
	var ce C.vsg_err
	return check(C.vsg_gather_merge_keys(e.h, (*C.uint64_t)(dLocal), C.uint32_t(nq),
		C.uint32_t(kIn), C.uint32_t(k), (*C.uint64_t)(dOut), stream, &ce), &ce)
}
