// batcher.h — dynamic batcher for concurrent /search requests (SURVEY.md §8
// (b) "Threading" and (f) rank 2).
//
// rag/vector-service answers every /search with one Points.Search call for
// one query (rag/vector-service/main.go:249-254); net/http runs the handlers
// concurrently (main.go:77). Here concurrent handlers hand their query to the
// service's worker thread(s) (Options::workers), which coalesce whatever is
// queued into a few vs_search(nq > 1) calls: a batch of bf16 queries then takes the MFMA path
// (one pass over the corpus for up to 256 queries) instead of nq GEMV passes.
//
// Exactness: requests of one collection are searched together with
// k_max = the largest k among them, and each request keeps the first k of its
// k_max results. The engine orders results by (score desc, row asc), a total
// order, so that prefix is exactly the top k. Requests with k above the
// engine's batched-MFMA limit (128) are grouped separately, so a single large
// k never moves the small-k requests off the MFMA path.
//
// Batching policy: no timer by default. Each turn the worker makes one engine
// call for the group (collection, dim, k class) of the oldest queued request,
// taking all of that group's queued requests (up to max_batch). While it runs,
// new requests queue up, so the batch size follows the offered load (1 when
// idle, up to max_batch under load), a lone request waits for nothing, and
// with several collections each call finds its collection's whole backlog.
// max_wait_us > 0 adds a linger before a non-full batch.
//
// Two calls in flight (Options::workers = 2, lead_us): the engine waits for
// the device outside its lock, so a second worker's call runs on the device
// right behind the first; that worker forms its batch only lead_us before
// the first call is expected to end (each collection's recent service
// time), so the batches stay as large as with one worker. A request meeting
// an idle batcher (nothing queued or in flight) runs on its own thread
// (caller_runs): no hand-off to a worker and back.
//
// Devices (lanes): an engine that places collections on different devices
// (VS_FLAG_PLACE_COLLECTIONS) runs their calls concurrently. Every request's
// lane is its collection's device (vs_collection_placement; -1 for a striped
// collection, which uses every device). The in-flight bookkeeping, the
// lead_us timing and caller_runs are per lane, and a worker takes the oldest
// request of the least busy lane, so a call on one device never waits for
// the calls of another.
//
// Filtered requests ("filter":"match") carry the id of their device-resident
// filter (vs_filter_create) and are grouped by it too: requests sharing a
// filter become one vs_search_filter_id call (the MFMA pass with the bitmap
// fused for dense filters, per-query gathers for selective ones).
#pragma once
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/vsearch.h"

namespace vsbatch {

struct Options {
  bool enabled = true;
  uint32_t max_batch = 256;  // queries per engine call
  uint32_t max_wait_us = 0;  // linger for a non-full batch (0 = none)
  // worker threads taking turns: with 2, the next call's batch assembly,
  // query copy and launch wait on the engine while the current call runs,
  // instead of following its return (and its results' hand-out); the engine
  // waits for the device outside its lock, so the two calls run back to back
  uint32_t workers = 2;
  // with a call in flight, a second worker forms its batch only lead_us
  // before that call is expected to end (its collection's recent call time),
  // not at once: requests arriving meanwhile still join, so pipelining the
  // calls does not shrink the batches (0 = form at once)
  uint32_t lead_us = 300;
  // a request that finds nothing queued and nothing in flight runs on the
  // calling thread instead of being handed to a worker (not with a linger:
  // max_wait_us asks for batches to be waited for)
  bool caller_runs = true;
};

struct Stats {
  uint64_t requests = 0;      // searches served through the batcher
  uint64_t engine_calls = 0;  // vs_search calls they took
  uint64_t max_batch = 0;     // largest nq of one call
  uint64_t hist[10] = {};     // calls by nq: 1, 2-3, 4-7, ..., 256+
};

class Batcher {
 public:
  Batcher(vs_engine* eng, Options opt);
  ~Batcher();  // drains the queue, then joins the workers
  Batcher(const Batcher&) = delete;
  Batcher& operator=(const Batcher&) = delete;

  // Blocks until the request's batch ran. Same contract as vs_search for one
  // query of `dim` floats: scores / rows hold k entries, *count the valid ones.
  // On failure returns the engine's status with its message in *err.
  // `filter_id` != 0: vs_search_filter_id semantics with that filter.
  int search(const std::string& coll, const float* q, uint32_t dim, uint32_t k, float* scores,
             uint64_t* rows, uint32_t* count, std::string* err, uint64_t filter_id = 0);

  Stats stats();
  const Options& options() const { return opt_; }

 private:
  struct Req;
  void run();
  void execute(std::vector<Req*>& batch);
  int64_t begin_call(const std::string& coll, int lane, int64_t t0);
  void end_call(const std::string& coll, int lane, int64_t t0, int64_t end);

  // (mu_ held) the lane of a collection, and the queued request to serve next
  int lane_of(const std::string& coll);
  std::deque<Req*>::iterator pick();

  vs_engine* eng_;
  Options opt_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Req*> queue_;
  bool stop_ = false;
  // per lane (device): calls in flight, expected end (steady clock, us) of
  // each and of the last one; end of the last call that completed
  struct Lane {
    std::vector<int64_t> inflight_end;
    int64_t free_at = 0, last_done = 0;
  };
  std::map<int, Lane> lanes_;
  // recent service time per collection (exponential average, us)
  std::map<std::string, double> call_us_;
  Stats stats_;
  std::vector<std::thread> workers_;
};

}  // namespace vsbatch
