// batcher.cpp — see batcher.h.
#include "batcher.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>
#include <tuple>

namespace vsbatch {

namespace {
// The engine's batched MFMA path serves k <= 128 (vs_kernels.h kMfmaMaxK);
// larger k run the per-query GEMV path whatever the batch.
constexpr uint32_t kMfmaMaxK = 128;
}  // namespace

struct Batcher::Req {
  const std::string* coll;
  const float* q;
  uint32_t dim, k;
  uint64_t filter_id;
  float* scores;
  uint64_t* rows;
  uint32_t* count;
  int rc = VS_OK;
  std::string err;
  bool done = false;  // (under *mu)
  int lane = -1;  // the collection's device (vs_collection_placement)
  // the waiter's own mutex and condition (r05: a finished call wakes its
  // requests through these, not through mu_, so the ~75 handler threads of
  // a C5 batch do not queue on the batcher's lock to return)
  std::mutex* mu = nullptr;
  std::condition_variable* cv = nullptr;
};

Batcher::Batcher(vs_engine* eng, Options opt) : eng_(eng), opt_(opt) {
  if (opt_.max_batch == 0) opt_.max_batch = 1;
  if (opt_.workers == 0) opt_.workers = 1;
  for (uint32_t i = 0; i < opt_.workers; ++i) workers_.emplace_back([this] { run(); });
}

Batcher::~Batcher() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
}

namespace {
int64_t now_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
std::chrono::steady_clock::time_point deadline_in(int64_t us) {
  return std::chrono::steady_clock::now() + std::chrono::microseconds(us);
}
}  // namespace

int Batcher::search(const std::string& coll, const float* q, uint32_t dim, uint32_t k,
                    float* scores, uint64_t* rows, uint32_t* count, std::string* err,
                    uint64_t filter_id) {
  std::mutex done_mu;
  std::condition_variable done_cv;
  Req r{&coll, q, dim, k, filter_id, scores, rows, count};
  r.mu = &done_mu;
  r.cv = &done_cv;
  std::unique_lock<std::mutex> lk(mu_);
  if (stop_) {
    if (err) *err = "service is closing";
    return VS_ERR_INVALID_ARG;
  }
  r.lane = lane_of(coll);
  bool lane_queued = false;
  for (const Req* x : queue_) lane_queued = lane_queued || x->lane == r.lane;
  if (opt_.caller_runs && !opt_.max_wait_us && !lane_queued &&
      lanes_[r.lane].inflight_end.empty()) {
    // Nothing queued and nothing in flight on this request's device: run it
    // on the calling thread (no hand-off to a worker and back: two thread
    // wake-ups less on an idle service). Requests arriving meanwhile queue as
    // usual and the workers treat this call as one in flight.
    std::vector<Req*> batch{&r};
    const int64_t t0 = now_us(), end = begin_call(coll, r.lane, t0);
    lk.unlock();
    execute(batch);
    lk.lock();
    end_call(coll, r.lane, t0, end);
    cv_.notify_all();
  } else {
    queue_.push_back(&r);
    cv_.notify_all();
    lk.unlock();
    std::unique_lock<std::mutex> dl(done_mu);
    done_cv.wait(dl, [&] { return r.done; });  // rc / err / results written before done
  }
  if (r.rc != VS_OK && err) *err = r.err;
  return r.rc;
}

int Batcher::lane_of(const std::string& coll) {
  int32_t dev = -1;
  if (vs_collection_placement(eng_, coll.c_str(), &dev) != VS_OK) dev = -1;
  return dev;
}

// The oldest queued request of a lane with the fewest calls in flight: an
// idle device is served first, and within a lane requests keep their order.
std::deque<Batcher::Req*>::iterator Batcher::pick() {
  auto best = queue_.end();
  size_t best_n = SIZE_MAX;
  for (auto it = queue_.begin(); it != queue_.end(); ++it) {
    const size_t n = lanes_[(*it)->lane].inflight_end.size();
    if (n < best_n) {
      best = it;
      best_n = n;
      if (n == 0) break;
    }
  }
  return best;
}

// (mu_ held) registers a call of `coll` on `lane` starting at t0: a device
// runs the calls in flight on it one after another, so it starts when the
// ones ahead of it are expected to end, and takes its collection's recent
// service time. Returns its expected end.
int64_t Batcher::begin_call(const std::string& coll, int lane, int64_t t0) {
  auto est = call_us_.find(coll);
  Lane& L = lanes_[lane];
  L.free_at = std::max(L.free_at, t0) + (int64_t)(est == call_us_.end() ? 0.0 : est->second);
  L.inflight_end.push_back(L.free_at);
  return L.free_at;
}

// (mu_ held) the call registered as (t0, end) returned: its service time
// (from its start, or from the previous call's end on its device when it
// queued behind one) updates the collection's average.
void Batcher::end_call(const std::string& coll, int lane, int64_t t0, int64_t end) {
  Lane& L = lanes_[lane];
  const int64_t t1 = now_us();
  const double took = (double)(t1 - std::max(t0, L.last_done));
  L.last_done = t1;
  double& avg = call_us_[coll];
  avg = avg == 0.0 ? took : 0.8 * avg + 0.2 * took;
  L.inflight_end.erase(std::find(L.inflight_end.begin(), L.inflight_end.end(), end));
  if (L.inflight_end.empty()) L.free_at = 0;
}

Stats Batcher::stats() {
  std::lock_guard<std::mutex> g(mu_);
  return stats_;
}


void Batcher::run() {
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    cv_.wait(lk, [&] { return stop_ || !queue_.empty(); });
    if (queue_.empty()) break;  // stop_ and drained
    if (opt_.max_wait_us && queue_.size() < opt_.max_batch && !stop_) {
      cv_.wait_until(lk, deadline_in(opt_.max_wait_us),
                     [&] { return stop_ || queue_.size() >= opt_.max_batch; });
      // another worker may have taken the whole queue while this one lingered
      if (queue_.empty()) continue;
    }
    // Another call in flight on the chosen request's device: form this batch
    // late, lead_us before the earliest of them is expected to end (or at
    // once when it ends earlier), so requests arriving in the meantime still
    // join it.
    {
      const int lane = (*pick())->lane;
      const std::vector<int64_t>& fl = lanes_[lane].inflight_end;
      if (opt_.lead_us && !fl.empty() && !stop_) {
        const int64_t wake = *std::min_element(fl.begin(), fl.end()) - (int64_t)opt_.lead_us;
        const size_t n0 = fl.size();
        const int64_t t = now_us();
        if (wake > t)
          cv_.wait_until(lk, deadline_in(wake - t), [&] {
            return stop_ || lanes_[lane].inflight_end.size() < n0 ||
                   queue_.size() >= opt_.max_batch;
          });
        if (queue_.empty()) continue;  // another worker took it
      }
    }
    // One engine call per turn, for the group (collection, dim, k class) of
    // the chosen request: all of that group's queued requests, up to
    // max_batch, go together; other groups keep queueing meanwhile, so the
    // next call of each collection finds its whole backlog (a group never
    // waits behind more than one call of every other group: no starvation).
    const Req* first = *pick();
    std::vector<Req*> batch;
    for (auto it = queue_.begin(); it != queue_.end() && batch.size() < opt_.max_batch;) {
      Req* r = *it;
      if (*r->coll == *first->coll && r->dim == first->dim && r->filter_id == first->filter_id &&
          (r->k > kMfmaMaxK) == (first->k > kMfmaMaxK)) {
        batch.push_back(r);
        it = queue_.erase(it);
      } else {
        ++it;
      }
    }
    const std::string coll = *batch.front()->coll;
    const int lane = batch.front()->lane;
    const int64_t t0 = now_us(), end = begin_call(coll, lane, t0);
    lk.unlock();
    execute(batch);
    lk.lock();
    end_call(coll, lane, t0, end);
    lk.unlock();
    // (a request's waiter may return -- and its Req go out of scope -- as
    // soon as its mutex is released: nothing here touches r after that)
    for (Req* r : batch) {
      std::lock_guard<std::mutex> g(*r->mu);
      r->done = true;
      r->cv->notify_one();
    }
    lk.lock();
    cv_.notify_all();  // a worker waiting to form its batch late
  }
}

void Batcher::execute(std::vector<Req*>& batch) {
  // group: collection, dim, filter, k class (MFMA-eligible or not); arrival
  // order kept
  std::map<std::tuple<std::string, uint32_t, uint64_t, bool>, std::vector<Req*>> groups;
  for (Req* r : batch) groups[{*r->coll, r->dim, r->filter_id, r->k > kMfmaMaxK}].push_back(r);
  std::vector<float> q, sc;
  std::vector<uint64_t> rw;
  std::vector<uint32_t> cn;
  for (auto& kv : groups) {
    const std::string& coll = std::get<0>(kv.first);
    const uint32_t dim = std::get<1>(kv.first);
    const uint64_t fid = std::get<2>(kv.first);
    auto& reqs = kv.second;
    for (size_t b0 = 0; b0 < reqs.size(); b0 += opt_.max_batch) {
      const size_t nq = std::min<size_t>(opt_.max_batch, reqs.size() - b0);
      uint32_t kmax = 1;
      for (size_t i = 0; i < nq; ++i) kmax = std::max(kmax, reqs[b0 + i]->k);
      q.resize(nq * dim);
      for (size_t i = 0; i < nq; ++i)
        std::memcpy(q.data() + i * dim, reqs[b0 + i]->q, (size_t)dim * 4);
      sc.resize(nq * kmax);
      rw.resize(nq * kmax);
      cn.resize(nq);
      const int rc =
          fid ? vs_search_filter_id(eng_, coll.c_str(), q.data(), (uint32_t)nq, dim, kmax, fid,
                                    sc.data(), rw.data(), cn.data())
              : vs_search(eng_, coll.c_str(), q.data(), (uint32_t)nq, dim, kmax, sc.data(),
                          rw.data(), cn.data());
      const std::string err = rc == VS_OK ? std::string() : std::string(vs_last_error());
      for (size_t i = 0; i < nq; ++i) {
        Req* r = reqs[b0 + i];
        r->rc = rc;
        if (rc != VS_OK) {
          r->err = err;
          continue;
        }
        const uint32_t c = std::min(cn[i], r->k);  // top k = the first k of top kmax
        std::memcpy(r->scores, sc.data() + i * kmax, (size_t)c * 4);
        std::memcpy(r->rows, rw.data() + i * kmax, (size_t)c * 8);
        *r->count = c;
      }
      std::lock_guard<std::mutex> g(mu_);
      stats_.requests += nq;
      stats_.engine_calls += 1;
      stats_.max_batch = std::max<uint64_t>(stats_.max_batch, nq);
      int h = 0;
      while (h < 9 && (size_t(2) << h) <= nq) ++h;
      stats_.hist[h] += 1;
    }
  }
}

}  // namespace vsbatch
