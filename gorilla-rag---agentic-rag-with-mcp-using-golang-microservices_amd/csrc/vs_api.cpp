// vs_api.cpp — the C-ABI of include/vsearch.h.
//
// A vs_engine replaces the Qdrant server and the gRPC client globals of
// rag/vector-service/main.go:44-65 (one handle per process). It is built
// from one DevEngine per HIP device it drives (vs_dev.h):
//
//  * vs_open: one device, one shard. Every call goes straight to the device
//    engine; nothing here is on that path.
//  * vs_open_multi: S shards over D distinct devices. Every
//    collection is row-striped: global row g lives on shard g % S at local
//    row g / S, so appends spread evenly over the shards whatever the order
//    in which rows arrive. A search runs every shard's scan (local top-k in
//    local rows), maps the keys to global rows on the device, merges the
//    shards of each device, exchanges one [nq][k] key list per device with
//    ONE RCCL all-gather over xGMI (a communicator from ncclCommInitAll in
//    this process) and merges the D lists on the first device; one D2H of
//    nq x k keys. Messages are P x nq x k x 8 bytes: latency-bound.
//
//  * vs_open_multi with VS_FLAG_PLACE_COLLECTIONS: every collection lives
//    whole on one of the devices (the least loaded at creation), and each
//    call goes straight to that device's engine: calls for collections on
//    different devices run concurrently, with no collective (the reference
//    serves three independent collections from concurrent handlers,
//    rag/vector-service/main.go:77, :80-119).
//
// All kinds answer the same C-ABI, so the C++ service mirror and the cgo
// binding serve a sharded collection unchanged. A host search (vs_search*)
// holds the devices' work locks only while it enqueues: its queries and keys
// go through pinned per-call slots and it waits for the device outside the
// locks, so concurrent calls overlap their host work with the devices'.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/vsearch.h"
#include "vs_common.h"
#include "vs_dev.h"
#include "vs_kernels.h"

using vsd::DevBuf;
using vsd::DevEngine;
using vsd::fail;
using vsd::fail_hip;

namespace {

std::atomic<uint64_t> g_scoll_gen{1};

// A row-striped collection of a multi-shard engine.
struct SColl {
  std::string name;
  uint64_t gen = 0;
  uint32_t dim = 0;
  int metric = VS_METRIC_COSINE, dtype = VS_DTYPE_F32;
  uint64_t rows = 0;      // global rows (striped collections)
  std::shared_mutex mu;   // upsert / generate / restore = writer, search = reader
  std::vector<std::string> iname;  // shard s -> its collection's name on its device
  int home = -1;          // placed engines: index of the device holding the whole collection
  uint64_t reserved = 0;  // placed: bytes counted against its device at creation
  // false while vs_collection_create / vs_restore is still making it on the
  // devices: the name is taken (a second create fails EXISTS) but every
  // other call, vs_collection_drop included, sees "not found", so only the
  // creating call can take it back out (and return its reservation, once)
  std::atomic<bool> ready{false};
};

// A device-resident filter of a multi-shard engine: one per shard.
struct SFilter {
  uint64_t coll_gen = 0, rows = 0;
  std::vector<uint64_t> dev_fid;   // shard s (placed: entry 0) -> filter id on its device engine
  std::vector<uint32_t> dev_idx;   // ... and that device's index
};

int not_found(const char* name) {
  return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (name ? name : "") + " not found");
}

}  // namespace

struct vs_engine {
  std::vector<DevEngine*> dev;                 // distinct devices, first-use order
  std::vector<uint32_t> shard_dev;             // shard -> dev index
  std::vector<std::vector<uint32_t>> dev_shards;  // dev index -> its shards, ascending
  bool sharded = false;                        // vs_open_multi with more than one shard
  std::mutex map_mu;
  std::unordered_map<std::string, std::shared_ptr<SColl>> colls;
  std::mutex filt_mu;
  std::unordered_map<uint64_t, SFilter> filters;
  uint64_t next_filter = 1;
  // per-device scratch of the multi-shard search (guarded by that device
  // context's work_mu)
  struct Scratch {
    DevBuf q, keys, merged, gather, out, allow;
    hipEvent_t qev = nullptr;  // dev 0: the caller's queries are ready
    hipEvent_t kev = nullptr;  // placed: this device's keys reached dev 0
  };
  // One context set: search context j of every device (vs_dev.h DevStore),
  // its scratch, its RCCL communicator (ncclCommInitAll; none when placed)
  // and its pinned staging. Set 0 holds the devices' primary contexts (the
  // device-pointer searches use it); a host search takes an idle set, so
  // concurrent host searches run on separate streams of every device.
  struct CtxSet {
    std::vector<DevEngine*> dev;
    std::vector<Scratch> scr;
    std::vector<ncclComm_t> comm;
    std::vector<std::unique_ptr<vsd::HostSlot>> host_slots;  // guarded by dev[0]'s work_mu
    std::atomic<int> inflight{0};
  };
  std::vector<std::unique_ptr<CtxSet>> sets;
  // Striped engines: every set's all-gather is enqueued under coll_mu and
  // waits, on each device, for the previous one (coll_ev[d], recorded after
  // it), so the collectives of different sets' communicators execute in ONE
  // order on every device. Without it two sets' collectives over the same
  // GPUs could start in opposite orders on two devices, each kernel waiting
  // for a peer that runs the other: RCCL's documented deadlock for
  // concurrent communicators.
  std::mutex coll_mu;
  std::vector<hipEvent_t> coll_ev;  // per device index; armed after the first collective
  bool coll_armed = false;
  // VS_FLAG_PLACE_COLLECTIONS: whole collections per device; bytes reserved
  // and collections per device (the placement balance), guarded by map_mu
  bool placed = false;
  std::vector<uint64_t> dev_bytes;
  std::vector<uint32_t> dev_colls;
  // one process per GPU (vs_comm_init): the ranks' communicator and the
  // all-gather output of vs_gather_merge_keys (guarded by gm_mu, below)
  ncclComm_t pcomm = nullptr;
  uint32_t pranks = 0, prank = 0;
  DevBuf pgather;
  // (r05) the exchange's own stream order: vs_gather_merge_keys touches only
  // pgather (and, for k <= kMaxK, a scratch-free merge), so it orders itself
  // after the previous exchange (gm_ev on gm_stream) instead of joining the
  // primary context's search stream -- an exchange on a side stream then
  // overlaps the next batch's search. Every exchange, the
  // large-k one too, holds gm_mu and follows gm_ev, so no two exchanges
  // share pgather at once whatever streams they run on.
  std::mutex gm_mu;
  hipStream_t gm_stream = nullptr;
  hipEvent_t gm_ev = nullptr;
  uint32_t shards() const { return (uint32_t)shard_dev.size(); }
};

namespace {

std::shared_ptr<SColl> find_scoll(vs_engine* E, const char* name) {
  std::lock_guard<std::mutex> g(E->map_mu);
  auto it = E->colls.find(name ? name : "");
  return it == E->colls.end() || !it->second->ready.load(std::memory_order_acquire) ? nullptr
                                                                                    : it->second;
}

DevEngine* shard_eng(vs_engine* E, uint32_t s) { return E->dev[E->shard_dev[s]]; }

// number of global rows g in [lo, hi) with g % S == s, and the first one
void stripe_range(uint64_t lo, uint64_t hi, uint32_t S, uint32_t s, uint64_t* first,
                  uint64_t* count) {
  const uint64_t g0 = lo + ((uint64_t)s + S - lo % S) % S;
  *first = g0;
  *count = g0 < hi ? (hi - 1 - g0) / S + 1 : 0;
}

// bit g of a global bitmap -> bit g / S of shard s's local bitmap
void deinterleave_bits(const uint64_t* allow, uint64_t rows, uint32_t S, uint32_t s,
                       std::vector<uint64_t>* out) {
  const uint64_t nl = rows > s ? (rows - 1 - s) / S + 1 : 0;
  out->assign((nl + 63) / 64 + 1, 0);
  for (uint64_t l = 0; l < nl; ++l) {
    const uint64_t g = l * S + s;
    if ((allow[g >> 6] >> (g & 63)) & 1) (*out)[l >> 6] |= 1ull << (l & 63);
  }
}

using CtxSet = vs_engine::CtxSet;

// Holds the work lock of every device context of a set, in device order (the
// one lock order of the library: single-device calls take one of them).
struct AllWork {
  std::vector<std::unique_lock<std::mutex>> locks;
  AllWork() = default;
  explicit AllWork(const CtxSet& cs) {
    for (DevEngine* d : cs.dev) locks.emplace_back(d->work_mu);
  }
};

// The context set a host search should use: set 0 for a heavy search
// (vs_engine.cpp heavy_search: batched scans of large shards queue on one
// stream per device), else an idle one whose locks are all free (taken on
// return), else the least busy one (waited for).
CtxSet* pick_set(vs_engine* E, AllWork* aw, bool heavy) {
  if (heavy) {
    *aw = AllWork(*E->sets[0]);
    return E->sets[0].get();
  }
  for (auto& up : E->sets) {
    CtxSet* cs = up.get();
    if (cs->inflight.load(std::memory_order_relaxed) != 0) continue;
    AllWork w;
    bool ok = true;
    for (DevEngine* d : cs->dev) {
      std::unique_lock<std::mutex> g(d->work_mu, std::try_to_lock);
      if (!g.owns_lock()) {
        ok = false;
        break;
      }
      w.locks.push_back(std::move(g));
    }
    if (ok) {
      *aw = std::move(w);
      return cs;
    }
  }
  CtxSet* best = E->sets[0].get();
  for (auto& up : E->sets)
    if (up->inflight.load(std::memory_order_relaxed) < best->inflight.load(std::memory_order_relaxed))
      best = up.get();
  *aw = AllWork(*best);
  return best;
}

int nccl_fail(ncclResult_t r, const char* what) {
  return fail(VS_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(r));
}

// Per-shard filter inputs of one multi-shard search.
struct ShardFilter {
  const uint64_t* bits = nullptr;  // device bitmap (local rows)
  uint64_t allowed = 0;
  const uint32_t* list = nullptr;  // compacted rows (selective resident filters)
};

// The multi-shard search. Queries: host h_q, or device d_q0 on dev 0
// (ordered on the caller's stream cs0 when caller_stream; dev 0's work then
// runs on it). The final [nq][k] keys (global rows) are written
// to d_out on dev 0 (null: the engine's result buffer the set's scr[0].out),
// ordered on dev 0's current stream. The caller holds
// sc.mu (reader) and every device's work lock (AllWork).
// Filters: h_allow (global bitmap, shipped per call; the per-shard host
// bitmaps live in *bits_keep until the caller has synchronised) or fid
// (resident).
int sharded_search(vs_engine* E, CtxSet& cx, SColl& sc, const float* h_q, const float* d_q0,
                   bool caller_stream, hipStream_t cs0, uint32_t nq, uint32_t k,
                   const uint64_t* h_allow, std::vector<std::vector<uint64_t>>* bits_keep,
                   const SFilter* fid, std::vector<std::shared_ptr<vsd::DevFilter>>* fkeep,
                   uint64_t* d_out) {
  const uint32_t S = E->shards(), D = (uint32_t)E->dev.size(), dim = sc.dim;
  const size_t qbytes = (size_t)nq * dim * 4, lbytes = (size_t)nq * k * 8;
  std::vector<std::vector<std::shared_ptr<vsd::Collection>>> held(D);
  std::vector<std::shared_lock<std::shared_mutex>> rlocks;
  if (h_allow) bits_keep->assign(S, {});
  // 1. every shard's scan, device by device (all asynchronous: the devices
  //    scan in parallel)
  for (uint32_t d = 0; d < D; ++d) {
    DevEngine* de = cx.dev[d];
    auto& sc_d = cx.scr[d];
    VS_HIP(vsd::set_dev(de), "hipSetDevice");
    VS_HIP(vsd::use_stream(de, d == 0 && caller_stream ? cs0 : de->own), "stream order");
    const uint32_t m = (uint32_t)E->dev_shards[d].size();
    const size_t abytes = h_allow ? ((sc.rows / S + 2 + 63) / 64 + 1) * 8 * m : 0;
    if (sc_d.keys.bytes < lbytes * m || sc_d.merged.bytes < lbytes || sc_d.q.bytes < qbytes ||
        sc_d.gather.bytes < lbytes * D || sc_d.out.bytes < lbytes || sc_d.allow.bytes < abytes) {
      VS_HIP(hipStreamSynchronize(de->stream), "sync");
      VS_HIP(sc_d.keys.ensure(lbytes * m), "alloc shard keys");
      VS_HIP(sc_d.merged.ensure(lbytes), "alloc merged keys");
      VS_HIP(sc_d.q.ensure(qbytes), "alloc queries");
      VS_HIP(sc_d.gather.ensure(lbytes * D), "alloc gathered keys");
      VS_HIP(sc_d.out.ensure(lbytes), "alloc result keys");
      VS_HIP(sc_d.allow.ensure(abytes), "alloc shard bitmaps");
    }
    const float* q_d = nullptr;
    if (h_q) {
      VS_HIP(hipMemcpyAsync(sc_d.q.p, h_q, qbytes, hipMemcpyHostToDevice, de->stream), "query H2D");
      q_d = sc_d.q.as<float>();
    } else if (d == 0) {
      q_d = d_q0;
    } else {  // peer copy from dev 0, after the caller's stream produced them
      VS_HIP(hipStreamWaitEvent(de->stream, cx.scr[0].qev, 0), "query order");
      VS_HIP(hipMemcpyPeerAsync(sc_d.q.p, de->device, d_q0, cx.dev[0]->device, qbytes,
                                de->stream),
             "query peer copy");
      q_d = sc_d.q.as<float>();
    }
    for (uint32_t j = 0; j < m; ++j) {
      const uint32_t s = E->dev_shards[d][j];
      auto c = vsd::find_coll(de, sc.iname[s].c_str());
      if (!c) return fail(VS_ERR_INTERNAL, "shard " + std::to_string(s) + " of " + sc.name +
                                               " is missing");
      rlocks.emplace_back(c->mu);
      held[d].push_back(c);
      ShardFilter f;
      if (h_allow) {
        std::vector<uint64_t>& bits_tmp = (*bits_keep)[s];
        deinterleave_bits(h_allow, sc.rows, S, s, &bits_tmp);
        const size_t wb = ((sc.rows / S + 2 + 63) / 64 + 1) * 8;
        uint64_t* dst = (uint64_t*)((char*)sc_d.allow.p + wb * j);
        VS_HIP(hipMemcpyAsync(dst, bits_tmp.data(), std::min(wb, bits_tmp.size() * 8),
                              hipMemcpyHostToDevice, de->stream),
               "shard bitmap H2D");
        f.bits = dst;
        f.allowed = vsd::popcount_rows(bits_tmp.data(), c->rows);
      } else if (fid) {
        std::shared_ptr<vsd::DevFilter> dfp = vsd::find_filter(de, fid->dev_fid[s]);
        if (!dfp) return fail(VS_ERR_NOT_FOUND, "filter shard not found");
        const vsd::DevFilter* df = dfp.get();
        fkeep->push_back(std::move(dfp));  // until the device is done with it
        if (df->coll_gen != c->gen || df->rows != c->rows)
          return fail(VS_ERR_INVALID_ARG, "filter was built for another collection state");
        f.bits = df->bits.as<uint64_t>();
        f.allowed = df->allowed;
        f.list = df->list.p ? df->list.as<uint32_t>() : nullptr;
      }
      uint64_t* keys = sc_d.keys.as<uint64_t>() + (size_t)j * nq * k;
      const int rc = vsd::search_core(de, *c, q_d, nq, k, keys, f.bits, f.allowed, f.list);
      if (rc != VS_OK) return rc;
    }
  }
  // 2. local rows -> global rows; the shards of a device merged on it
  std::vector<const uint64_t*> send(D);
  for (uint32_t d = 0; d < D; ++d) {
    DevEngine* de = cx.dev[d];
    auto& sc_d = cx.scr[d];
    VS_HIP(vsd::set_dev(de), "hipSetDevice");
    const uint32_t m = (uint32_t)E->dev_shards[d].size();
    for (uint32_t j = 0; j < m; ++j)
      VS_HIP(vsk::launch_remap_keys(sc_d.keys.as<uint64_t>() + (size_t)j * nq * k,
                                    (uint64_t)nq * k, S, E->dev_shards[d][j], 0, de->stream),
             "remap keys");
    if (m > 1) {
      const int rc = vsd::merge_any(de, sc_d.keys.as<uint64_t>(), m, (uint64_t)nq * k, k, nq, k,
                                    k, sc_d.merged.as<uint64_t>());
      if (rc != VS_OK) return rc;
      send[d] = sc_d.merged.as<uint64_t>();
    } else {
      send[d] = sc_d.keys.as<uint64_t>();
    }
  }
  // 3. one all-gather of the devices' lists over RCCL, merged on dev 0; in
  //    the engine's one collective order (coll_mu / coll_ev)
  {
    std::lock_guard<std::mutex> cg(E->coll_mu);
    if (E->coll_armed)
      for (uint32_t d = 0; d < D; ++d) {
        VS_HIP(vsd::set_dev(cx.dev[d]), "hipSetDevice");
        VS_HIP(hipStreamWaitEvent(cx.dev[d]->stream, E->coll_ev[d], 0), "collective order");
      }
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return nccl_fail(r, "ncclGroupStart");
    for (uint32_t d = 0; d < D; ++d) {
      r = ncclAllGather(send[d], cx.scr[d].gather.p, (size_t)nq * k, ncclUint64, cx.comm[d],
                        cx.dev[d]->stream);
      if (r != ncclSuccess) {
        (void)ncclGroupEnd();
        return nccl_fail(r, "ncclAllGather");
      }
    }
    r = ncclGroupEnd();
    if (r != ncclSuccess) return nccl_fail(r, "ncclGroupEnd");
    for (uint32_t d = 0; d < D; ++d) {
      VS_HIP(vsd::set_dev(cx.dev[d]), "hipSetDevice");
      VS_HIP(hipEventRecord(E->coll_ev[d], cx.dev[d]->stream), "collective order");
    }
    E->coll_armed = true;
  }
  DevEngine* d0 = cx.dev[0];
  VS_HIP(vsd::set_dev(d0), "hipSetDevice");
  return vsd::merge_any(d0, cx.scr[0].gather.as<uint64_t>(), D, (uint64_t)nq * k, k, nq, k, k,
                        d_out ? d_out : cx.scr[0].out.as<uint64_t>());
}

DevEngine* home_eng(vs_engine* E, const SColl& sc) { return E->dev[sc.home]; }

int sharded_search_host(vs_engine* E, const char* coll, const float* queries, uint32_t nq,
                        uint32_t dim, uint32_t k, const uint64_t* allow, uint64_t allow_words,
                        uint64_t filter_id, float* out_scores, uint64_t* out_rows,
                        uint32_t* out_count) {
  if (k == 0) return fail(VS_ERR_INVALID_ARG, "k must be at least 1");
  if (nq == 0) return VS_OK;
  if (!queries) return fail(VS_ERR_INVALID_ARG, "queries is NULL");
  auto sc = find_scoll(E, coll);
  if (!sc) return not_found(coll);
  SFilter f;
  if (filter_id) {
    std::lock_guard<std::mutex> g(E->filt_mu);
    auto it = E->filters.find(filter_id);
    if (it == E->filters.end())
      return fail(VS_ERR_NOT_FOUND, "filter " + std::to_string(filter_id) + " not found");
    f = it->second;
  }
  if (sc->home >= 0) {  // placed: the device engine's own (concurrent) host search
    if (filter_id && f.coll_gen != sc->gen)
      return fail(VS_ERR_INVALID_ARG, "filter " + std::to_string(filter_id) +
                                          " was built for another collection state");
    return vsd::search_host(home_eng(E, *sc), sc->iname[0].c_str(), queries, nq, dim, k, allow,
                            allow_words, out_scores, out_rows, out_count,
                            filter_id ? f.dev_fid[0] : 0);
  }
  if (dim != sc->dim)
    return fail(VS_ERR_DIM_MISMATCH, "Vector dimension error: expected dim: " +
                                         std::to_string(sc->dim) + ", got " + std::to_string(dim));
  std::shared_lock<std::shared_mutex> rl(sc->mu);
  if (allow && allow_words < (sc->rows + 63) / 64)
    return fail(VS_ERR_INVALID_ARG, "filter bitmap has " + std::to_string(allow_words) +
                                        " words, the collection needs " +
                                        std::to_string((sc->rows + 63) / 64));
  if (filter_id && (f.coll_gen != sc->gen || f.rows != sc->rows))
    return fail(VS_ERR_INVALID_ARG, "filter " + std::to_string(filter_id) +
                                        " was built for another collection state");
  // min(k, rows) searched and sized; the outputs keep stride k (vs_engine.cpp search_host)
  const uint32_t ko = k;
  k = (uint32_t)std::min<uint64_t>(k, std::max<uint64_t>(sc->rows, 1));
  const size_t qbytes = (size_t)nq * dim * 4, kbytes = (size_t)nq * k * 8;
  std::vector<std::vector<uint64_t>> bits_keep;  // alive until the wait below
  std::vector<std::shared_ptr<vsd::DevFilter>> fkeep;  // likewise
  // a context set (one search context per device): an idle one if any, so
  // concurrent host searches run on separate streams of every device
  // heavy: a batched search whose shards are large (the per-shard test of
  // vsd::heavy_search on a shard's share of the rows)
  vsd::Collection probe;
  probe.dim = sc->dim;
  probe.dtype = sc->dtype;
  probe.rows = sc->rows / std::max<uint32_t>(1, E->shards());
  AllWork aw;
  CtxSet& cx = *pick_set(E, &aw, vsd::heavy_search(probe, nq));
  cx.inflight.fetch_add(1, std::memory_order_relaxed);
  struct Leave {
    CtxSet& cx;
    ~Leave() { cx.inflight.fetch_sub(1, std::memory_order_relaxed); }
  } leave{cx};
  DevEngine* d0 = cx.dev[0];
  // an idle pinned staging slot: the queries go H2D to every device from it
  // and the keys come back into it, asynchronously (one slot per call in flight)
  vsd::HostSlot* hs = nullptr;
  for (auto& x : cx.host_slots)
    if (!x->busy) {
      hs = x.get();
      break;
    }
  if (!hs) {
    cx.host_slots.push_back(std::make_unique<vsd::HostSlot>());
    hs = cx.host_slots.back().get();
  }
  VS_HIP(vsd::set_dev(d0), "hipSetDevice");
  VS_HIP(hs->ensure(qbytes, kbytes), "alloc pinned staging");
  std::memcpy(hs->in, queries, qbytes);
  hs->busy = true;
  // a failure after the first enqueue drains every device before the slot is
  // released (queued copies may still read or write it)
  auto abandon = [&](int rc) {
    const std::string msg = vsd::last_error();
    for (DevEngine* de : cx.dev) {
      (void)vsd::set_dev(de);
      (void)hipStreamSynchronize(de->stream);
    }
    hs->busy = false;
    return fail(rc, msg);
  };
  int rc = sharded_search(E, cx, *sc, (const float*)hs->in, nullptr, false, nullptr, nq, k, allow,
                          &bits_keep, filter_id ? &f : nullptr, &fkeep, nullptr);
  if (rc != VS_OK) return abandon(rc);
  hipError_t e = vsd::set_dev(d0);
  if (e != hipSuccess) return abandon(vsd::fail_hip(e, "hipSetDevice"));
  e = hipMemcpyAsync(hs->out, cx.scr[0].out.p, kbytes, hipMemcpyDeviceToHost, d0->stream);
  if (e == hipSuccess) e = hipEventRecord(hs->done, d0->stream);
  if (e != hipSuccess) return abandon(vsd::fail_hip(e, "keys D2H"));
  // wait outside the work locks: the next call enqueues behind this one on
  // every device (all scratch is ordered by the devices' streams)
  aw.locks.clear();
  const hipError_t we = vsd::wait_event(hs->done);
  if (we == hipSuccess) vsd::decode_host((const uint64_t*)hs->out, nq, k, out_scores, out_rows, out_count, ko);
  {
    std::lock_guard<std::mutex> g(d0->work_mu);
    hs->busy = false;
  }
  VS_HIP(we, "search sync");
  return VS_OK;
}

// The device-pointer search of a placed collection on device `home` != 0:
// the queries (dev 0, ordered on cs) are copied to the home device, searched
// there on its own stream, and the keys copied back to d_keys on dev 0; cs
// waits for them. Holds the home device's work lock while it enqueues.
int placed_search_keys(vs_engine* E, SColl& sc, const float* d_q, uint32_t nq, uint32_t k,
                       uint64_t* d_keys, hipStream_t cs) {
  CtxSet& cx = *E->sets[0];  // the primary contexts, as every device-pointer search
  DevEngine* d0 = E->dev[0];
  DevEngine* de = home_eng(E, sc);
  auto& sd = cx.scr[sc.home];
  auto c = vsd::find_coll(de, sc.iname[0].c_str());
  if (!c) return not_found(sc.name.c_str());
  std::shared_lock<std::shared_mutex> rl(c->mu);
  const size_t qbytes = (size_t)nq * c->dim * 4, kbytes = (size_t)nq * k * 8;
  std::unique_lock<std::mutex> g0(d0->work_mu, std::defer_lock), gh(de->work_mu, std::defer_lock);
  std::lock(g0, gh);  // dev 0's events + the home device's scratch
  VS_HIP(vsd::set_dev(d0), "hipSetDevice");
  VS_HIP(hipEventRecord(cx.scr[0].qev, cs), "query event");
  VS_HIP(vsd::set_dev(de), "hipSetDevice");
  VS_HIP(vsd::use_stream(de, de->own), "stream order");
  if (sd.q.bytes < qbytes || sd.keys.bytes < kbytes) {
    VS_HIP(hipStreamSynchronize(de->stream), "sync");
    VS_HIP(sd.q.ensure(qbytes), "alloc queries");
    VS_HIP(sd.keys.ensure(kbytes), "alloc keys");
  }
  VS_HIP(hipStreamWaitEvent(de->stream, cx.scr[0].qev, 0), "query order");
  VS_HIP(hipMemcpyPeerAsync(sd.q.p, de->device, d_q, d0->device, qbytes, de->stream), "query peer copy");
  const int rc = vsd::search_core(de, *c, sd.q.as<float>(), nq, k, sd.keys.as<uint64_t>());
  if (rc != VS_OK) return rc;
  VS_HIP(hipMemcpyPeerAsync(d_keys, d0->device, sd.keys.p, de->device, kbytes, de->stream),
         "keys peer copy");
  VS_HIP(hipEventRecord(sd.kev, de->stream), "keys event");
  VS_HIP(vsd::set_dev(d0), "hipSetDevice");
  VS_HIP(hipStreamWaitEvent(cs, sd.kev, 0), "keys order");
  return VS_OK;
}

// stored rows of a sharded collection, global rows [first, first + n), in
// global order, through per-shard reads (fp32 widened, or raw stored bytes)
template <bool RAW>
int sharded_read(vs_engine* E, SColl& sc, uint64_t first, uint64_t n, void* out) {
  const uint32_t S = E->shards();
  const size_t elem = sc.dtype == VS_DTYPE_BF16 ? 2 : 4;
  const size_t ob = RAW ? elem * sc.dim : 4 * (size_t)sc.dim;  // output bytes per row
  std::vector<unsigned char> tmp;
  for (uint32_t s = 0; s < S; ++s) {
    uint64_t g0, cnt;
    stripe_range(first, first + n, S, s, &g0, &cnt);
    if (!cnt) continue;
    tmp.resize(cnt * ob);
    DevEngine* de = shard_eng(E, s);
    const int rc = RAW ? vsd::read_raw(de, sc.iname[s].c_str(), g0 / S, cnt, tmp.data())
                       : vsd::read_rows(de, sc.iname[s].c_str(), g0 / S, cnt, (float*)tmp.data());
    if (rc != VS_OK) return rc;
    for (uint64_t i = 0; i < cnt; ++i)
      std::memcpy((unsigned char*)out + (g0 + i * S - first) * ob, tmp.data() + i * ob, ob);
  }
  return VS_OK;
}

int sharded_checksum(vs_engine* E, SColl& sc, uint64_t* out) {
  uint64_t sum = 0;
  for (uint32_t s = 0; s < E->shards(); ++s) {
    uint64_t part = 0;
    const int rc = vsd::checksum_shard(shard_eng(E, s), sc.iname[s].c_str(), E->shards(), s, &part);
    if (rc != VS_OK) return rc;
    sum += part;
  }
  *out = sum;
  return VS_OK;
}

// ---- snapshot file format (shared with vs_engine.cpp's single-device form) ----
struct SnapHeader {
  char magic[8];
  uint32_t version, header_bytes;
  uint32_t dim;
  int32_t metric, dtype;
  uint32_t elem_bytes;
  uint64_t rows, row_base, data_bytes;
  uint64_t data_checksum;
  uint64_t header_checksum;
  uint8_t reserved[56];
};
static_assert(sizeof(SnapHeader) == 128, "snapshot header is 128 bytes");
constexpr char kSnapMagic[8] = {'V', 'S', 'N', 'A', 'P', '0', '1', '\0'};
constexpr uint64_t kSnapChunk = 64ull << 20;

uint64_t header_sum(const SnapHeader& h) {
  uint64_t w[8], s = 0;
  std::memcpy(w, &h, 64);
  for (int i = 0; i < 8; ++i) s += vs::snap_word(w[i], (uint64_t)i);
  return s;
}

int sharded_drop(vs_engine* E, const char* name);
int sharded_create(vs_engine* E, const char* name, uint32_t dim, int metric, int dtype,
                   uint64_t capacity_hint, uint64_t row_base, const char* restore_path = nullptr);
void unplace(vs_engine* E, const SColl& sc);

// The same file as an unsharded snapshot of the collection (rows in global
// order, the global checksum), so a snapshot restores on any shard layout.
int sharded_snapshot(vs_engine* E, const char* coll, const char* path) {
  auto sc = find_scoll(E, coll);
  if (!sc) return not_found(coll);
  if (sc->home >= 0) return vsd::snapshot(home_eng(E, *sc), sc->iname[0].c_str(), path);
  std::shared_lock<std::shared_mutex> rl(sc->mu);  // upserts wait, searches proceed
  SnapHeader h{};
  std::memcpy(h.magic, kSnapMagic, 8);
  h.version = 1;
  h.header_bytes = sizeof(SnapHeader);
  h.dim = sc->dim;
  h.metric = sc->metric;
  h.dtype = sc->dtype;
  h.elem_bytes = sc->dtype == VS_DTYPE_BF16 ? 2 : 4;
  h.rows = sc->rows;
  h.row_base = 0;
  h.data_bytes = h.rows * h.dim * (uint64_t)h.elem_bytes;
  int rc = sharded_checksum(E, *sc, &h.data_checksum);
  if (rc != VS_OK) return rc;
  h.header_checksum = header_sum(h);
  const std::string tmp = std::string(path) + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return fail(VS_ERR_IO, "cannot open " + tmp + " for writing");
  bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1;
  const uint64_t rb = (uint64_t)h.dim * h.elem_bytes;
  const uint64_t per = std::max<uint64_t>(1, kSnapChunk / rb);
  std::vector<unsigned char> buf;
  for (uint64_t r0 = 0; ok && r0 < h.rows; r0 += per) {
    const uint64_t n = std::min(per, h.rows - r0);
    buf.resize(n * rb);
    rc = sharded_read<true>(E, *sc, r0, n, buf.data());
    if (rc != VS_OK) {
      std::fclose(f);
      return rc;
    }
    ok = std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
  }
  ok = (std::fclose(f) == 0) && ok;
  if (!ok || std::rename(tmp.c_str(), path) != 0)
    return fail(VS_ERR_IO, std::string("cannot write ") + path);
  return VS_OK;
}

int sharded_restore(vs_engine* E, const char* coll, const char* path) {
  if (E->placed) {  // dim / metric / dtype come from the file on the home device
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail(VS_ERR_IO, std::string("cannot open ") + path);
    SnapHeader h{};
    const bool ok = std::fread(&h, sizeof(h), 1, f) == 1;
    std::fclose(f);
    if (!ok || std::memcmp(h.magic, kSnapMagic, 8) != 0)
      return fail(VS_ERR_IO, std::string("not a vsearch snapshot (bad header): ") + path);
    return sharded_create(E, coll, h.dim, h.metric, h.dtype, h.rows, h.row_base, path);
  }
  FILE* f = std::fopen(path, "rb");
  if (!f) return fail(VS_ERR_IO, std::string("cannot open ") + path);
  SnapHeader h{};
  const bool hdr_ok = std::fread(&h, sizeof(h), 1, f) == 1 &&
                      std::memcmp(h.magic, kSnapMagic, 8) == 0 && h.version == 1 &&
                      h.header_bytes == sizeof(SnapHeader) && header_sum(h) == h.header_checksum;
  const uint32_t elem = h.dtype == VS_DTYPE_BF16 ? 2 : 4;
  if (!hdr_ok || h.elem_bytes != elem || h.data_bytes != h.rows * h.dim * (uint64_t)elem) {
    std::fclose(f);
    return fail(VS_ERR_IO, std::string("not a vsearch snapshot (bad header): ") + path);
  }
  if (h.row_base != 0) {
    std::fclose(f);
    return fail(VS_ERR_INVALID_ARG, "a sharded engine restores snapshots with row_base 0 only");
  }
  int rc = sharded_create(E, coll, h.dim, h.metric, h.dtype, h.rows, 0);
  if (rc != VS_OK) {
    std::fclose(f);
    return rc;
  }
  auto sc = find_scoll(E, coll);
  const uint32_t S = E->shards();
  const uint64_t rb = (uint64_t)h.dim * elem;
  const uint64_t per = std::max<uint64_t>(S, (kSnapChunk / rb) / S * S);
  std::vector<unsigned char> buf, part;
  std::string msg;
  {
    std::unique_lock<std::shared_mutex> wl(sc->mu);
    for (uint64_t r0 = 0; rc == VS_OK && r0 < h.rows; r0 += per) {
      const uint64_t n = std::min(per, h.rows - r0);
      buf.resize(n * rb);
      if (std::fread(buf.data(), 1, buf.size(), f) != buf.size()) {
        rc = VS_ERR_IO;
        msg = std::string("truncated snapshot: ") + path;
        break;
      }
      for (uint32_t s = 0; s < S && rc == VS_OK; ++s) {
        uint64_t g0, cnt;
        stripe_range(r0, r0 + n, S, s, &g0, &cnt);
        part.resize(cnt * rb);
        for (uint64_t i = 0; i < cnt; ++i)
          std::memcpy(part.data() + i * rb, buf.data() + (g0 + i * S - r0) * rb, rb);
        rc = vsd::append_raw(shard_eng(E, s), sc->iname[s].c_str(), cnt, part.data());
        if (rc != VS_OK) msg = vsd::last_error();
      }
      if (rc == VS_OK) sc->rows = r0 + n;
    }
    uint64_t sum = 0;
    if (rc == VS_OK) {
      rc = sharded_checksum(E, *sc, &sum);
      if (rc != VS_OK) msg = vsd::last_error();
      else if (sum != h.data_checksum) {
        rc = VS_ERR_IO;
        msg = std::string("snapshot checksum mismatch: ") + path;
      }
    }
  }
  std::fclose(f);
  if (rc != VS_OK) {
    (void)sharded_drop(E, coll);
    return fail(rc, msg);
  }
  return VS_OK;
}

// a placed collection leaves the engine's map and its device's balance
void unplace(vs_engine* E, const SColl& sc) {
  std::lock_guard<std::mutex> g(E->map_mu);
  auto it = E->colls.find(sc.name);
  if (it != E->colls.end() && it->second.get() == &sc) E->colls.erase(it);
  E->dev_bytes[sc.home] -= sc.reserved;
  E->dev_colls[sc.home] -= 1;
}

// restore_path (placed engines only): the collection is made by vs_restore of
// that snapshot on its device instead of created empty
int sharded_create(vs_engine* E, const char* name, uint32_t dim, int metric, int dtype,
                   uint64_t capacity_hint, uint64_t row_base, const char* restore_path) {
  if (!name || !*name) return fail(VS_ERR_INVALID_ARG, "collection name required");
  auto sc = std::make_shared<SColl>();
  sc->name = name;
  sc->gen = g_scoll_gen.fetch_add(1);
  sc->dim = dim;
  sc->metric = metric;
  sc->dtype = dtype;
  if (E->placed) {
    // the whole collection on the device with the fewest reserved bytes
    // (then the fewest collections, then the lowest index)
    sc->iname.push_back(std::string(name) + "\x1fp");
    sc->reserved = capacity_hint * dim * (dtype == VS_DTYPE_BF16 ? 2u : 4u) +
                   vsd::q8_reserve_bytes(E->dev[0]->flags, dim, dtype, capacity_hint);
    {
      std::lock_guard<std::mutex> g(E->map_mu);
      if (E->colls.count(name))
        return fail(VS_ERR_EXISTS, std::string("collection ") + name + " already exists");
      uint32_t best = 0;
      for (uint32_t d = 1; d < E->dev.size(); ++d)
        if (std::make_pair(E->dev_bytes[d], E->dev_colls[d]) <
            std::make_pair(E->dev_bytes[best], E->dev_colls[best]))
          best = d;
      sc->home = (int)best;
      E->dev_bytes[best] += sc->reserved;
      E->dev_colls[best] += 1;
      E->colls[name] = sc;
    }
    const int rc =
        restore_path
            ? vsd::restore(home_eng(E, *sc), sc->iname[0].c_str(), restore_path)
            : vsd::collection_create(home_eng(E, *sc), sc->iname[0].c_str(), dim, metric, dtype,
                                     capacity_hint, row_base);
    if (rc != VS_OK) {
      const std::string msg = vsd::last_error();
      unplace(E, *sc);
      return fail(rc, msg);
    }
    sc->ready.store(true, std::memory_order_release);
    return VS_OK;
  }
  if (row_base != 0)
    return fail(VS_ERR_INVALID_ARG, "row_base must be 0 on a sharded engine (rows are striped)");
  const uint32_t S = E->shards();
  for (uint32_t s = 0; s < S; ++s) sc->iname.push_back(std::string(name) + "\x1f" + std::to_string(s));
  {
    std::lock_guard<std::mutex> g(E->map_mu);
    if (E->colls.count(name))
      return fail(VS_ERR_EXISTS, std::string("collection ") + name + " already exists");
    E->colls[name] = sc;
  }
  for (uint32_t s = 0; s < S; ++s) {
    const uint64_t cap = capacity_hint ? (capacity_hint + S - 1 - s) / S : 0;
    const int rc = vsd::collection_create(shard_eng(E, s), sc->iname[s].c_str(), dim, metric,
                                          dtype, cap, 0);
    if (rc != VS_OK) {
      const std::string msg = vsd::last_error();
      for (uint32_t t = 0; t < s; ++t) (void)vsd::collection_drop(shard_eng(E, t), sc->iname[t].c_str());
      std::lock_guard<std::mutex> g(E->map_mu);
      E->colls.erase(name);
      return fail(rc, msg);
    }
  }
  sc->ready.store(true, std::memory_order_release);
  return VS_OK;
}

int sharded_drop(vs_engine* E, const char* name) {
  std::shared_ptr<SColl> sc;
  {
    std::lock_guard<std::mutex> g(E->map_mu);
    auto it = E->colls.find(name ? name : "");
    if (it == E->colls.end() || !it->second->ready.load(std::memory_order_acquire))
      return not_found(name);  // absent, or still being made by its creating call
    sc = it->second;
    E->colls.erase(it);
  }
  std::unique_lock<std::shared_mutex> wl(sc->mu);
  {
    std::lock_guard<std::mutex> g(E->filt_mu);
    for (auto it = E->filters.begin(); it != E->filters.end();)
      it = it->second.coll_gen == sc->gen ? E->filters.erase(it) : std::next(it);
  }
  if (sc->home >= 0) {
    (void)vsd::collection_drop(home_eng(E, *sc), sc->iname[0].c_str());  // frees its filters
    std::lock_guard<std::mutex> g(E->map_mu);
    E->dev_bytes[sc->home] -= sc->reserved;
    E->dev_colls[sc->home] -= 1;
    return VS_OK;
  }
  for (uint32_t s = 0; s < E->shards(); ++s)
    (void)vsd::collection_drop(shard_eng(E, s), sc->iname[s].c_str());  // frees shard filters
  return VS_OK;
}

int sharded_upsert(vs_engine* E, const char* coll, uint64_t n, uint32_t dim, const uint64_t* rows,
                   const float* vecs) {
  if (n == 0) return VS_OK;
  if (!rows || !vecs) return fail(VS_ERR_INVALID_ARG, "rows and vecs are required");
  auto sc = find_scoll(E, coll);
  if (!sc) return not_found(coll);
  if (sc->home >= 0) return vsd::upsert(home_eng(E, *sc), sc->iname[0].c_str(), n, dim, rows, vecs);
  if (dim != sc->dim)
    return fail(VS_ERR_DIM_MISMATCH, "Vector dimension error: expected dim: " +
                                         std::to_string(sc->dim) + ", got " + std::to_string(dim));
  std::unique_lock<std::shared_mutex> wl(sc->mu);
  // the same contract as one device: appended rows exactly [rows, rows + m)
  std::vector<uint64_t> fresh;
  for (uint64_t i = 0; i < n; ++i)
    if (rows[i] >= sc->rows) fresh.push_back(rows[i]);
  std::sort(fresh.begin(), fresh.end());
  fresh.erase(std::unique(fresh.begin(), fresh.end()), fresh.end());
  for (size_t i = 0; i < fresh.size(); ++i)
    if (fresh[i] != sc->rows + i)
      return fail(VS_ERR_INVALID_ARG, "upsert would leave a hole: appended rows must be "
                                      "contiguous from the current row count");
  const uint64_t total = sc->rows + fresh.size();
  if (total >= 0xFFFFFFFFull) return fail(VS_ERR_INVALID_ARG, "too many rows");
  const uint32_t S = E->shards();
  std::vector<std::vector<uint64_t>> lrows(S);
  std::vector<std::vector<float>> lvecs(S);
  for (uint64_t i = 0; i < n; ++i) {  // request order kept: the last duplicate wins
    const uint32_t s = (uint32_t)(rows[i] % S);
    lrows[s].push_back(rows[i] / S);
    lvecs[s].insert(lvecs[s].end(), vecs + i * dim, vecs + (i + 1) * dim);
  }
  for (uint32_t s = 0; s < S; ++s) {
    if (lrows[s].empty()) continue;
    const int rc = vsd::upsert(shard_eng(E, s), sc->iname[s].c_str(), lrows[s].size(), dim,
                               lrows[s].data(), lvecs[s].data());
    if (rc != VS_OK) return rc;  // earlier shards keep their rows
  }
  sc->rows = total;
  return VS_OK;
}

int sharded_generate(vs_engine* E, const char* coll, uint64_t n, uint64_t seed) {
  auto sc = find_scoll(E, coll);
  if (!sc) return not_found(coll);
  if (sc->home >= 0)
    return vsd::generate(home_eng(E, *sc), sc->iname[0].c_str(), n, seed, UINT64_MAX, 1);
  if (n == 0) return VS_OK;
  std::unique_lock<std::shared_mutex> wl(sc->mu);
  if (sc->rows + n >= 0xFFFFFFFFull) return fail(VS_ERR_INVALID_ARG, "too many rows");
  const uint32_t S = E->shards();
  for (uint32_t s = 0; s < S; ++s) {
    uint64_t g0, cnt;
    stripe_range(sc->rows, sc->rows + n, S, s, &g0, &cnt);
    if (!cnt) continue;
    const int rc = vsd::generate(shard_eng(E, s), sc->iname[s].c_str(), cnt, seed, g0, S);
    if (rc != VS_OK) return rc;
  }
  sc->rows += n;
  return VS_OK;
}

int sharded_filter_create(vs_engine* E, const char* coll, const uint64_t* allow,
                          uint64_t allow_words, uint64_t* filter_id) {
  if (!allow || !filter_id) return fail(VS_ERR_INVALID_ARG, "NULL argument");
  auto sc = find_scoll(E, coll);
  if (!sc) return not_found(coll);
  SFilter f;
  f.coll_gen = sc->gen;
  if (sc->home >= 0) {  // the device engine binds it to the collection's state
    uint64_t id = 0;
    const int rc = vsd::filter_create(home_eng(E, *sc), sc->iname[0].c_str(), allow, allow_words, &id);
    if (rc != VS_OK) return rc;
    f.dev_fid.push_back(id);
    f.dev_idx.push_back((uint32_t)sc->home);
    std::lock_guard<std::mutex> g(E->filt_mu);
    *filter_id = E->next_filter++;
    E->filters.emplace(*filter_id, std::move(f));
    return VS_OK;
  }
  std::shared_lock<std::shared_mutex> rl(sc->mu);
  if (allow_words < (sc->rows + 63) / 64)
    return fail(VS_ERR_INVALID_ARG, "filter bitmap has " + std::to_string(allow_words) +
                                        " words, the collection needs " +
                                        std::to_string((sc->rows + 63) / 64));
  f.rows = sc->rows;
  std::vector<uint64_t> bits;
  for (uint32_t s = 0; s < E->shards(); ++s) {
    deinterleave_bits(allow, sc->rows, E->shards(), s, &bits);
    uint64_t id = 0;
    const int rc = vsd::filter_create(shard_eng(E, s), sc->iname[s].c_str(), bits.data(),
                                      bits.size(), &id);
    if (rc != VS_OK) {
      const std::string msg = vsd::last_error();
      for (uint32_t t = 0; t < s; ++t) (void)vsd::filter_drop(shard_eng(E, t), f.dev_fid[t]);
      return fail(rc, msg);
    }
    f.dev_fid.push_back(id);
    f.dev_idx.push_back(E->shard_dev[s]);
  }
  std::lock_guard<std::mutex> g(E->filt_mu);
  *filter_id = E->next_filter++;
  E->filters.emplace(*filter_id, std::move(f));
  return VS_OK;
}

int sharded_filter_drop(vs_engine* E, uint64_t filter_id) {
  SFilter f;
  {
    std::lock_guard<std::mutex> g(E->filt_mu);
    auto it = E->filters.find(filter_id);
    if (it == E->filters.end())
      return fail(VS_ERR_NOT_FOUND, "filter " + std::to_string(filter_id) + " not found");
    f = std::move(it->second);
    E->filters.erase(it);
  }
  for (uint32_t s = 0; s < f.dev_fid.size(); ++s)  // gone already if its collection was dropped
    (void)vsd::filter_drop(E->dev[f.dev_idx[s]], f.dev_fid[s]);
  return VS_OK;
}

void destroy(vs_engine* E) {
  for (auto& up : E->sets) {
    CtxSet& cx = *up;
    for (size_t d = 0; d < cx.dev.size(); ++d) {
      if (!cx.dev[d]) continue;
      (void)hipSetDevice(cx.dev[d]->device);
      (void)hipStreamSynchronize(cx.dev[d]->stream);
      if (d < cx.scr.size()) {
        auto& x = cx.scr[d];  // freed with the device current
        if (x.qev) (void)hipEventDestroy(x.qev);
        if (x.kev) (void)hipEventDestroy(x.kev);
        for (DevBuf* b : {&x.q, &x.keys, &x.merged, &x.gather, &x.out, &x.allow}) b->release();
      }
      if (d < cx.comm.size() && cx.comm[d]) (void)ncclCommDestroy(cx.comm[d]);
    }
    if (!cx.dev.empty() && cx.dev[0]) {
      (void)hipSetDevice(cx.dev[0]->device);
      cx.host_slots.clear();
    }
  }
  E->sets.clear();
  for (size_t d = 0; d < E->coll_ev.size(); ++d)
    if (E->coll_ev[d]) {
      (void)hipSetDevice(E->dev[d]->device);
      (void)hipEventDestroy(E->coll_ev[d]);
    }
  if (!E->dev.empty() && E->dev[0]) {
    (void)hipSetDevice(E->dev[0]->device);
    (void)hipStreamSynchronize(E->dev[0]->stream);
    if (E->gm_ev) (void)hipEventSynchronize(E->gm_ev);  // the last exchange read pgather
    E->pgather.release();
    if (E->gm_ev) (void)hipEventDestroy(E->gm_ev);
    if (E->pcomm) (void)ncclCommDestroy(E->pcomm);
  }
  E->colls.clear();
  for (DevEngine* d : E->dev) vsd::close(d);
  delete E;
}

}  // namespace

extern "C" {

const char* vs_last_error(void) { return vsd::last_error(); }

size_t vs_copy_last_error(char* buf, size_t len) {
  const char* m = vsd::last_error();
  const size_t n = std::strlen(m);
  if (buf && len) {
    const size_t c = n < len - 1 ? n : len - 1;
    std::memcpy(buf, m, c);
    buf[c] = '\0';
  }
  return n;
}

int vs_runtime_check(void) { return vsd::one_hip_runtime(); }

int vs_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int vs_open(const vs_config* cfg, vs_engine** out) {
  if (!out) return fail(VS_ERR_INVALID_ARG, "out is NULL");
  *out = nullptr;
  DevEngine* d = nullptr;
  const int rc = vsd::open(cfg ? cfg->device : -1, cfg ? cfg->flags : 0, &d);
  if (rc != VS_OK) return rc;
  auto* E = new vs_engine();
  E->dev.push_back(d);
  E->shard_dev.push_back(0);
  E->dev_shards.push_back({0});
  *out = E;
  return VS_OK;
}

int vs_open_multi(const vs_config_multi* cfg, vs_engine** out) {
  if (!out || !cfg) return fail(VS_ERR_INVALID_ARG, "cfg and out are required");
  *out = nullptr;
  if (cfg->n_shards == 0 || cfg->n_shards > 4096)
    return fail(VS_ERR_INVALID_ARG, "n_shards must be in [1, 4096]");
  const int ndev = vs_device_count();
  if (ndev <= 0) return fail(VS_ERR_DEVICE, "no HIP device available (the engine has no CPU fallback)");
  std::vector<int> ord(cfg->n_shards);
  for (uint32_t s = 0; s < cfg->n_shards; ++s) {
    ord[s] = cfg->devices ? cfg->devices[s] : (int)s;
    if (ord[s] < 0 || ord[s] >= ndev)
      return fail(VS_ERR_INVALID_ARG, "shard " + std::to_string(s) + ": device ordinal " +
                                          std::to_string(ord[s]) + " out of range");
  }
  auto* E = new vs_engine();
  E->sharded = cfg->n_shards > 1;
  E->placed = E->sharded && (cfg->flags & VS_FLAG_PLACE_COLLECTIONS);
  // VS_FLAG_ENGINE_PER_SHARD: a device engine per entry, repeated ordinals included
  const bool per_shard = E->placed && (cfg->flags & VS_FLAG_ENGINE_PER_SHARD);
  std::vector<int> devlist;
  for (uint32_t s = 0; s < cfg->n_shards; ++s) {
    auto it = per_shard ? devlist.end() : std::find(devlist.begin(), devlist.end(), ord[s]);
    uint32_t d = (uint32_t)(it - devlist.begin());
    if (it == devlist.end()) {
      DevEngine* de = nullptr;
      const int rc = vsd::open(ord[s], cfg->flags, &de);
      if (rc != VS_OK) {
        const std::string msg = vsd::last_error();
        destroy(E);
        return fail(rc, msg);
      }
      devlist.push_back(ord[s]);
      E->dev.push_back(de);
      E->dev_shards.emplace_back();
    }
    E->shard_dev.push_back(d);
    E->dev_shards[d].push_back(s);
  }
  if (E->sharded) {
    E->dev_bytes.assign(E->dev.size(), 0);
    E->dev_colls.assign(E->dev.size(), 0);
    if (!E->placed) {
      E->coll_ev.assign(E->dev.size(), nullptr);
      for (size_t d = 0; d < E->dev.size(); ++d) {
        (void)hipSetDevice(E->dev[d]->device);
        if (hipEventCreateWithFlags(&E->coll_ev[d], hipEventDisableTiming) != hipSuccess) {
          destroy(E);
          return fail(VS_ERR_DEVICE, "event");
        }
      }
    }
    // context set j = search context j of every device
    size_t nsets = SIZE_MAX;
    for (DevEngine* de : E->dev) nsets = std::min(nsets, de->store->ctx.size());
    for (size_t j = 0; j < nsets; ++j) {
      auto cs = std::make_unique<CtxSet>();
      for (DevEngine* de : E->dev) cs->dev.push_back(de->store->ctx[j]);
      cs->scr.resize(E->dev.size());
      E->sets.push_back(std::move(cs));
      CtxSet& cx = *E->sets.back();
      if (!E->placed) {  // placed collections never exchange keys: no communicator
        cx.comm.assign(E->dev.size(), nullptr);
        const ncclResult_t r = ncclCommInitAll(cx.comm.data(), (int)devlist.size(), devlist.data());
        if (r != ncclSuccess) {
          const std::string msg = std::string("ncclCommInitAll: ") + ncclGetErrorString(r);
          cx.comm.clear();
          destroy(E);
          return fail(VS_ERR_DEVICE, msg);
        }
      }
      for (size_t d = 0; d < E->dev.size(); ++d) {
        (void)hipSetDevice(E->dev[d]->device);
        if ((d == 0 && hipEventCreateWithFlags(&cx.scr[0].qev, hipEventDisableTiming) != hipSuccess) ||
            hipEventCreateWithFlags(&cx.scr[d].kev, hipEventDisableTiming) != hipSuccess) {
          destroy(E);
          return fail(VS_ERR_DEVICE, "event");
        }
      }
    }
  }
  *out = E;
  return VS_OK;
}

int vs_collection_placement(vs_engine* eng, const char* name, int32_t* device) {
  if (!eng || !device) return fail(VS_ERR_INVALID_ARG, "engine and device are required");
  if (!eng->sharded) {
    if (!vsd::find_coll(eng->dev[0], name)) return not_found(name);
    *device = eng->dev[0]->device;
    return VS_OK;
  }
  auto sc = find_scoll(eng, name);
  if (!sc) return not_found(name);
  *device = sc->home >= 0 ? home_eng(eng, *sc)->device
                          : (eng->dev.size() == 1 ? eng->dev[0]->device : -1);
  return VS_OK;
}

int vs_engine_layout(vs_engine* eng, uint32_t* n_shards, uint32_t* n_devices) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (n_shards) *n_shards = eng->shards();
  if (n_devices) *n_devices = (uint32_t)eng->dev.size();
  return VS_OK;
}

void vs_close(vs_engine* eng) {
  if (eng) destroy(eng);
}

int vs_collection_create(vs_engine* eng, const char* name, uint32_t dim, int metric, int dtype,
                         uint64_t capacity_hint, uint64_t row_base) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (!eng->sharded)
    return vsd::collection_create(eng->dev[0], name, dim, metric, dtype, capacity_hint, row_base);
  if (dim == 0 || dim > 65536) return fail(VS_ERR_INVALID_ARG, "dim must be in [1, 65536]");
  if (metric != VS_METRIC_COSINE && metric != VS_METRIC_DOT)
    return fail(VS_ERR_INVALID_ARG, "unknown metric");
  if (dtype != VS_DTYPE_F32 && dtype != VS_DTYPE_BF16)
    return fail(VS_ERR_INVALID_ARG, "unknown dtype");
  return sharded_create(eng, name, dim, metric, dtype, capacity_hint, row_base);
}

int vs_collection_info(vs_engine* eng, const char* name, uint32_t* dim, uint64_t* rows,
                       int* metric, int* dtype) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (!eng->sharded) return vsd::collection_info(eng->dev[0], name, dim, rows, metric, dtype);
  auto sc = find_scoll(eng, name);
  if (!sc) return not_found(name);
  if (sc->home >= 0)
    return vsd::collection_info(home_eng(eng, *sc), sc->iname[0].c_str(), dim, rows, metric, dtype);
  std::shared_lock<std::shared_mutex> rl(sc->mu);
  if (dim) *dim = sc->dim;
  if (rows) *rows = sc->rows;
  if (metric) *metric = sc->metric;
  if (dtype) *dtype = sc->dtype;
  return VS_OK;
}

int vs_collection_drop(vs_engine* eng, const char* name) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (!eng->sharded) return vsd::collection_drop(eng->dev[0], name);
  return sharded_drop(eng, name);
}

int vs_collection_prefilter_bytes(vs_engine* eng, const char* name, uint64_t* bytes) {
  if (!eng || !bytes) return fail(VS_ERR_INVALID_ARG, "engine and bytes are required");
  if (!eng->sharded) return vsd::prefilter_bytes(eng->dev[0], name, bytes);
  auto sc = find_scoll(eng, name);
  if (!sc) return not_found(name);
  if (sc->home >= 0) return vsd::prefilter_bytes(home_eng(eng, *sc), sc->iname[0].c_str(), bytes);
  uint64_t sum = 0;
  for (uint32_t s = 0; s < eng->shards(); ++s) {
    uint64_t part = 0;
    const int rc = vsd::prefilter_bytes(shard_eng(eng, s), sc->iname[s].c_str(), &part);
    if (rc != VS_OK) return rc;
    sum += part;
  }
  *bytes = sum;
  return VS_OK;
}

int vs_collection_spec_stats(vs_engine* eng, const char* name, uint64_t out[4]) {
  if (!eng || !out) return fail(VS_ERR_INVALID_ARG, "engine and out are required");
  if (!eng->sharded) return vsd::spec_stats(eng->dev[0], name, out);
  auto sc = find_scoll(eng, name);
  if (!sc) return not_found(name);
  if (sc->home >= 0) return vsd::spec_stats(home_eng(eng, *sc), sc->iname[0].c_str(), out);
  uint64_t sum[4] = {0, 0, 0, 0};
  for (uint32_t s = 0; s < eng->shards(); ++s) {
    uint64_t part[4];
    const int rc = vsd::spec_stats(shard_eng(eng, s), sc->iname[s].c_str(), part);
    if (rc != VS_OK) return rc;
    for (int j = 0; j < 4; ++j) sum[j] += part[j];
  }
  std::memcpy(out, sum, sizeof(sum));
  return VS_OK;
}

int vs_upsert(vs_engine* eng, const char* coll, uint64_t n, uint32_t dim, const uint64_t* rows,
              const float* vecs) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (!eng->sharded) return vsd::upsert(eng->dev[0], coll, n, dim, rows, vecs);
  return sharded_upsert(eng, coll, n, dim, rows, vecs);
}

int vs_generate(vs_engine* eng, const char* coll, uint64_t n, uint64_t seed) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (!eng->sharded) return vsd::generate(eng->dev[0], coll, n, seed, UINT64_MAX, 1);
  return sharded_generate(eng, coll, n, seed);
}

int vs_generate_vectors(vs_engine* eng, uint64_t seed, uint64_t row0, uint64_t n, uint32_t dim,
                        float* d_out, void* stream) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (const int rt = vsd::one_hip_runtime()) return rt;
  return vsd::generate_vectors(eng->dev[0], seed, row0, n, dim, d_out, stream);
}

int vs_read_rows(vs_engine* eng, const char* coll, uint64_t first, uint64_t n, float* out) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (!eng->sharded) return vsd::read_rows(eng->dev[0], coll, first, n, out);
  auto sc = find_scoll(eng, coll);
  if (!sc) return not_found(coll);
  if (sc->home >= 0) return vsd::read_rows(home_eng(eng, *sc), sc->iname[0].c_str(), first, n, out);
  std::shared_lock<std::shared_mutex> rl(sc->mu);
  if (first + n > sc->rows || first + n < first)
    return fail(VS_ERR_INVALID_ARG, "row range out of bounds");
  if (n == 0) return VS_OK;
  if (!out) return fail(VS_ERR_INVALID_ARG, "out is NULL");
  return sharded_read<false>(eng, *sc, first, n, out);
}

int vs_search(vs_engine* eng, const char* coll, const float* queries, uint32_t nq, uint32_t dim,
              uint32_t k, float* out_scores, uint64_t* out_rows, uint32_t* out_count) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (!eng->sharded)
    return vsd::search_host(eng->dev[0], coll, queries, nq, dim, k, nullptr, 0, out_scores,
                            out_rows, out_count);
  return sharded_search_host(eng, coll, queries, nq, dim, k, nullptr, 0, 0, out_scores, out_rows,
                             out_count);
}

int vs_search_filtered(vs_engine* eng, const char* coll, const float* queries, uint32_t nq,
                       uint32_t dim, uint32_t k, const uint64_t* allow, uint64_t allow_words,
                       float* out_scores, uint64_t* out_rows, uint32_t* out_count) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (!allow) return fail(VS_ERR_INVALID_ARG, "allow bitmap is NULL");
  if (!eng->sharded)
    return vsd::search_host(eng->dev[0], coll, queries, nq, dim, k, allow, allow_words, out_scores,
                            out_rows, out_count);
  return sharded_search_host(eng, coll, queries, nq, dim, k, allow, allow_words, 0, out_scores,
                             out_rows, out_count);
}

int vs_filter_create(vs_engine* eng, const char* coll, const uint64_t* allow, uint64_t allow_words,
                     uint64_t* filter_id) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (!eng->sharded) return vsd::filter_create(eng->dev[0], coll, allow, allow_words, filter_id);
  return sharded_filter_create(eng, coll, allow, allow_words, filter_id);
}

int vs_filter_drop(vs_engine* eng, uint64_t filter_id) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (!eng->sharded) return vsd::filter_drop(eng->dev[0], filter_id);
  return sharded_filter_drop(eng, filter_id);
}

int vs_search_filter_id(vs_engine* eng, const char* coll, const float* queries, uint32_t nq,
                        uint32_t dim, uint32_t k, uint64_t filter_id, float* out_scores,
                        uint64_t* out_rows, uint32_t* out_count) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (!filter_id) return fail(VS_ERR_INVALID_ARG, "filter id 0");
  if (!eng->sharded)
    return vsd::search_host(eng->dev[0], coll, queries, nq, dim, k, nullptr, 0, out_scores,
                            out_rows, out_count, filter_id);
  return sharded_search_host(eng, coll, queries, nq, dim, k, nullptr, 0, filter_id, out_scores,
                             out_rows, out_count);
}

int vs_search_keys(vs_engine* eng, const char* coll, const float* d_queries, uint32_t nq,
                   uint32_t dim, uint32_t k, uint64_t* d_keys, void* stream) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (const int rt = vsd::one_hip_runtime()) return rt;
  if (!eng->sharded)
    return vsd::search_keys(eng->dev[0], coll, d_queries, nq, dim, k, d_keys, stream);
  if (k == 0) return fail(VS_ERR_INVALID_ARG, "k must be at least 1");
  if (nq == 0) return VS_OK;
  if (!d_queries || !d_keys) return fail(VS_ERR_INVALID_ARG, "NULL device pointer");
  auto sc = find_scoll(eng, coll);
  if (!sc) return not_found(coll);
  if (sc->home == 0)
    return vsd::search_keys(eng->dev[0], sc->iname[0].c_str(), d_queries, nq, dim, k, d_keys, stream);
  if (sc->home > 0) {
    uint32_t cdim = 0;
    const int rc = vsd::collection_info(home_eng(eng, *sc), sc->iname[0].c_str(), &cdim, nullptr,
                                        nullptr, nullptr);
    if (rc != VS_OK) return rc;
    if (dim != cdim)
      return fail(VS_ERR_DIM_MISMATCH, "Vector dimension error: expected dim: " +
                                           std::to_string(cdim) + ", got " + std::to_string(dim));
    return placed_search_keys(eng, *sc, d_queries, nq, k, d_keys, (hipStream_t)stream);
  }
  if (dim != sc->dim)
    return fail(VS_ERR_DIM_MISMATCH, "Vector dimension error: expected dim: " +
                                         std::to_string(sc->dim) + ", got " + std::to_string(dim));
  std::shared_lock<std::shared_mutex> rl(sc->mu);
  CtxSet& cx = *eng->sets[0];  // the primary contexts: the caller's stream orders the work
  AllWork aw(cx);
  DevEngine* d0 = eng->dev[0];
  VS_HIP(vsd::set_dev(d0), "hipSetDevice");
  hipStream_t cs = (hipStream_t)stream;
  // the other devices copy the queries once the caller's stream wrote them
  if (eng->dev.size() > 1) VS_HIP(hipEventRecord(cx.scr[0].qev, cs), "query event");
  return sharded_search(eng, cx, *sc, nullptr, d_queries, true, cs, nq, k, nullptr, nullptr,
                        nullptr, nullptr, d_keys);
}

int vs_merge_keys(vs_engine* eng, const uint64_t* d_lists, uint32_t n_lists, uint32_t nq,
                  uint32_t k_in, uint32_t k, uint64_t* d_out_keys, void* stream) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (const int rt = vsd::one_hip_runtime()) return rt;
  return vsd::merge_keys(eng->dev[0], d_lists, n_lists, nq, k_in, k, d_out_keys, stream);
}

int vs_comm_unique_id(unsigned char id[VS_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == VS_COMM_ID_BYTES, "RCCL unique id size");
  if (!id) return fail(VS_ERR_INVALID_ARG, "id is NULL");
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
  std::memcpy(id, &u, sizeof(u));
  return VS_OK;
}

int vs_comm_init(vs_engine* eng, uint32_t n_ranks, uint32_t rank,
                 const unsigned char id[VS_COMM_ID_BYTES]) {
  if (!eng || !id) return fail(VS_ERR_INVALID_ARG, "engine and id are required");
  if (eng->sharded)
    return fail(VS_ERR_INVALID_ARG, "a vs_open_multi engine holds its own communicator");
  if (n_ranks == 0 || rank >= n_ranks) return fail(VS_ERR_INVALID_ARG, "rank out of range");
  DevEngine* d0 = eng->dev[0];
  std::lock_guard<std::mutex> g(d0->work_mu);
  if (eng->pcomm) return fail(VS_ERR_EXISTS, "vs_comm_init was called already");
  VS_HIP(vsd::set_dev(d0), "hipSetDevice");
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  const ncclResult_t r = ncclCommInitRank(&c, (int)n_ranks, u, (int)rank);
  if (r != ncclSuccess) return nccl_fail(r, "ncclCommInitRank");
  eng->pcomm = c;
  eng->pranks = n_ranks;
  eng->prank = rank;
  return VS_OK;
}

int vs_gather_merge_keys(vs_engine* eng, const uint64_t* d_local, uint32_t nq, uint32_t k_in,
                         uint32_t k, uint64_t* d_out_keys, void* stream) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (!eng->pcomm) return fail(VS_ERR_INVALID_ARG, "vs_comm_init has not been called");
  if (const int rt = vsd::one_hip_runtime()) return rt;
  if (k == 0 || k_in == 0) return fail(VS_ERR_INVALID_ARG, "bad merge shape");
  if (nq == 0) return VS_OK;
  if (!d_local || !d_out_keys) return fail(VS_ERR_INVALID_ARG, "NULL device pointer");
  DevEngine* d0 = eng->dev[0];
  hipStream_t cs = (hipStream_t)stream;
  const size_t lbytes = (size_t)nq * k_in * 8;
  std::lock_guard<std::mutex> g(eng->gm_mu);
  VS_HIP(vsd::set_dev(d0), "hipSetDevice");
  if (!eng->gm_ev) VS_HIP(hipEventCreateWithFlags(&eng->gm_ev, hipEventDisableTiming), "event");
  // the gather buffer is reused: this exchange runs after the previous one
  // (gm_ev: recorded after every exchange, on its stream)
  if (eng->gm_stream && eng->gm_stream != cs)
    VS_HIP(hipStreamWaitEvent(cs, eng->gm_ev, 0), "stream order");
  eng->gm_stream = cs;
  if (eng->pgather.bytes < lbytes * eng->pranks) {
    // (cs waits for the previous exchange, so this also drains that one)
    VS_HIP(hipStreamSynchronize(cs), "sync");
    VS_HIP(eng->pgather.ensure(lbytes * eng->pranks), "alloc gathered keys");
  }
  const ncclResult_t r = ncclAllGather(d_local, eng->pgather.p, (size_t)nq * k_in, ncclUint64,
                                       eng->pcomm, cs);
  int rc = VS_OK;
  if (r != ncclSuccess) {
    rc = nccl_fail(r, "ncclAllGather");
  } else if (k > vsk::kMaxK || k_in > vsk::kMaxK) {
    // the large-k merge uses the primary context's scratch: its stream order
    // too (lock order: gm_mu, then work_mu; nothing takes them the other way)
    std::lock_guard<std::mutex> w(d0->work_mu);
    const hipError_t e = vsd::use_stream(d0, cs);
    rc = e != hipSuccess ? ::vsd::fail_hip(e, "stream order")
                         : vsd::merge_any(d0, eng->pgather.as<uint64_t>(), eng->pranks,
                                          (uint64_t)nq * k_in, k_in, nq, k_in, k, d_out_keys);
  } else {
    const hipError_t e = vsk::launch_merge(eng->pgather.as<uint64_t>(), eng->pranks,
                                           (uint64_t)nq * k_in, k_in, nq, k_in, k, d_out_keys, cs);
    if (e != hipSuccess) rc = ::vsd::fail_hip(e, "merge");
  }
  // recorded whatever happened above: the next exchange waits for every
  // operation this one enqueued on pgather
  VS_HIP(hipEventRecord(eng->gm_ev, cs), "stream order");
  return rc;
}

int vs_decode_keys(vs_engine* eng, const uint64_t* d_keys, uint32_t nq, uint32_t k,
                   float* out_scores, uint64_t* out_rows, uint32_t* out_count, void* stream) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (const int rt = vsd::one_hip_runtime()) return rt;
  return vsd::decode_keys(eng->dev[0], d_keys, nq, k, out_scores, out_rows, out_count, stream);
}

int vs_checksum(vs_engine* eng, const char* coll, uint64_t* out) {
  if (!eng || !out) return fail(VS_ERR_INVALID_ARG, "engine and out are required");
  if (!eng->sharded) return vsd::checksum(eng->dev[0], coll, out);
  auto sc = find_scoll(eng, coll);
  if (!sc) return not_found(coll);
  if (sc->home >= 0) return vsd::checksum(home_eng(eng, *sc), sc->iname[0].c_str(), out);
  std::shared_lock<std::shared_mutex> rl(sc->mu);
  return sharded_checksum(eng, *sc, out);
}

int vs_snapshot(vs_engine* eng, const char* coll, const char* path) {
  if (!eng || !path) return fail(VS_ERR_INVALID_ARG, "engine and path are required");
  if (!eng->sharded) return vsd::snapshot(eng->dev[0], coll, path);
  return sharded_snapshot(eng, coll, path);
}

int vs_restore(vs_engine* eng, const char* coll, const char* path) {
  if (!eng || !path || !coll || !*coll)
    return fail(VS_ERR_INVALID_ARG, "engine, collection and path are required");
  if (!eng->sharded) return vsd::restore(eng->dev[0], coll, path);
  return sharded_restore(eng, coll, path);
}

int vs_health(vs_engine* eng, char* buf, size_t len) {
  if (!eng || !buf || len == 0) return fail(VS_ERR_INVALID_ARG, "bad health buffer");
  if (!eng->sharded) return vsd::health(eng->dev[0], buf, len);
  // {"status","engine","shards","device_name","collections","devices":[...]}
  std::string devs;
  bool healthy = true;
  std::string name0;
  for (size_t d = 0; d < eng->dev.size(); ++d) {
    char one[1024];
    const int rc = vsd::health(eng->dev[d], one, sizeof(one));
    healthy = healthy && rc == VS_OK;
    if (d) devs.push_back(',');
    devs.append(one);
    if (d == 0) {
      const char* dn = std::strstr(one, "\"device_name\":\"");
      if (dn) {
        dn += 15;
        const char* e = std::strchr(dn, '"');
        if (e) name0.assign(dn, e);
      }
    }
  }
  size_t ncoll;
  {
    std::lock_guard<std::mutex> g(eng->map_mu);
    ncoll = eng->colls.size();
  }
  const int n = std::snprintf(buf, len,
                              "{\"status\":\"%s\",\"engine\":\"vsearch-hip\",\"shards\":%u,"
                              "\"device_name\":\"%s\",\"collections\":%zu,"
                              "\"devices\":[%s]}",
                              healthy ? "healthy" : "degraded", eng->shards(), name0.c_str(), ncoll,
                              devs.c_str());
  if (n < 0 || (size_t)n >= len) return fail(VS_ERR_INVALID_ARG, "health buffer too small");
  return healthy ? VS_OK : fail(VS_ERR_DEVICE, "a device is degraded");
}

int vs_timing(vs_engine* eng, double* scan_ms_avg, uint64_t* scan_count, double* merge_ms_avg,
              uint64_t* merge_count, int reset) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  double sm = 0, mm = 0;
  uint64_t sn = 0, mn = 0;
  for (DevEngine* d : eng->dev) {
    double a = 0, b = 0;
    uint64_t x = 0, y = 0;
    const int rc = vsd::timing(d, &a, &x, &b, &y, reset);
    if (rc != VS_OK) return rc;
    sm += a, mm += b, sn += x, mn += y;
  }
  if (scan_ms_avg) *scan_ms_avg = sn ? sm / sn : 0.0;
  if (scan_count) *scan_count = sn;
  if (merge_ms_avg) *merge_ms_avg = mn ? mm / mn : 0.0;
  if (merge_count) *merge_count = mn;
  return VS_OK;
}

}  // extern "C"
