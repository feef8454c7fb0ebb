// vs_spec_host.h — the host side of the speculative bound's bookkeeping
// (DESIGN.md §5 "Speculative bound"): which k a search context may start a
// speculative batch from, and what the device's advice words say about it.
// Header-only and free of HIP, so vs_engine.cpp (search_mfma) runs it and
// tests/tsan/spec_driver.cpp runs the same code under ThreadSanitizer with
// many contexts, a device stand-in and a writer.
//
// Shared state and who touches it:
//  * SpecSeen maps: one per search context, only under that context's
//    work_mu (no sharing);
//  * Collection::q8_gen: written by a store-side call (the collection's
//    writer lock), read by searches (its reader lock);
//  * the advice words (coherent mapped host memory): written by the device
//    (system-scope atomic stores), reset by writers, read and counted off by
//    any context -- relaxed atomics only; they are hints, exactness never
//    rests on them (every speculative batch is checked on the device);
//  * the host-skip counter: a relaxed atomic.
#pragma once
#include <atomic>
#include <bitset>
#include <cstdint>
#include <unordered_map>

namespace vsd {

// k of the batched path: 0 .. kMfmaMaxK (vs_kernels.h kQ8SpecK; asserted
// equal in vs_engine.cpp)
constexpr uint32_t kSpecK = 129;
// While a k's speculative bound is judged loose, one batch in kLooseRecord
// records (and re-judges) it; the others run the sample path alone.
constexpr uint8_t kLooseRecord = 8;
// A context's spec_seen map is cleared when it grows past this many
// collections (it is a hint: dropped collections' entries go with the rest).
constexpr size_t kSpecSeenMax = 256;

// Per collection (Collection::gen): the int8 copy generation and the k this
// context has answered a batch of on its stream (a later batch of this
// context may then try the speculative bound).
struct SpecSeen {
  uint64_t q8_gen = 0;
  std::bitset<kSpecK> k;
  uint8_t loose_tick[kSpecK] = {};  // batches while the advice said loose
};
using SpecSeenMap = std::unordered_map<uint64_t, SpecSeen>;

struct SpecPlan {
  int spec_k = -1;      // the k' >= k whose ratio the batch starts from; -1: sample path
  bool record = true;   // the sample path's answer teaches the ratio
  SpecSeen* seen = nullptr;
};

// The plan of one unfiltered batch of k (work_mu of the context held, the
// collection's reader lock held). advice: the collection's 2 x kSpecK words
// ([k] loose, [kSpecK + k] cool-down batches left); force: tests' forced
// failures, which ignore the advice.
inline SpecPlan spec_plan(SpecSeenMap& map, uint64_t gen, uint64_t q8_gen, uint32_t k,
                          uint32_t* advice, bool force, std::atomic<uint64_t>& host_skips) {
  SpecPlan p;
  if (map.size() > kSpecSeenMax && !map.count(gen)) map.clear();
  SpecSeen* seen = &map[gen];
  p.seen = seen;
  if (seen->q8_gen != q8_gen) seen->q8_gen = q8_gen, seen->k.reset();
  for (uint32_t kk = k; kk < kSpecK && p.spec_k < 0; ++kk)
    if (seen->k[kk]) p.spec_k = (int)kk;
  // The device's advice (vs_kernels.h Q8SpecK). Loose: the last sample-path
  // record found the bound loose for this k, so the sample path alone and its
  // record only every kLooseRecord-th batch (which re-judges it). A cool-down
  // after a failed check: the sample path and its record, one batch counted
  // off (never below 0, whatever other contexts do meanwhile).
  if (p.spec_k >= 0 && !force) {
    uint32_t* cool = &advice[kSpecK + k];
    uint32_t n = __atomic_load_n(cool, __ATOMIC_RELAXED);
    while (n && !__atomic_compare_exchange_n(cool, &n, n - 1, false, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED)) {
    }
    if (__atomic_load_n(&advice[k], __ATOMIC_RELAXED) != 0u) {
      p.spec_k = -1;
      p.record = seen->loose_tick[k]++ % kLooseRecord == 0;
    } else if (n) {
      p.spec_k = -1;
    }
    if (p.spec_k < 0) host_skips.fetch_add(1, std::memory_order_relaxed);
  }
  return p;
}

// After the batch is enqueued: this context may try k from now on.
inline void spec_seen_mark(const SpecPlan& p, uint32_t k) {
  if (p.seen) p.seen->k[k] = true;
}

// A store-side write (the collection's writer lock held): every advice word
// back to "try, no cool-down" (the device-side state is reset on the stream).
inline void spec_advice_reset(uint32_t* advice) {
  for (uint32_t i = 0; i < 2 * kSpecK; ++i) __atomic_store_n(&advice[i], 0u, __ATOMIC_RELAXED);
}

}  // namespace vsd
