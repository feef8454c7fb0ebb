// ThreadSanitizer driver for the speculative bound's host bookkeeping
// (csrc/vs_spec_host.h). Test-only: no HIP, no device.
//
// The engine's sharing pattern, stood in for by threads:
//  * C search contexts, each with its own SpecSeen map and work mutex, taking
//    a collection's reader lock for every batch and planning it with
//    spec_plan (mixed k), then marking it seen;
//  * a "device" thread storing loose flags and cool-down lengths into the
//    advice words with relaxed atomic stores (the kernels' system-scope
//    stores);
//  * a writer taking the collection's writer lock, bumping q8_gen and
//    resetting the advice (q8_spec_reset);
//  * a dropper that replaces collections (new gen), so the maps grow and are
//    cleared past kSpecSeenMax.
// Pass: no TSAN report, and every plan is well-formed (spec_k in [k, 129) or
// -1; a skip counted for every advice-forced sample path).
//   clang++ -std=c++17 -O1 -g -fsanitize=thread -pthread -I<csrc> spec_driver.cpp
//   spec_driver THREADS ITERS
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <random>
#include <shared_mutex>
#include <thread>
#include <vector>

#include "vs_spec_host.h"

using namespace vsd;

struct Coll {
  std::shared_mutex mu;
  uint64_t gen = 0;
  uint64_t q8_gen = 1;
  uint32_t advice[2 * kSpecK] = {};
  std::atomic<uint64_t> host_skips{0};
};

int main(int argc, char** argv) {
  const int nctx = argc > 1 ? std::atoi(argv[1]) : 8;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 20000;
  constexpr int kColls = 4;
  std::vector<Coll> colls(kColls);
  for (int i = 0; i < kColls; ++i) colls[i].gen = (uint64_t)i + 1;
  std::atomic<uint64_t> next_gen{100};
  std::atomic<uint64_t> forced_skips{0};
  std::atomic<bool> bad{false}, stop{false};
  struct Ctx {
    std::mutex work_mu;
    SpecSeenMap seen;
  };
  std::vector<Ctx> ctx(nctx);
  std::vector<std::thread> th;
  for (int t = 0; t < nctx; ++t)
    th.emplace_back([&, t] {
      std::mt19937 rng(t + 1);
      const uint32_t ks[] = {1, 3, 10, 50, 64, 100, 128};
      for (int i = 0; i < iters; ++i) {
        Coll& c = colls[rng() % kColls];
        const uint32_t k = ks[rng() % 7];
        Ctx& x = ctx[rng() % nctx];  // any context, as pick_context hands them out
        std::shared_lock<std::shared_mutex> rl(c.mu);
        std::lock_guard<std::mutex> g(x.work_mu);
        const uint64_t before = c.host_skips.load(std::memory_order_relaxed);
        SpecPlan p = spec_plan(x.seen, c.gen, c.q8_gen, k, c.advice, false, c.host_skips);
        if (p.spec_k != -1 && (p.spec_k < (int)k || p.spec_k >= (int)kSpecK)) bad = true;
        if (!p.seen) bad = true;
        if (p.spec_k < 0 && c.host_skips.load(std::memory_order_relaxed) > before)
          forced_skips.fetch_add(1, std::memory_order_relaxed);
        spec_seen_mark(p, k);
      }
    });
  std::thread device([&] {
    std::mt19937 rng(99);
    while (!stop.load(std::memory_order_relaxed)) {
      Coll& c = colls[rng() % kColls];
      const uint32_t k = rng() % kSpecK;
      if (rng() & 1)
        __atomic_store_n(&c.advice[k], rng() & 1u, __ATOMIC_RELAXED);
      else
        __atomic_store_n(&c.advice[kSpecK + k], rng() % 5u, __ATOMIC_RELAXED);
    }
  });
  std::thread writer([&] {
    std::mt19937 rng(7);
    while (!stop.load(std::memory_order_relaxed)) {
      Coll& c = colls[rng() % kColls];
      std::unique_lock<std::shared_mutex> wl(c.mu);
      c.q8_gen = next_gen.fetch_add(1);
      spec_advice_reset(c.advice);
      if (rng() % 8 == 0) c.gen = next_gen.fetch_add(1);  // dropped and recreated
    }
  });
  for (auto& x : th) x.join();
  stop = true;
  device.join();
  writer.join();
  uint64_t skips = 0;
  for (auto& c : colls) skips += c.host_skips.load();
  size_t maxmap = 0;
  for (auto& x : ctx) maxmap = x.seen.size() > maxmap ? x.seen.size() : maxmap;
  if (bad || maxmap > kSpecSeenMax + 1) {
    std::printf("FAIL bad=%d maxmap=%zu\n", (int)bad.load(), maxmap);
    return 1;
  }
  std::printf("ok %d contexts, %llu host skips (%llu seen by the planners), maps <= %zu\n", nctx,
              (unsigned long long)skips, (unsigned long long)forced_skips.load(), maxmap);
  return 0;
}
