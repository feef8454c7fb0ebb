// concurrency_probe.cpp: what two host threads calling vs_search at once
// gain over one, by engine kind and collection size. No
// Python in the process (no GIL): per config, T threads each make N calls
// of one query (k = 10) or a 16-query batch; one JSON line with the wall
// time per call of 1 thread and per call-pair of 2 threads.
//
//   g++ -O2 -std=c++17 -Iinclude -o tools/concurrency_probe tools/concurrency_probe.cpp \
//     -L<pkg>/lib -lvsearch -Wl,-rpath,<pkg>/lib -pthread
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "vsearch.h"

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int run(vs_engine* eng, const char* coll, uint32_t dim, uint32_t nq, int threads, int calls,
               double* sec) {
  std::vector<std::thread> th;
  std::vector<int> rcs(threads, 0);
  const double t0 = now_s();
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t] {
      std::vector<float> q((size_t)nq * dim), s((size_t)nq * 10);
      std::vector<uint64_t> r((size_t)nq * 10);
      std::vector<uint32_t> c(nq);
      for (size_t i = 0; i < q.size(); ++i) q[i] = (float)((i * 2654435761u + t) % 1000) / 1000.f - 0.5f;
      for (int i = 0; i < calls && !rcs[t]; ++i)
        rcs[t] = vs_search(eng, coll, q.data(), nq, dim, 10, s.data(), r.data(), c.data());
    });
  for (auto& x : th) x.join();
  *sec = now_s() - t0;
  for (int rc : rcs)
    if (rc) return rc;
  return 0;
}

int main(int argc, char** argv) {
  const int calls = argc > 1 ? std::atoi(argv[1]) : 400;
  const uint32_t dim = 256;
  struct Eng {
    const char* name;
    std::vector<int32_t> devs;
  };
  for (const Eng& e : {Eng{"single", {0}}, Eng{"shards_0_0", {0, 0}}, Eng{"shards_0_0_0_0", {0, 0, 0, 0}}}) {
    vs_engine* eng = nullptr;
    int rc;
    if (e.devs.size() == 1) {
      vs_config cfg = {e.devs[0], 0u};
      rc = vs_open(&cfg, &eng);
    } else {
      vs_config_multi cfg = {e.devs.data(), (uint32_t)e.devs.size(), 0u};
      rc = vs_open_multi(&cfg, &eng);
    }
    if (rc) {
      std::fprintf(stderr, "open %s: %s\n", e.name, vs_last_error());
      return 1;
    }
    for (uint64_t rows : {20000ull, 200000ull, 2000000ull}) {
      const std::string coll = "c" + std::to_string(rows);
      if (vs_collection_create(eng, coll.c_str(), dim, VS_METRIC_DOT, VS_DTYPE_BF16, rows, 0) ||
          vs_generate(eng, coll.c_str(), rows, 7)) {
        std::fprintf(stderr, "create: %s\n", vs_last_error());
        return 1;
      }
      for (uint32_t nq : {1u, 16u}) {
        double w, s1, s2;
        run(eng, coll.c_str(), dim, nq, 1, 30, &w);  // warm
        if (run(eng, coll.c_str(), dim, nq, 1, calls, &s1) ||
            run(eng, coll.c_str(), dim, nq, 2, calls, &s2)) {
          std::fprintf(stderr, "search: %s\n", vs_last_error());
          return 1;
        }
        std::printf("{\"engine\": \"%s\", \"rows\": %llu, \"dim\": %u, \"nq\": %u, "
                    "\"one_thread_us_per_call\": %.1f, \"two_threads_us_per_pair\": %.1f, "
                    "\"ratio\": %.3f, \"spin_us\": \"%s\"}\n",
                    e.name, (unsigned long long)rows, dim, nq, s1 / calls * 1e6, s2 / calls * 1e6,
                    s2 / s1, std::getenv("VS_SPIN_US") ? std::getenv("VS_SPIN_US") : "60");
        std::fflush(stdout);
      }
      vs_collection_drop(eng, coll.c_str());
    }
    vs_close(eng);
  }
  return 0;
}
