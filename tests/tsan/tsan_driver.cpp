// ThreadSanitizer driver for the service layer (tests/test_tsan_service.py).
// Built with -fsanitize=thread together with csrc/service/*.cpp and the CPU
// test double tests/tsan/fake_engine.cpp; many threads call vsvc_handle at
// once (searches through the batcher, filtered searches through the filter
// cache, upserts that invalidate it, health / collection listings, malformed
// bodies), alongside vsvc_stats, vsvc_validate and a snapshot / restore of a
// second service. Exit status 0 and no TSAN report is the pass condition.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/vsearch_service.h"

namespace {

std::atomic<int> g_bad{0};

int call(vsvc* s, const char* method, const char* path, const std::string& body) {
  int status = 0;
  char* resp = nullptr;
  size_t len = 0;
  const char* ct = nullptr;
  const int rc = vsvc_handle(s, method, path, body.data(), body.size(), &status, &resp, &len, &ct);
  if (rc != VS_OK) g_bad++;
  vsvc_free(resp);
  return status;
}

std::string vec_json(std::mt19937& rng, int dim) {
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  std::string s = "[";
  for (int d = 0; d < dim; ++d) {
    char b[32];
    std::snprintf(b, sizeof b, "%s%.4f", d ? "," : "", u(rng));
    s += b;
  }
  return s + "]";
}

std::string uuid(int t, int i) {
  char b[40];
  std::snprintf(b, sizeof b, "%08x-0000-4000-8000-%012x", 0x1000 + t, i);
  return b;
}

}  // namespace

int main(int argc, char** argv) {
  const int threads = argc > 1 ? std::atoi(argv[1]) : 8;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 60;
  const char* snapdir = argc > 3 ? argv[3] : nullptr;
  const int dim = 16;
  vs_engine* eng = nullptr;
  if (vs_open(nullptr, &eng) != VS_OK) return 2;
  const char* cfg =
      "{\"collections\":[{\"name\":\"a\",\"dim\":16},{\"name\":\"b\",\"dim\":16,"
      "\"metric\":\"Dot\"}],\"batching\":{\"enabled\":true,\"max_batch\":16,"
      "\"max_wait_us\":200,\"workers\":2},\"filter\":\"match\"}";
  vsvc* svc = nullptr;
  if (vsvc_open(eng, cfg, &svc) != VS_OK) return 3;
  if (vsvc_bulk_generate(svc, "b", 500, 7) != VS_OK) return 4;

  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      std::mt19937 rng(1234 + t);
      for (int i = 0; i < iters; ++i) {
        const char* coll = (i + t) % 3 == 0 ? "b" : "a";
        switch ((i + t) % 6) {
          case 0: {  // upsert (invalidates the collection's filter cache)
            std::string body = std::string("{\"collection\":\"") + coll + "\",\"points\":[";
            for (int p = 0; p < 3; ++p)
              body += std::string(p ? "," : "") + "{\"id\":\"" + uuid(t, i * 3 + p) +
                      "\",\"vector\":" + vec_json(rng, dim) + ",\"payload\":{\"doc\":\"d" +
                      std::to_string(p) + "\",\"t\":" + std::to_string(t % 2) + "}}";
            body += "]}";
            if (call(svc, "POST", "/upsert", body) != 200) g_bad++;
            break;
          }
          case 1:
          case 2: {  // plain search (batched)
            const std::string body = std::string("{\"collection\":\"") + coll +
                                     "\",\"query\":" + vec_json(rng, dim) +
                                     ",\"top_k\":" + std::to_string(1 + i % 7) + "}";
            const int st = call(svc, "POST", "/search", body);
            if (st != 200) g_bad++;
            break;
          }
          case 3: {  // filtered search (filter cache + resident filters)
            const std::string body = std::string("{\"collection\":\"") + coll +
                                     "\",\"query\":" + vec_json(rng, dim) +
                                     ",\"top_k\":5,\"filter\":{\"t\":" + std::to_string(i % 2) +
                                     "}}";
            if (call(svc, "POST", "/search", body) != 200) g_bad++;
            break;
          }
          case 4:  // listings and health
            if (call(svc, "GET", "/health", "") != 200) g_bad++;
            if (call(svc, "GET", "/collections", "") != 200) g_bad++;
            break;
          default: {  // malformed requests and the engine-free helpers
            if (call(svc, "POST", "/search", "{\"query\":[1,2") != 400) g_bad++;
            if (call(svc, "GET", "/search", "") != 405) g_bad++;
            char* msg = nullptr;
            vsvc_validate("/search", "{\"top_k\":\"x\"}", 13, &msg);
            vsvc_free(msg);
            char* st = nullptr;
            if (vsvc_stats(svc, &st) == VS_OK) vsvc_free(st);
            break;
          }
        }
      }
    });
  for (auto& th : pool) th.join();

  // snapshot while searches run, then restore into a fresh service
  if (snapdir) {
    std::atomic<bool> stop{false};
    std::thread searcher([&] {
      std::mt19937 rng(99);
      while (!stop.load())
        call(svc, "POST", "/search",
             "{\"collection\":\"b\",\"query\":" + vec_json(rng, dim) + ",\"top_k\":3}");
    });
    const int rc = vsvc_snapshot(svc, snapdir);
    stop = true;
    searcher.join();
    if (rc != VS_OK) return 5;
    vs_engine* eng2 = nullptr;
    vsvc* svc2 = nullptr;
    if (vs_open(nullptr, &eng2) != VS_OK || vsvc_open(eng2, cfg, &svc2) != VS_OK) return 6;
    if (vsvc_restore(svc2, snapdir) != VS_OK) return 7;
    const std::string q1 = "[1,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0]";
    if (call(svc2, "POST", "/search", "{\"collection\":\"b\",\"query\":" + q1 + ",\"top_k\":3}") !=
        200)
      return 8;
    vsvc_close(svc2);
    vs_close(eng2);
  }
  // the HTTP listener under concurrent keep-alive and per-request connections,
  // with in-process searches beside it; stopped while idle connections remain
  {
    vsvc_http* http = nullptr;
    if (vsvc_http_start(svc, "127.0.0.1:0", &http) != VS_OK) return 10;
    const std::string addr = "127.0.0.1:" + std::to_string(vsvc_http_port(http));
    std::vector<std::thread> lg;
    std::atomic<int> lg_bad{0};
    for (int ka = 0; ka < 2; ++ka)
      lg.emplace_back([&, ka] {
        const std::string spec = "{\"collections\":[\"a\",\"b\"],\"dim\":" + std::to_string(dim) +
                                 ",\"clients\":6,\"seconds\":0.5,\"http\":\"" + addr +
                                 "\",\"keepalive\":" + (ka ? "true" : "false") + "}";
        char* rep = nullptr;
        if (vsvc_loadgen(nullptr, spec.c_str(), &rep) != VS_OK || !rep ||
            std::strstr(rep, "\"errors\":0,") == nullptr) {
          std::fprintf(stderr, "http loadgen: %s\n", rep ? rep : "(none)");
          lg_bad++;
        }
        vsvc_free(rep);
      });
    std::mt19937 rng(7);
    for (int i = 0; i < 50; ++i)
      if (call(svc, "POST", "/search",
               "{\"collection\":\"a\",\"query\":" + vec_json(rng, dim) + ",\"top_k\":4}") != 200)
        g_bad++;
    for (auto& t : lg) t.join();
    if (lg_bad.load()) return 11;
    vsvc_http_stop(http);
  }
  char* st = nullptr;
  if (vsvc_stats(svc, &st) == VS_OK) {
    std::printf("stats %s\n", st);
    vsvc_free(st);
  }
  vsvc_close(svc);
  vs_close(eng);
  if (g_bad.load()) {
    std::fprintf(stderr, "unexpected statuses: %d\n", g_bad.load());
    return 9;
  }
  std::printf("ok %d threads x %d iterations\n", threads, iters);
  return 0;
}
