// loadgen.cpp — closed-loop /search load generator (include/vsearch_service.h
// vsvc_loadgen).
//
// Each client thread plays rag/retrieval-service's searchVectorDB
// (rag/retrieval-service/main.go:219-276) in a loop: it posts the body that
// json.Marshal(map[string]interface{}{...}) builds there (keys sorted:
// collection, filter, query, top_k; a nil filters map encodes as null),
// checks the 200 status and that the reply decodes with a results array, and
// sends the next request at once. The bodies are pre-encoded (queries are
// random unit vectors, one pool per run, floats printed with 9 significant
// digits, which round-trip through Go's decimal -> float32 parse), so the
// loop measures the service: decode, batcher, engine, reply encode.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/vsearch_service.h"
#include "json.h"

using vsjson::Json;

namespace {

char* dup_str(const std::string& s) {
  char* p = (char*)std::malloc(s.size() + 1);
  if (p) std::memcpy(p, s.c_str(), s.size() + 1);
  return p;
}

double num_or(const Json& o, const char* key, double dflt) {
  const Json* v = o.get(key);
  return v && v->kind == Json::Number ? v->num : dflt;
}

}  // namespace

extern "C" int vsvc_loadgen(vsvc* svc, const char* spec_json, char** report) {
  if (!svc || !spec_json || !report) return VS_ERR_INVALID_ARG;
  *report = nullptr;
  Json spec;
  std::string perr;
  if (!vsjson::parse(spec_json, std::strlen(spec_json), &spec, &perr)) return VS_ERR_INVALID_ARG;
  const Json* cl = spec.get("collections");
  if (!cl || cl->kind != Json::Array || cl->arr.empty()) return VS_ERR_INVALID_ARG;
  std::vector<std::string> colls;
  for (const auto& c : cl->arr) {
    if (c.kind != Json::String) return VS_ERR_INVALID_ARG;
    colls.push_back(c.str);
  }
  const int dim = (int)num_or(spec, "dim", 0);
  const int clients = (int)num_or(spec, "clients", 16);
  const double seconds = num_or(spec, "seconds", 5.0);
  const int k_min = (int)num_or(spec, "k_min", 3), k_max = (int)num_or(spec, "k_max", 50);
  const int nqueries = (int)num_or(spec, "queries", 256);
  const uint64_t seed = (uint64_t)num_or(spec, "seed", 1);
  if (dim < 1 || dim > 65536 || clients < 1 || clients > 4096 || !(seconds > 0) ||
      seconds > 3600 || k_min < 1 || k_max < k_min || nqueries < 1 || nqueries > 1 << 16)
    return VS_ERR_INVALID_ARG;

  // body pool: one query string per pool entry, reused with varying k / collection
  std::vector<std::string> qtext(nqueries);
  {
    std::mt19937_64 rng(seed);
    std::normal_distribution<float> nd;
    std::vector<float> v(dim);
    char buf[32];
    for (auto& t : qtext) {
      double s = 0;
      for (auto& x : v) x = nd(rng), s += (double)x * x;
      const float inv = (float)(1.0 / std::sqrt(s > 0 ? s : 1.0));
      t.push_back('[');
      for (int d = 0; d < dim; ++d) {
        std::snprintf(buf, sizeof(buf), "%.9g", v[d] * inv);
        if (d) t.push_back(',');
        t.append(buf);
      }
      t.push_back(']');
    }
  }

  std::atomic<uint64_t> requests{0}, errors{0};
  std::mutex mu;
  std::string first_error;
  std::vector<std::vector<float>> lat(clients);
  const auto t0 = std::chrono::steady_clock::now();
  const auto deadline = t0 + std::chrono::duration_cast<std::chrono::steady_clock::duration>(
                                 std::chrono::duration<double>(seconds));
  std::vector<std::thread> th;
  for (int c = 0; c < clients; ++c) {
    th.emplace_back([&, c] {
      std::mt19937_64 rng(seed * 7919 + (uint64_t)c + 1);
      std::string body;
      auto& my = lat[c];
      while (std::chrono::steady_clock::now() < deadline) {
        const std::string& coll = colls[rng() % colls.size()];
        const int k = k_min + (int)(rng() % (uint64_t)(k_max - k_min + 1));
        body.clear();
        body.append("{\"collection\":");
        vsjson::encode_string(coll, &body);
        body.append(",\"filter\":null,\"query\":");
        body.append(qtext[rng() % qtext.size()]);
        body.append(",\"top_k\":");
        body.append(std::to_string(k));
        body.push_back('}');
        int status = 0;
        char* resp = nullptr;
        size_t n = 0;
        const char* ct = nullptr;
        const auto a = std::chrono::steady_clock::now();
        const int rc = vsvc_handle(svc, "POST", "/search", body.data(), body.size(), &status,
                                   &resp, &n, &ct);
        const auto b = std::chrono::steady_clock::now();
        bool ok = rc == VS_OK && status == 200 && resp;
        if (ok) {  // the caller decodes results[] (main.go:244-257)
          Json r;
          std::string e;
          const Json* res = nullptr;
          ok = vsjson::parse(resp, n, &r, &e) && (res = r.get("results")) &&
               res->kind == Json::Array && (int)res->arr.size() <= k;
        }
        if (!ok) {
          errors.fetch_add(1);
          std::lock_guard<std::mutex> g(mu);
          if (first_error.empty())
            first_error = "status " + std::to_string(status) + ": " +
                          (resp ? std::string(resp, std::min<size_t>(n, 300)) : "");
        }
        vsvc_free(resp);
        requests.fetch_add(1);
        my.push_back(std::chrono::duration<float, std::milli>(b - a).count());
      }
    });
  }
  for (auto& t : th) t.join();
  const double el =
      std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::vector<float> all;
  for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) -> double {
    if (all.empty()) return 0.0;
    size_t i = (size_t)std::ceil(p * all.size()) - 1;
    return all[std::min(i, all.size() - 1)];
  };
  Json o = Json::object();
  o.obj.emplace_back("requests", Json::number((double)requests.load()));
  o.obj.emplace_back("errors", Json::number((double)errors.load()));
  o.obj.emplace_back("seconds", Json::number(el));
  o.obj.emplace_back("qps", Json::number(requests.load() / el));
  Json l = Json::object();
  l.obj.emplace_back("p50", Json::number(pct(0.50)));
  l.obj.emplace_back("p90", Json::number(pct(0.90)));
  l.obj.emplace_back("p99", Json::number(pct(0.99)));
  l.obj.emplace_back("max", Json::number(all.empty() ? 0.0 : all.back()));
  o.obj.emplace_back("lat_ms", std::move(l));
  o.obj.emplace_back("first_error", Json::string(first_error));
  std::string s;
  vsjson::encode(o, &s, false);
  *report = dup_str(s);
  return *report ? VS_OK : VS_ERR_OOM;
}
