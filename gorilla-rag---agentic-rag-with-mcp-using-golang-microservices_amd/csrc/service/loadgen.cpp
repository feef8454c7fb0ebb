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
//
// With "http":"host:port" the same bodies go over TCP as HTTP/1.1 POSTs
// (http.Post in retrieval-service, main.go:229-233) to a listener
// (vsvc_http_start, or any server with the reference's routes): each client
// keeps one keep-alive connection (Go's Transport reuses idle connections),
// or opens one per request with "keepalive":false; a keep-alive connection
// the server closed is re-dialled once.
#include <unistd.h>

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
#include "http.h"
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

// One client's HTTP/1.1 connection to the listener.
struct HttpClient {
  std::string host, host_hdr;
  int port = 0;
  bool keepalive = true;
  int fd = -1;
  std::string buf;

  ~HttpClient() { drop(); }
  void drop() {
    if (fd >= 0) ::close(fd);
    fd = -1;
    buf.clear();
  }
  // POST path body -> *r; false on a transport error (*err says which)
  bool post(const std::string& path, const std::string& body, vshttp::Response* r,
            std::string* err) {
    std::string req = "POST " + path + " HTTP/1.1\r\nHost: " + host_hdr +
                      "\r\nUser-Agent: vsvc-loadgen\r\nContent-Type: application/json\r\n"
                      "Content-Length: " + std::to_string(body.size()) + "\r\n";
    if (!keepalive) req += "Connection: close\r\n";
    req += "\r\n";
    req += body;
    for (int attempt = 0; attempt < 2; ++attempt) {
      const bool fresh = fd < 0;
      if (fresh) {
        fd = vshttp::connect_tcp(host, port);
        if (fd < 0) {
          *err = "connect failed";
          return false;
        }
      }
      if (!vshttp::send_all(fd, req.data(), req.size())) {
        drop();
        if (fresh) break;
        continue;  // a reused connection the server had closed
      }
      for (;;) {
        size_t used = 0;
        const vshttp::Frame f = vshttp::parse_response(buf.data(), buf.size(), r, &used);
        if (f == vshttp::Frame::kBad) {
          *err = "malformed response";
          drop();
          return false;
        }
        if (f == vshttp::Frame::kDone) {
          buf.erase(0, used);
          if (r->status >= 100 && r->status < 200) continue;  // 100 Continue
          if (!r->keep_alive || !keepalive) drop();
          return true;
        }
        if (!vshttp::recv_some(fd, &buf)) break;
      }
      const bool got_nothing = buf.empty();
      drop();
      if (fresh || !got_nothing) break;  // re-dial only an idle connection that was closed
    }
    *err = "connection closed";
    return false;
  }
};

}  // namespace

extern "C" int vsvc_loadgen(vsvc* svc, const char* spec_json, char** report) {
  if (!spec_json || !report) return VS_ERR_INVALID_ARG;
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
  // TCP mode: "http":"host:port"
  std::string http_host;
  int http_port = 0;
  const Json* hv = spec.get("http");
  const bool use_http = hv && hv->kind == Json::String;
  if (hv && !use_http && hv->kind != Json::Null) return VS_ERR_INVALID_ARG;
  if (use_http && !vshttp::split_addr(hv->str, &http_host, &http_port)) return VS_ERR_INVALID_ARG;
  if (!use_http && !svc) return VS_ERR_INVALID_ARG;
  const Json* kav = spec.get("keepalive");
  const bool keepalive = !(kav && kav->kind == Json::Bool && !kav->b);
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
      HttpClient hc;
      if (use_http) {
        hc.host = http_host.empty() ? std::string("127.0.0.1") : http_host;
        hc.port = http_port;
        hc.host_hdr = hc.host + ":" + std::to_string(http_port);
        hc.keepalive = keepalive;
      }
      vshttp::Response hr;
      std::string terr;
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
        int rc;
        if (use_http) {
          rc = hc.post("/search", body, &hr, &terr) ? VS_OK : VS_ERR_IO;
          status = rc == VS_OK ? hr.status : 0;
          resp = rc == VS_OK ? (char*)hr.body.data() : nullptr;
          n = rc == VS_OK ? hr.body.size() : 0;
        } else {
          rc = vsvc_handle(svc, "POST", "/search", body.data(), body.size(), &status, &resp, &n,
                           &ct);
        }
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
            first_error = rc != VS_OK && use_http
                              ? "transport: " + terr
                              : "status " + std::to_string(status) + ": " +
                                    (resp ? std::string(resp, std::min<size_t>(n, 300)) : "");
        }
        if (!use_http) vsvc_free(resp);
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
  o.obj.emplace_back("transport", Json::string(use_http ? "http" : "inproc"));
  std::string s;
  vsjson::encode(o, &s, false);
  *report = dup_str(s);
  return *report ? VS_OK : VS_ERR_OOM;
}
