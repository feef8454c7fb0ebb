// server_main.cpp — vsearch_server: the vector-service process for hosts
// without a Go toolchain. The reference's main (rag/vector-service/main.go:
// 53-78) dials Qdrant, creates the three collections and serves four routes
// on :PORT; this binary opens the HIP engine instead of the gRPC client, opens
// the handler mirror over it (vsvc_open: the same collections) and serves the
// same routes on the same port through vsvc_http_start.
//
// Environment (the reference's getEnv idiom, main.go:393-398):
//   PORT               listen port, default 8082 (main.go:75)
//   VS_DEVICES         "0" (default) or a comma list "0,1,...,7": one engine
//                      row-striping every collection over those devices
//                      (vs_open_multi; RCCL all-gather of the per-device top-k)
//   VS_PLACEMENT       "stripes" (default: every collection row-striped over
//                      VS_DEVICES) or "collections" (each collection whole on
//                      one device, calls for different collections concurrent,
//                      no collective: VS_FLAG_PLACE_COLLECTIONS)
//   VS_SERVICE_CONFIG  path of a vsvc_open config JSON (collections, batching,
//                      filter mode); unset = the reference's defaults
//   VS_DATA_DIR        restore every collection snapshotted there at start,
//                      snapshot all of them there on SIGINT / SIGTERM (what
//                      Qdrant's storage volume gives the reference,
//                      docker-compose.yml); VS_SNAPSHOT_DIR is an alias (the
//                      Go service's name, go/vector-service/main.go)
//   VS_BULK            "coll=rows[:seed],..." synthetic bulk rows per
//                      collection at start (benchmark corpora, vsvc_bulk_generate)
// Prints "Vector Service starting on port <PORT>" (main.go:76) once listening.
#include <signal.h>
#include <sys/stat.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../../include/vsearch_service.h"

namespace {

std::string get_env(const char* key, const char* dflt) {
  const char* v = std::getenv(key);
  return v && *v ? std::string(v) : std::string(dflt);
}

int fail(const char* what, int rc) {
  std::fprintf(stderr, "vsearch_server: %s failed: %d %s\n", what, rc, vs_last_error());
  return 1;
}

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::stringstream ss(s);
  std::string item;
  while (std::getline(ss, item, sep))
    if (!item.empty()) out.push_back(item);
  return out;
}

}  // namespace

int main() {
  // SIGINT / SIGTERM are taken by sigwait below, blocked before any thread starts
  sigset_t sigs;
  sigemptyset(&sigs);
  sigaddset(&sigs, SIGINT);
  sigaddset(&sigs, SIGTERM);
  pthread_sigmask(SIG_BLOCK, &sigs, nullptr);

  const std::string port = get_env("PORT", "8082");
  std::vector<int32_t> devs;
  for (const std::string& d : split(get_env("VS_DEVICES", "0"), ',')) devs.push_back(std::atoi(d.c_str()));
  if (devs.empty()) devs.push_back(0);

  vs_engine* eng = nullptr;
  int rc;
  if (devs.size() == 1) {
    vs_config cfg = {devs[0], 0u};
    rc = vs_open(&cfg, &eng);
  } else {
    const std::string placement = get_env("VS_PLACEMENT", "stripes");
    if (placement != "stripes" && placement != "collections") {
      std::fprintf(stderr, "vsearch_server: VS_PLACEMENT must be stripes or collections\n");
      return 1;
    }
    vs_config_multi cfg = {devs.data(), (uint32_t)devs.size(),
                           placement == "collections" ? VS_FLAG_PLACE_COLLECTIONS : 0u};
    rc = vs_open_multi(&cfg, &eng);
  }
  if (rc != VS_OK) return fail("vs_open", rc);

  std::string config;
  const std::string cpath = get_env("VS_SERVICE_CONFIG", "");
  if (!cpath.empty()) {
    std::ifstream f(cpath);
    if (!f) {
      std::fprintf(stderr, "vsearch_server: cannot read %s\n", cpath.c_str());
      return 1;
    }
    std::stringstream ss;
    ss << f.rdbuf();
    config = ss.str();
  }
  vsvc* svc = nullptr;
  rc = vsvc_open(eng, config.empty() ? nullptr : config.c_str(), &svc);
  if (rc != VS_OK) return fail("vsvc_open", rc);

  // VS_SNAPSHOT_DIR is the Go service's name for it (go/vector-service/main.go)
  const std::string data_dir = get_env("VS_DATA_DIR", get_env("VS_SNAPSHOT_DIR", "").c_str());
  if (!data_dir.empty()) {
    ::mkdir(data_dir.c_str(), 0755);
    rc = vsvc_restore(svc, data_dir.c_str());
    if (rc != VS_OK) std::fprintf(stderr, "vsearch_server: restore from %s: %d %s\n",
                                  data_dir.c_str(), rc, vs_last_error());
  }
  for (const std::string& spec : split(get_env("VS_BULK", ""), ',')) {
    const size_t eq = spec.find('=');
    if (eq == std::string::npos) {
      std::fprintf(stderr, "vsearch_server: bad VS_BULK entry %s\n", spec.c_str());
      return 1;
    }
    const std::string coll = spec.substr(0, eq);
    const std::vector<std::string> nv = split(spec.substr(eq + 1), ':');
    const uint64_t n = nv.empty() ? 0 : std::strtoull(nv[0].c_str(), nullptr, 10);
    const uint64_t seed = nv.size() > 1 ? std::strtoull(nv[1].c_str(), nullptr, 10) : 1;
    rc = vsvc_bulk_generate(svc, coll.c_str(), n, seed);
    if (rc != VS_OK) return fail("vsvc_bulk_generate", rc);
  }

  vsvc_http* http = nullptr;
  rc = vsvc_http_start(svc, (":" + port).c_str(), &http);
  if (rc != VS_OK) return fail("listen", rc);
  std::printf("Vector Service starting on port %d\n", vsvc_http_port(http));
  std::fflush(stdout);

  int sig = 0;
  sigwait(&sigs, &sig);
  std::printf("signal %d: shutting down\n", sig);
  vsvc_http_stop(http);
  if (!data_dir.empty()) {
    rc = vsvc_snapshot(svc, data_dir.c_str());
    if (rc != VS_OK) std::fprintf(stderr, "vsearch_server: snapshot to %s: %d %s\n",
                                  data_dir.c_str(), rc, vs_last_error());
  }
  vsvc_close(svc);
  vs_close(eng);
  std::fflush(stdout);
  return rc == VS_OK ? 0 : 1;
}
