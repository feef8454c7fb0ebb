// vector_service.cpp — rag/vector-service's handlers restated over the
// engine C-ABI (see include/vsearch_service.h for the route map).
//
// Each handler follows the Go function line by line in behaviour: the same
// decode step (json.NewDecoder(r.Body).Decode into the request struct), the
// same validation order and messages, the same response structs. Where the
// reference forwards to Qdrant, the engine is called instead and Qdrant's
// gRPC error shape ("rpc error: code = ... desc = ...") is kept in the
// messages, as the Go service surfaces err.Error() verbatim.
#include <algorithm>
#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../../include/vsearch_service.h"
#include "batcher.h"
#include "json.h"

using vsjson::Json;

namespace {

struct CollState {
  std::string name;
  uint32_t dim = 0;
  std::shared_mutex mu;                              // upsert = writer, search = reader
  // Rows [0, bulk) came from vsvc_bulk_generate: their UUIDs are synthetic
  // and invertible (bulk_uuid / bulk_row), so no per-row host state exists
  // for them; a payload upserted onto one lands in bulk_payload.
  uint64_t bulk = 0, bulk_tag = 0;
  std::unordered_map<uint64_t, Json> bulk_payload;
  std::unordered_map<std::string, uint64_t> row_of;  // canonical UUID -> row (>= bulk)
  std::vector<std::string> uuid_of;                  // row - bulk -> UUID
  std::vector<Json> payload_of;                      // row - bulk -> payload (a decoded map)

  uint64_t nrows() const { return bulk + uuid_of.size(); }

  // filter pre-masks (filter mode "match"), cached per canonical filter text
  // and invalidated by any upsert (version); each also lives on the device
  // (vs_filter_create) so a repeated filter ships no bitmap per search
  uint64_t version = 0;
  std::mutex fmu;
  struct FilterEntry {
    uint64_t version = 0;
    std::shared_ptr<std::vector<uint64_t>> mask;
    uint64_t device_id = 0;  // 0: not resident (the mask is sent per call)
  };
  std::unordered_map<std::string, FilterEntry> fcache;
};

// Synthetic UUID of bulk row r: version 4, variant 10, the collection's
// 48-bit tag in the first 12 hex digits and r in the last 62 bits.
std::string bulk_uuid(uint64_t tag, uint64_t r) {
  const uint64_t hi = (tag << 16) | 0x4000u, lo = 0x8000000000000000ull | r;
  char b[40];
  std::snprintf(b, sizeof(b), "%08x-%04x-%04x-%04x-%012llx", (unsigned)(hi >> 32),
                (unsigned)((hi >> 16) & 0xFFFF), (unsigned)(hi & 0xFFFF), (unsigned)(lo >> 48),
                (unsigned long long)(lo & 0xFFFFFFFFFFFFull));
  return b;
}

// Inverse of bulk_uuid on a canonical UUID; false if it is not one of cs's.
bool bulk_row(const CollState& cs, const std::string& canon, uint64_t* row) {
  if (!cs.bulk || canon.size() != 36) return false;
  uint64_t hi = 0, lo = 0;
  int nd = 0;
  for (char ch : canon) {
    if (ch == '-') continue;
    const int v = ch >= '0' && ch <= '9' ? ch - '0' : (ch >= 'a' && ch <= 'f' ? ch - 'a' + 10 : -1);
    if (v < 0) return false;
    uint64_t& w = nd < 16 ? hi : lo;
    w = (w << 4) | (uint64_t)v;
    ++nd;
  }
  if (nd != 32 || hi != ((cs.bulk_tag << 16) | 0x4000u) || (lo >> 62) != 2) return false;
  const uint64_t r = lo & 0x3FFFFFFFFFFFFFFFull;
  if (r >= cs.bulk) return false;
  *row = r;
  return true;
}

std::string uuid_at(const CollState& cs, uint64_t row) {
  if (row < cs.bulk) return bulk_uuid(cs.bulk_tag, row);
  return row < cs.nrows() ? cs.uuid_of[row - cs.bulk] : std::string();
}

const Json& payload_at(const CollState& cs, uint64_t row) {
  static const Json kEmpty = Json::object();
  if (row < cs.bulk) {
    auto it = cs.bulk_payload.find(row);
    return it == cs.bulk_payload.end() ? kEmpty : it->second;
  }
  return row < cs.nrows() ? cs.payload_of[row - cs.bulk] : kEmpty;
}

struct Response {
  int status = 200;
  std::string body;
  const char* type = "application/json";
};

const char* kJsonType = "application/json";
const char* kTextType = "text/plain; charset=utf-8";

// respondError (main.go:388-392)
Response error_json(const std::string& msg, int status) {
  Json o = Json::object();
  o.obj.emplace_back("error", Json::string(msg));
  Response r;
  r.status = status;
  vsjson::encode(o, &r.body);
  r.body.push_back('\n');
  return r;
}

// http.Error(w, msg, code)
Response error_text(const std::string& msg, int status) {
  Response r;
  r.status = status;
  r.type = kTextType;
  r.body = msg + "\n";
  return r;
}

std::string last_error() { return vs_last_error(); }

std::string grpc_error(int rc, const std::string& msg) {
  const char* code = rc == VS_ERR_NOT_FOUND ? "NotFound"
                     : (rc == VS_ERR_INVALID_ARG || rc == VS_ERR_DIM_MISMATCH) ? "InvalidArgument"
                     : rc == VS_ERR_OOM ? "ResourceExhausted"
                                        : "Internal";
  return std::string("rpc error: code = ") + code + " desc = " + msg;
}

std::string not_found(const std::string& coll) {
  return grpc_error(VS_ERR_NOT_FOUND, "Not found: Collection `" + coll + "` doesn't exist!");
}

std::string dim_error(uint32_t want, size_t got) {
  return grpc_error(VS_ERR_DIM_MISMATCH, "Wrong input: Vector dimension error: expected dim: " +
                                             std::to_string(want) + ", got " + std::to_string(got));
}

// Uuid::parse_str (upstream Qdrant, rust `uuid` crate): simple, hyphenated,
// braced or urn forms, any hex case; canonical form is lowercase hyphenated.
bool canonical_uuid(const std::string& in, std::string* out) {
  std::string s = in;
  if (s.size() == 45 && s.compare(0, 9, "urn:uuid:") == 0) s = s.substr(9);
  if (s.size() == 38 && s.front() == '{' && s.back() == '}') s = s.substr(1, 36);
  std::string hex;
  if (s.size() == 36) {
    for (size_t i = 0; i < 36; ++i) {
      bool dash = (i == 8 || i == 13 || i == 18 || i == 23);
      if (dash) {
        if (s[i] != '-') return false;
      } else {
        hex.push_back(s[i]);
      }
    }
  } else if (s.size() == 32) {
    hex = s;
  } else {
    return false;
  }
  for (char& c : hex) {
    if (c >= 'A' && c <= 'F') c = (char)(c - 'A' + 'a');
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f'))) return false;
  }
  *out = hex.substr(0, 8) + "-" + hex.substr(8, 4) + "-" + hex.substr(12, 4) + "-" +
         hex.substr(16, 4) + "-" + hex.substr(20, 12);
  return true;
}

// Go decodes numbers inside interface{} values with ParseFloat(s, 64): a
// literal beyond float64's range is an UnmarshalTypeError.
bool interface_numbers_ok(const Json& v) {
  switch (v.kind) {
    case Json::Number: return std::abs(v.num) <= 1.7976931348623157e308;
    case Json::Array:
      for (const auto& e : v.arr)
        if (!interface_numbers_ok(e)) return false;
      return true;
    case Json::Object:
      for (const auto& e : v.obj)
        if (!interface_numbers_ok(e.second)) return false;
      return true;
    default: return true;
  }
}

// ---- request decoding (json.Decoder.Decode into the Go structs) -------------
struct SearchRequest {  // main.go:26-31
  std::string collection;
  std::vector<float> query;
  int64_t top_k = 0;
  Json filter;  // Filter map[string]interface{}: decoded; the reference never uses it
};

// A JSON number literal at b[i..) (the grammar json.Decoder accepts):
// -?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)?. Returns its end, or 0 when
// there is none; *integer is whether it has neither fraction nor exponent.
size_t json_number_end(const char* b, size_t n, size_t i, bool* integer) {
  auto digit = [&](size_t j) { return j < n && b[j] >= '0' && b[j] <= '9'; };
  *integer = true;
  if (i < n && b[i] == '-') ++i;
  if (!digit(i)) return 0;
  if (b[i] == '0') ++i;
  else
    while (digit(i)) ++i;
  if (i < n && b[i] == '.') {
    *integer = false;
    if (!digit(++i)) return 0;
    while (digit(i)) ++i;
  }
  if (i < n && (b[i] == 'e' || b[i] == 'E')) {
    *integer = false;
    ++i;
    if (i < n && (b[i] == '+' || b[i] == '-')) ++i;
    if (!digit(i)) return 0;
    while (digit(i)) ++i;
  }
  return i;
}

// Fast path for the body retrieval-service sends (main.go:221-226): one
// object whose keys are exactly "collection", "query", "top_k" and "filter",
// each at most once, in any order; collection a string of printable ASCII
// without escapes, query an array of numbers, top_k an integer literal,
// filter null. The query's float32s come straight from the literals
// (from_chars: the correctly rounded float32, as Go's ParseFloat(s, 32)),
// with no JSON tree. Anything else -- other keys, case-folded keys,
// duplicates, escapes, nulls inside the query, a filter object, a number out
// of range, a syntax error -- returns false and the generic decoder below
// answers it (with Go's semantics and errors). A 768-number body decodes
// ~3x faster this way. Trailing bytes after the object are ignored, as
// json.Decoder.Decode ignores them.
bool decode_search_fast(const char* b, size_t n, SearchRequest* req) {
  size_t i = 0;
  auto ws = [&] {
    while (i < n && (b[i] == ' ' || b[i] == '\t' || b[i] == '\n' || b[i] == '\r')) ++i;
  };
  ws();
  if (i >= n || b[i] != '{') return false;
  ++i;
  bool seen_c = false, seen_q = false, seen_k = false, seen_f = false;
  for (;;) {
    ws();
    if (i >= n || b[i] != '"') return false;  // also the empty object: generic path
    const size_t ks = ++i;
    while (i < n && b[i] != '"' && b[i] != '\\') ++i;
    if (i >= n || b[i] != '"') return false;
    const std::string key(b + ks, i - ks);
    ++i;
    ws();
    if (i >= n || b[i] != ':') return false;
    ++i;
    ws();
    if (i >= n) return false;
    if (key == "collection") {
      if (seen_c || b[i] != '"') return false;
      seen_c = true;
      const size_t s0 = ++i;
      while (i < n && b[i] != '"' && b[i] != '\\' && (unsigned char)b[i] >= 0x20 &&
             (unsigned char)b[i] < 0x80)
        ++i;
      if (i >= n || b[i] != '"') return false;
      req->collection.assign(b + s0, i - s0);
      ++i;
    } else if (key == "query") {
      if (seen_q || b[i] != '[') return false;
      seen_q = true;
      ++i;
      req->query.clear();
      ws();
      if (i < n && b[i] == ']') {
        ++i;
      } else {
        for (;;) {
          ws();
          bool integer;
          const size_t e = json_number_end(b, n, i, &integer);
          if (!e) return false;
          float f;
          const auto r = std::from_chars(b + i, b + e, f);
          if (r.ec != std::errc() || r.ptr != b + e) return false;  // out of range: generic
          req->query.push_back(f);
          i = e;
          ws();
          if (i < n && b[i] == ',') {
            ++i;
            continue;
          }
          if (i < n && b[i] == ']') {
            ++i;
            break;
          }
          return false;
        }
      }
    } else if (key == "top_k") {
      if (seen_k) return false;
      seen_k = true;
      bool integer;
      const size_t e = json_number_end(b, n, i, &integer);
      if (!e || !integer) return false;
      int64_t v;
      const auto r = std::from_chars(b + i, b + e, v);
      if (r.ec != std::errc() || r.ptr != b + e) return false;
      req->top_k = v;
      i = e;
    } else if (key == "filter") {
      if (seen_f || n - i < 4 || std::memcmp(b + i, "null", 4) != 0) return false;
      seen_f = true;
      i += 4;
    } else {
      return false;
    }
    ws();
    if (i < n && b[i] == ',') {
      ++i;
      continue;
    }
    if (i < n && b[i] == '}') return true;
    return false;
  }
}

// The generic decode (a JSON tree, then Go's field rules). Returns "" on
// success, else the decode error.
std::string decode_search_generic(const char* body, size_t len, SearchRequest* req) {
  Json root;
  std::string err;
  if (!vsjson::parse(body, len, &root, &err)) return err;
  if (root.kind == Json::Null) return "";
  if (root.kind != Json::Object) return "cannot unmarshal into SearchRequest";
  std::string first;
  if (const Json* c = root.field("collection")) {
    if (c->kind == Json::String) req->collection = c->str;
    else if (c->kind != Json::Null && first.empty()) first = "collection: not a string";
  }
  if (const Json* q = root.field("query")) {
    if (q->kind == Json::Array) {
      req->query.assign(q->arr.size(), 0.0f);
      for (size_t i = 0; i < q->arr.size(); ++i) {
        const Json& e = q->arr[i];
        if (e.kind == Json::Number) {
          float f;
          if (!vsjson::parse_float32(e.str, &f)) {
            if (first.empty()) first = "cannot unmarshal number " + e.str + " into float32";
          } else {
            req->query[i] = f;
          }
        } else if (e.kind != Json::Null && first.empty()) {
          first = "query: non-numeric element";
        }
      }
    } else if (q->kind == Json::Null) {
      req->query.clear();
    } else if (first.empty()) {
      first = "query: not an array";
    }
  }
  if (const Json* k = root.field("top_k")) {
    if (k->kind == Json::Number) {
      int64_t v;
      if (!vsjson::parse_int64(k->str, &v)) {
        if (first.empty()) first = "cannot unmarshal number " + k->str + " into int";
      } else {
        req->top_k = v;
      }
    } else if (k->kind != Json::Null && first.empty()) {
      first = "top_k: not a number";
    }
  }
  if (const Json* f = root.field("filter")) {
    if (f->kind == Json::Object) {
      if (!interface_numbers_ok(*f) && first.empty()) first = "filter: number out of range";
      req->filter = *f;
    } else if (f->kind != Json::Null && first.empty()) {
      first = "filter: not an object";
    }
  }
  return first;
}

// Returns "" on success, else the decode error.
std::string decode_search(const char* body, size_t len, SearchRequest* req) {
  {
    SearchRequest fast;
    if (decode_search_fast(body, len, &fast)) {
      *req = std::move(fast);
      return "";
    }
  }
  return decode_search_generic(body, len, req);
}

struct UpsertRequest {  // main.go:21-24
  std::string collection;
  std::vector<const Json*> points;  // nullptr = a JSON null point (nil map)
  Json root;
};

std::string decode_upsert(const char* body, size_t len, UpsertRequest* req) {
  std::string err;
  if (!vsjson::parse(body, len, &req->root, &err)) return err;
  const Json& root = req->root;
  if (root.kind == Json::Null) return "";
  if (root.kind != Json::Object) return "cannot unmarshal into UpsertRequest";
  std::string first;
  if (const Json* c = root.field("collection")) {
    if (c->kind == Json::String) req->collection = c->str;
    else if (c->kind != Json::Null && first.empty()) first = "collection: not a string";
  }
  if (const Json* p = root.field("points")) {
    if (p->kind == Json::Array) {
      for (const auto& e : p->arr) {
        if (e.kind == Json::Object) {
          if (!interface_numbers_ok(e) && first.empty()) first = "point: number out of range";
          req->points.push_back(&e);
        } else if (e.kind == Json::Null) {
          req->points.push_back(nullptr);
        } else if (first.empty()) {
          first = "points: element is not an object";
        }
      }
    } else if (p->kind != Json::Null && first.empty()) {
      first = "points: not an array";
    }
  }
  return first;
}

// convertVector (main.go:343-375) for a decoded interface{}
bool convert_vector(const Json& v, std::vector<float>* out, std::string* err) {
  if (v.kind != Json::Array) {
    *err = "point vector must be an array";
    return false;
  }
  out->resize(v.arr.size());
  for (size_t i = 0; i < v.arr.size(); ++i) {
    if (v.arr[i].kind != Json::Number) {
      *err = "vector contains non-numeric value";
      return false;
    }
    (*out)[i] = (float)v.arr[i].num;  // float32(num): float64 -> float32, round to nearest even
  }
  return true;
}

}  // namespace

struct vsvc {
  vs_engine* eng = nullptr;
  std::vector<std::string> listed;  // the /collections reply (hard-coded in the reference)
  std::mutex mu;
  std::unordered_map<std::string, std::shared_ptr<CollState>> colls;
  vsbatch::Options batch_opt;
  std::unique_ptr<vsbatch::Batcher> batcher;  // coalesces concurrent /search (batcher.h)
  bool filter_match = false;  // "filter":"match": apply SearchRequest.Filter (f-4)

  std::shared_ptr<CollState> find(const std::string& name) {
    std::lock_guard<std::mutex> g(mu);
    auto it = colls.find(name);
    return it == colls.end() ? nullptr : it->second;
  }
};

namespace {

// healthHandler (main.go:121-136)
Response handle_health(vsvc* svc) {
  char buf[1024];
  int rc = vs_health(svc->eng, buf, sizeof(buf));
  Json o = Json::object();
  Json eng_info;
  std::string perr;
  bool parsed = vsjson::parse(buf, std::strlen(buf), &eng_info, &perr);
  std::string status = "healthy";
  if (rc != VS_OK) {
    status = "degraded";
    o.obj.emplace_back("error", Json::string(last_error()));
  } else if (parsed) {
    const Json* dn = eng_info.get("device_name");
    o.obj.emplace_back("engine", Json::string(std::string("vsearch-hip") +
                                              (dn ? " " + dn->str : std::string())));
  }
  o.obj.emplace_back("service", Json::string("vector-service"));
  o.obj.emplace_back("status", Json::string(status));
  Response r;
  vsjson::encode(o, &r.body);  // map[string]string: keys sorted
  r.body.push_back('\n');
  return r;
}

// collectionsHandler (main.go:138-147)
Response handle_collections(vsvc* svc, const std::string& method) {
  if (method != "GET") return error_text("Method not allowed", 405);
  Json arr = Json::array();
  for (const auto& n : svc->listed) arr.arr.push_back(Json::string(n));
  Json o = Json::object();
  o.obj.emplace_back("collections", std::move(arr));
  Response r;
  vsjson::encode(o, &r.body);
  r.body.push_back('\n');
  return r;
}

// upsertHandler (main.go:149-225)
Response handle_upsert(vsvc* svc, const std::string& method, const char* body, size_t len) {
  if (method != "POST") return error_text("Method not allowed", 405);
  UpsertRequest req;
  if (!decode_upsert(body, len, &req).empty()) return error_json("Invalid request body", 400);
  if (req.collection.empty()) return error_json("Collection name required", 400);

  const size_t n = req.points.size();
  std::vector<std::string> ids(n);
  std::vector<std::vector<float>> vecs(n);
  std::vector<Json> payloads(n, Json::object());
  for (size_t i = 0; i < n; ++i) {
    const Json* p = req.points[i];
    const Json* id = p ? p->get("id") : nullptr;
    if (!id || id->kind != Json::String) return error_json("Point ID must be a string", 400);
    ids[i] = id->str;
    const Json* v = p->get("vector");
    if (!v) return error_json("Point vector must be provided", 400);
    std::string err;
    if (!convert_vector(*v, &vecs[i], &err)) return error_json(err, 400);
    if (const Json* pl = p->get("payload"))
      if (pl->kind == Json::Object) payloads[i] = *pl;
  }

  // --- Points.Upsert(wait=true) ---
  auto cs = svc->find(req.collection);
  if (!cs) return error_json("Failed to upsert: " + not_found(req.collection), 500);
  std::vector<std::string> canon(n);
  for (size_t i = 0; i < n; ++i)
    if (!canonical_uuid(ids[i], &canon[i]))
      return error_json("Failed to upsert: " +
                            grpc_error(VS_ERR_INVALID_ARG, "Unable to parse UUID: " + ids[i]),
                        500);
  for (size_t i = 0; i < n; ++i)
    if (vecs[i].size() != cs->dim)
      return error_json("Failed to upsert: " + dim_error(cs->dim, vecs[i].size()), 500);

  std::unique_lock<std::shared_mutex> wl(cs->mu);
  const uint64_t base = cs->nrows();
  std::unordered_map<std::string, uint64_t> fresh;  // new UUIDs of this batch
  std::vector<uint64_t> rows(n);
  for (size_t i = 0; i < n; ++i) {
    auto it = cs->row_of.find(canon[i]);
    if (bulk_row(*cs, canon[i], &rows[i])) {
      // a bulk-generated point, overwritten by its id
    } else if (it != cs->row_of.end()) {
      rows[i] = it->second;
    } else {
      auto f = fresh.find(canon[i]);
      if (f != fresh.end()) {
        rows[i] = f->second;
      } else {
        rows[i] = base + fresh.size();
        fresh.emplace(canon[i], rows[i]);
      }
    }
  }
  if (n) {
    std::vector<float> flat(n * (size_t)cs->dim);
    for (size_t i = 0; i < n; ++i)
      std::memcpy(&flat[i * cs->dim], vecs[i].data(), (size_t)cs->dim * 4);
    int rc = vs_upsert(svc->eng, req.collection.c_str(), n, cs->dim, rows.data(), flat.data());
    if (rc != VS_OK) return error_json("Failed to upsert: " + grpc_error(rc, last_error()), 500);
  }
  cs->uuid_of.resize(base + fresh.size() - cs->bulk);
  cs->payload_of.resize(base + fresh.size() - cs->bulk);
  for (size_t i = 0; i < n; ++i) {  // in request order: the last duplicate wins
    if (rows[i] < cs->bulk) {
      cs->bulk_payload[rows[i]] = payloads[i];
      continue;
    }
    cs->row_of[canon[i]] = rows[i];
    cs->uuid_of[rows[i] - cs->bulk] = canon[i];
    cs->payload_of[rows[i] - cs->bulk] = payloads[i];
  }
  ++cs->version;  // cached filter masks are stale
  wl.unlock();

  Json o = Json::object();
  o.obj.emplace_back("status", Json::string("success"));
  o.obj.emplace_back("collection", Json::string(req.collection));
  o.obj.emplace_back("points", Json::number((double)n));
  Response r;
  vsjson::encode(o, &r.body);  // map[string]interface{}: keys sorted
  r.body.push_back('\n');
  return r;
}

// searchHandler (main.go:227-278)
// JSON value equality as Go's reflect.DeepEqual sees decoded interface{}
// values: numbers as float64, objects as maps (key order free).
bool json_equal(const Json& a, const Json& b) {
  if (a.kind != b.kind) return false;
  switch (a.kind) {
    case Json::Null: return true;
    case Json::Bool: return a.b == b.b;
    case Json::Number: return a.num == b.num;
    case Json::String: return a.str == b.str;
    case Json::Array:
      if (a.arr.size() != b.arr.size()) return false;
      for (size_t i = 0; i < a.arr.size(); ++i)
        if (!json_equal(a.arr[i], b.arr[i])) return false;
      return true;
    case Json::Object: {
      size_t n = 0;
      for (const auto& kv : a.obj) {
        const Json* o = b.get(kv.first);
        if (!o || !json_equal(*a.get(kv.first), *o)) return false;
      }
      for (const auto& kv : b.obj) n += a.get(kv.first) != nullptr;
      return n == b.obj.size();
    }
  }
  return false;
}

// A point matches a filter when its payload holds every filter key with an
// equal value (a conjunction of exact matches, as retrieval-service's
// map[string]string filters read).
bool payload_matches(const Json& payload, const Json& filter) {
  for (const auto& kv : filter.obj) {
    const Json* v = payload.kind == Json::Object ? payload.get(kv.first) : nullptr;
    if (!v || !json_equal(*v, *filter.get(kv.first))) return false;
  }
  return true;
}

// Allow bitmap of `filter` over cs's rows and its device-resident copy
// (reader lock held by the caller).
CollState::FilterEntry filter_mask(vs_engine* eng, const std::string& coll, CollState& cs,
                                   const Json& filter) {
  std::string key;
  vsjson::encode(filter, &key);  // canonical: sorted keys
  {
    std::lock_guard<std::mutex> g(cs.fmu);
    auto it = cs.fcache.find(key);
    if (it != cs.fcache.end()) {
      if (it->second.version == cs.version) return it->second;
      if (it->second.device_id) (void)vs_filter_drop(eng, it->second.device_id);
      cs.fcache.erase(it);
    }
  }
  const uint64_t n = cs.nrows();
  auto m = std::make_shared<std::vector<uint64_t>>((n + 63) / 64, 0);
  for (const auto& kv : cs.bulk_payload)  // other bulk rows have empty payloads
    if (payload_matches(kv.second, filter)) (*m)[kv.first >> 6] |= 1ull << (kv.first & 63);
  for (uint64_t i = 0; i < cs.payload_of.size(); ++i)
    if (payload_matches(cs.payload_of[i], filter)) {
      const uint64_t r = cs.bulk + i;
      (*m)[r >> 6] |= 1ull << (r & 63);
    }
  CollState::FilterEntry e;
  e.version = cs.version;
  e.mask = m;
  if (vs_filter_create(eng, coll.c_str(), m->data(), m->size(), &e.device_id) != VS_OK)
    e.device_id = 0;  // e.g. out of memory: send the mask per call instead
  std::lock_guard<std::mutex> g(cs.fmu);
  if (cs.fcache.size() >= 64) {
    for (auto& kv : cs.fcache)
      if (kv.second.device_id) (void)vs_filter_drop(eng, kv.second.device_id);
    cs.fcache.clear();
  }
  auto& slot = cs.fcache[key];
  if (slot.device_id) (void)vs_filter_drop(eng, slot.device_id);  // a concurrent build
  slot = e;
  return e;
}

Response handle_search(vsvc* svc, const std::string& method, const char* body, size_t len) {
  if (method != "POST") return error_text("Method not allowed", 405);
  SearchRequest req;
  if (!decode_search(body, len, &req).empty()) return error_json("Invalid request body", 400);
  if (req.top_k == 0) req.top_k = 5;
  // The reference sends Limit: uint64(req.TopK), so a negative top_k wraps to
  // a limit near 2^64 whose Qdrant reply is unpinned; here it is refused as a
  // bad request instead of returning every row.
  if (req.top_k < 0) return error_json("top_k must not be negative", 400);
  const uint64_t limit = (uint64_t)req.top_k;  // Limit: uint64(req.TopK)

  auto cs = svc->find(req.collection);
  if (!cs) return error_json("Search failed: " + not_found(req.collection), 500);
  std::shared_lock<std::shared_mutex> rl(cs->mu);
  if (req.query.size() != cs->dim)
    return error_json("Search failed: " + dim_error(cs->dim, req.query.size()), 500);
  const uint64_t rows = cs->nrows();
  // Qdrant returns min(limit, points): any limit is served (k > 1024 takes
  // the engine's large-k select), and buffers are sized by what can return
  uint64_t k = std::min<uint64_t>(limit, std::max<uint64_t>(rows, 1));
  std::vector<float> scores(k);
  std::vector<uint64_t> hit_rows(k);
  uint32_t count = 0;
  // Points.Search: through the batcher (one engine call for all concurrent
  // requests) or directly. The collection's read lock is held until the
  // reply is encoded, so rows and UUIDs cannot change underneath.
  int rc;
  std::string err;
  if (svc->filter_match && req.filter.kind == Json::Object && !req.filter.obj.empty()) {
    // filtered searches: through the batcher with the other requests of the
    // same resident filter, or directly
    auto f = filter_mask(svc->eng, req.collection, *cs, req.filter);
    rc = VS_ERR_NOT_FOUND;
    if (f.device_id && svc->batcher)
      rc = svc->batcher->search(req.collection, req.query.data(), cs->dim, (uint32_t)k,
                                scores.data(), hit_rows.data(), &count, &err, f.device_id);
    else if (f.device_id)
      rc = vs_search_filter_id(svc->eng, req.collection.c_str(), req.query.data(), 1, cs->dim,
                               (uint32_t)k, f.device_id, scores.data(), hit_rows.data(), &count);
    if (rc != VS_OK)  // not resident, or evicted by a concurrent request
      rc = vs_search_filtered(svc->eng, req.collection.c_str(), req.query.data(), 1, cs->dim,
                              (uint32_t)k, f.mask->data(), f.mask->size(), scores.data(),
                              hit_rows.data(), &count);
    if (rc != VS_OK) err = last_error();
  } else if (svc->batcher) {
    rc = svc->batcher->search(req.collection, req.query.data(), cs->dim, (uint32_t)k,
                              scores.data(), hit_rows.data(), &count, &err);
  } else {
    rc = vs_search(svc->eng, req.collection.c_str(), req.query.data(), 1, cs->dim, (uint32_t)k,
                   scores.data(), hit_rows.data(), &count);
    if (rc != VS_OK) err = last_error();
  }
  if (rc != VS_OK) return error_json("Search failed: " + grpc_error(rc, err), 500);

  // SearchResponse{Results, Count}: struct fields in declaration order
  std::string out;
  out.append("{\"results\":[");
  for (uint32_t j = 0; j < count; ++j) {
    if (j) out.push_back(',');
    const uint64_t row = hit_rows[j];
    out.append("{\"id\":");
    vsjson::encode_string(uuid_at(*cs, row), &out);
    out.append(",\"score\":");
    vsjson::encode_float64((double)scores[j], &out);  // float64(hit.GetScore())
    out.append(",\"payload\":");
    vsjson::encode(payload_at(*cs, row), &out);
    out.push_back('}');
  }
  out.append("],\"count\":");
  out.append(std::to_string(count));
  out.append("}\n");
  Response r;
  r.body = std::move(out);
  return r;
}

char* dup_bytes(const std::string& s) {
  char* p = (char*)std::malloc(s.size() + 1);
  if (p) {
    std::memcpy(p, s.data(), s.size());
    p[s.size()] = 0;
  }
  return p;
}

}  // namespace

extern "C" {

int vsvc_open(vs_engine* eng, const char* config_json, vsvc** out) {
  if (!eng || !out) return VS_ERR_INVALID_ARG;
  *out = nullptr;
  struct Spec {
    std::string name;
    uint32_t dim;
    int metric, dtype;
  };
  std::vector<Spec> specs;
  vsbatch::Options bopt;
  bool workers_given = false;
  bool filter_match = false;
  if (!config_json) {
    for (const char* n : {"regulatory_docs", "merchant_docs", "kyc_docs"})
      specs.push_back({n, 768, VS_METRIC_COSINE, VS_DTYPE_F32});
  } else {
    Json cfg;
    std::string err;
    if (!vsjson::parse(config_json, std::strlen(config_json), &cfg, &err)) return VS_ERR_INVALID_ARG;
    const Json* cl = cfg.get("collections");
    if (!cl || cl->kind != Json::Array) return VS_ERR_INVALID_ARG;
    for (const auto& c : cl->arr) {
      const Json* nm = c.get("name");
      const Json* dm = c.get("dim");
      const Json* mt = c.get("metric");
      const Json* dt = c.get("dtype");
      if (!nm || nm->kind != Json::String || !dm || dm->kind != Json::Number)
        return VS_ERR_INVALID_ARG;
      Spec s{nm->str, (uint32_t)dm->num, VS_METRIC_COSINE, VS_DTYPE_F32};
      if (mt && mt->kind == Json::String && (mt->str == "Dot" || mt->str == "dot"))
        s.metric = VS_METRIC_DOT;
      if (dt && dt->kind == Json::String && dt->str == "bf16") s.dtype = VS_DTYPE_BF16;
      specs.push_back(s);
    }
    // {"filter": "ignore" (the reference: main.go:30 vs :249-254) | "match"}
    if (const Json* fm = cfg.get("filter")) {
      if (fm->kind != Json::String || (fm->str != "ignore" && fm->str != "match"))
        return VS_ERR_INVALID_ARG;
      filter_match = fm->str == "match";
    }
    // {"batching": {"enabled": bool, "max_batch": n, "max_wait_us": n, "workers": n,
    //               "lead_us": n, "caller_runs": bool}}
    if (const Json* b = cfg.get("batching")) {
      if (b->kind != Json::Object) return VS_ERR_INVALID_ARG;
      if (const Json* e = b->get("enabled")) {
        if (e->kind != Json::Bool) return VS_ERR_INVALID_ARG;
        bopt.enabled = e->b;
      }
      if (const Json* m = b->get("max_batch")) {
        if (m->kind != Json::Number || m->num < 1 || m->num > 4096) return VS_ERR_INVALID_ARG;
        bopt.max_batch = (uint32_t)m->num;
      }
      if (const Json* nw = b->get("workers")) {
        if (nw->kind != Json::Number || nw->num < 1 || nw->num > 16) return VS_ERR_INVALID_ARG;
        bopt.workers = (uint32_t)nw->num;
        workers_given = true;
      }
      if (const Json* w = b->get("max_wait_us")) {
        if (w->kind != Json::Number || w->num < 0 || w->num > 1e6) return VS_ERR_INVALID_ARG;
        bopt.max_wait_us = (uint32_t)w->num;
      }
      if (const Json* cr = b->get("caller_runs")) {
        if (cr->kind != Json::Bool) return VS_ERR_INVALID_ARG;
        bopt.caller_runs = cr->b;
      }
      if (const Json* l = b->get("lead_us")) {
        if (l->kind != Json::Number || l->num < 0 || l->num > 1e6) return VS_ERR_INVALID_ARG;
        bopt.lead_us = (uint32_t)l->num;
      }
    }
  }
  auto svc = std::make_unique<vsvc>();
  svc->eng = eng;
  svc->batch_opt = bopt;
  svc->filter_match = filter_match;
  for (const auto& s : specs) {
    // initializeCollections: Get, and Create when NotFound (main.go:91-112)
    uint32_t dim = 0;
    uint64_t rows = 0;
    int rc = vs_collection_info(eng, s.name.c_str(), &dim, &rows, nullptr, nullptr);
    if (rc == VS_ERR_NOT_FOUND)
      rc = vs_collection_create(eng, s.name.c_str(), s.dim, s.metric, s.dtype, 0, 0);
    else if (rc == VS_OK && rows != 0)
      rc = VS_ERR_EXISTS;  // rows without UUIDs cannot be served through this layer
    if (rc != VS_OK) return rc;
    auto cs = std::make_shared<CollState>();
    cs->name = s.name;
    cs->dim = dim ? dim : s.dim;
    svc->colls[s.name] = cs;
    svc->listed.push_back(s.name);
  }
  // collections placed on different devices (VS_FLAG_PLACE_COLLECTIONS) run
  // their calls concurrently: two workers per device the collections use,
  // unless the config says otherwise
  if (!workers_given) {
    std::vector<int32_t> lanes;
    for (const auto& s : specs) {
      int32_t d = -1;
      if (vs_collection_placement(eng, s.name.c_str(), &d) == VS_OK &&
          std::find(lanes.begin(), lanes.end(), d) == lanes.end())
        lanes.push_back(d);
    }
    bopt.workers = (uint32_t)std::min<size_t>(16, 2 * std::max<size_t>(1, lanes.size()));
    svc->batch_opt.workers = bopt.workers;
  }
  if (bopt.enabled) svc->batcher = std::make_unique<vsbatch::Batcher>(eng, bopt);
  *out = svc.release();
  return VS_OK;
}

void vsvc_close(vsvc* svc) { delete svc; }  // the batcher drains and joins first

int vsvc_bulk_generate(vsvc* svc, const char* coll, uint64_t n, uint64_t seed) {
  if (!svc || !coll) return VS_ERR_INVALID_ARG;
  auto cs = svc->find(coll);
  if (!cs) return VS_ERR_NOT_FOUND;
  if (n >= (1ull << 40)) return VS_ERR_INVALID_ARG;
  std::unique_lock<std::shared_mutex> wl(cs->mu);
  if (cs->nrows() != 0) return VS_ERR_EXISTS;  // bulk rows come first
  const int rc = vs_generate(svc->eng, coll, n, seed);
  if (rc != VS_OK) return rc;
  uint64_t h = 1469598103934665603ull;  // FNV-1a of the name, mixed with the seed
  for (const char* p = coll; *p; ++p) h = (h ^ (uint8_t)*p) * 1099511628211ull;
  h ^= seed + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
  h = (h ^ (h >> 31)) * 0xBF58476D1CE4E5B9ull;
  cs->bulk_tag = ((h ^ (h >> 29)) & 0xFFFFFFFFFFFFull) | 1u;
  cs->bulk = n;
  ++cs->version;
  return VS_OK;
}

// Sidecar of a collection snapshot: the host half of the store (UUIDs,
// payloads, bulk range) as JSON; the rows go through vs_snapshot.
//   {"bulk":n,"bulk_tag":t,"bulk_payload":[[row,{..}],..],"points":[["uuid",{..}],..]}
// with points[i] = row bulk + i.
int vsvc_snapshot(vsvc* svc, const char* dir) {
  if (!svc || !dir) return VS_ERR_INVALID_ARG;
  for (const std::string& name : svc->listed) {
    auto cs = svc->find(name);
    std::shared_lock<std::shared_mutex> rl(cs->mu);  // upserts wait
    const std::string base = std::string(dir) + "/" + name;
    int rc = vs_snapshot(svc->eng, name.c_str(), (base + ".vsnap").c_str());
    if (rc != VS_OK) return rc;
    std::string out = "{\"bulk\":" + std::to_string(cs->bulk) +
                      ",\"bulk_tag\":" + std::to_string(cs->bulk_tag) + ",\"bulk_payload\":[";
    bool first = true;
    for (const auto& kv : cs->bulk_payload) {
      out.append(first ? "[" : ",[");
      first = false;
      out.append(std::to_string(kv.first));
      out.push_back(',');
      vsjson::encode(kv.second, &out);
      out.push_back(']');
    }
    out.append("],\"points\":[");
    for (size_t i = 0; i < cs->uuid_of.size(); ++i) {
      out.append(i ? ",[" : "[");
      vsjson::encode_string(cs->uuid_of[i], &out);
      out.push_back(',');
      vsjson::encode(cs->payload_of[i], &out);
      out.push_back(']');
    }
    out.append("]}\n");
    const std::string tmp = base + ".points.json.tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    bool ok = f && std::fwrite(out.data(), 1, out.size(), f) == out.size();
    if (f) ok = (std::fclose(f) == 0) && ok;
    if (!ok || std::rename(tmp.c_str(), (base + ".points.json").c_str()) != 0)
      return VS_ERR_IO;
  }
  return VS_OK;
}

namespace {
// A parsed, fully checked sidecar (vsvc_snapshot's <coll>.points.json).
struct Sidecar {
  uint64_t bulk = 0, bulk_tag = 0;
  std::vector<std::pair<uint64_t, Json>> bulk_payload;
  std::vector<std::string> uuids;  // canonical; row bulk + i
  std::vector<Json> payloads;
};

bool json_uint(const Json* v, uint64_t max, uint64_t* out) {
  if (!v || v->kind != Json::Number || !(v->num >= 0) || v->num > (double)max ||
      v->num != (double)(uint64_t)v->num)
    return false;
  *out = (uint64_t)v->num;
  return true;
}

// Every field is checked before anything is changed: integral, in-range
// counters; payload rows inside the bulk range; every point a [uuid, object]
// pair with a canonical, unique UUID that is not one of the bulk ids.
bool parse_sidecar(const std::string& text, Sidecar* sc) {
  Json side;
  std::string err;
  if (!vsjson::parse(text.data(), text.size(), &side, &err) || side.kind != Json::Object)
    return false;
  const Json* jbp = side.get("bulk_payload");
  const Json* jp = side.get("points");
  if (!json_uint(side.get("bulk"), (1ull << 40) - 1, &sc->bulk) ||
      !json_uint(side.get("bulk_tag"), (1ull << 48) - 1, &sc->bulk_tag) || !jbp ||
      jbp->kind != Json::Array || !jp || jp->kind != Json::Array)
    return false;
  if (sc->bulk && !(sc->bulk_tag & 1)) return false;  // vsvc_bulk_generate sets bit 0
  for (const auto& e : jbp->arr) {
    uint64_t row = 0;
    if (e.kind != Json::Array || e.arr.size() != 2 || !json_uint(&e.arr[0], sc->bulk - 1, &row) ||
        sc->bulk == 0 || e.arr[1].kind != Json::Object)
      return false;
    sc->bulk_payload.emplace_back(row, e.arr[1]);
  }
  std::unordered_map<std::string, uint64_t> seen;
  CollState probe;
  probe.bulk = sc->bulk;
  probe.bulk_tag = sc->bulk_tag;
  for (const auto& e : jp->arr) {
    std::string canon;
    uint64_t r;
    if (e.kind != Json::Array || e.arr.size() != 2 || e.arr[0].kind != Json::String ||
        e.arr[1].kind != Json::Object || !canonical_uuid(e.arr[0].str, &canon) ||
        canon != e.arr[0].str || bulk_row(probe, canon, &r) ||
        !seen.emplace(canon, sc->uuids.size()).second)
      return false;
    sc->uuids.push_back(canon);
    sc->payloads.push_back(e.arr[1]);
  }
  return true;
}
}  // namespace

int vsvc_restore(vsvc* svc, const char* dir) {
  if (!svc || !dir) return VS_ERR_INVALID_ARG;
  for (const std::string& name : svc->listed) {
    auto cs = svc->find(name);
    const std::string base = std::string(dir) + "/" + name;
    FILE* f = std::fopen((base + ".points.json").c_str(), "rb");
    if (!f) continue;  // nothing saved for this collection
    std::string text;
    char buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) text.append(buf, n);
    std::fclose(f);
    Sidecar sc;
    if (!parse_sidecar(text, &sc)) return VS_ERR_IO;  // nothing touched yet
    std::unique_lock<std::shared_mutex> wl(cs->mu);
    if (cs->nrows() != 0) return VS_ERR_EXISTS;  // restore only into an empty service
    uint32_t dim = 0;
    int metric = 0, dtype = 0;
    int rc = vs_collection_info(svc->eng, name.c_str(), &dim, nullptr, &metric, &dtype);
    if (rc != VS_OK) return rc;
    if ((rc = vs_collection_drop(svc->eng, name.c_str())) != VS_OK) return rc;
    rc = vs_restore(svc->eng, name.c_str(), (base + ".vsnap").c_str());
    uint64_t rows = 0;
    uint32_t rdim = 0;
    int rmetric = 0, rdtype = 0;
    if (rc == VS_OK)
      rc = vs_collection_info(svc->eng, name.c_str(), &rdim, &rows, &rmetric, &rdtype);
    if (rc == VS_OK && (rdim != dim || rmetric != metric || rdtype != dtype ||
                        rows != sc.bulk + sc.uuids.size()))
      rc = VS_ERR_IO;
    if (rc != VS_OK) {  // leave the collection as it was: empty
      (void)vs_collection_drop(svc->eng, name.c_str());
      (void)vs_collection_create(svc->eng, name.c_str(), dim, metric, dtype, 0, 0);
      return rc;
    }
    cs->bulk = sc.bulk;
    cs->bulk_tag = sc.bulk_tag;
    for (auto& e : sc.bulk_payload) cs->bulk_payload[e.first] = std::move(e.second);
    cs->row_of.reserve(sc.uuids.size());
    for (size_t i = 0; i < sc.uuids.size(); ++i) cs->row_of[sc.uuids[i]] = sc.bulk + i;
    cs->uuid_of = std::move(sc.uuids);
    cs->payload_of = std::move(sc.payloads);
    ++cs->version;
  }
  return VS_OK;
}

int vsvc_point_id(vsvc* svc, const char* coll, uint64_t row, char* buf, size_t len) {
  if (!svc || !coll || !buf || len < 37) return VS_ERR_INVALID_ARG;
  auto cs = svc->find(coll);
  if (!cs) return VS_ERR_NOT_FOUND;
  std::shared_lock<std::shared_mutex> rl(cs->mu);
  if (row >= cs->nrows()) return VS_ERR_INVALID_ARG;
  const std::string u = uuid_at(*cs, row);
  std::memcpy(buf, u.c_str(), u.size() + 1);
  return VS_OK;
}

int vsvc_stats(vsvc* svc, char** out) {
  if (!svc || !out) return VS_ERR_INVALID_ARG;
  vsbatch::Stats st;
  if (svc->batcher) st = svc->batcher->stats();
  Json o = Json::object();
  Json b = Json::object();
  b.obj.emplace_back("enabled", Json::boolean(svc->batcher != nullptr));
  b.obj.emplace_back("max_batch", Json::number(svc->batch_opt.max_batch));
  b.obj.emplace_back("max_wait_us", Json::number(svc->batch_opt.max_wait_us));
  b.obj.emplace_back("workers", Json::number(svc->batch_opt.workers));
  b.obj.emplace_back("lead_us", Json::number(svc->batch_opt.lead_us));
  b.obj.emplace_back("caller_runs", Json::boolean(svc->batch_opt.caller_runs));
  o.obj.emplace_back("batching", std::move(b));
  o.obj.emplace_back("requests", Json::number((double)st.requests));
  o.obj.emplace_back("engine_calls", Json::number((double)st.engine_calls));
  o.obj.emplace_back("largest_call", Json::number((double)st.max_batch));
  Json h = Json::array();
  for (uint64_t v : st.hist) h.arr.push_back(Json::number((double)v));
  o.obj.emplace_back("calls_by_log2_nq", std::move(h));
  std::string s;
  vsjson::encode(o, &s, false);
  *out = dup_bytes(s);
  return *out ? VS_OK : VS_ERR_OOM;
}

int vsvc_handle(vsvc* svc, const char* method, const char* path, const char* body,
                size_t body_len, int* status, char** resp, size_t* resp_len,
                const char** content_type) {
  if (!svc || !method || !path || !status || !resp) return VS_ERR_INVALID_ARG;
  if (!body) body = "";
  const std::string m = method, p = path;
  Response r;
  if (p == "/health") r = handle_health(svc);
  else if (p == "/collections") r = handle_collections(svc, m);
  else if (p == "/upsert") r = handle_upsert(svc, m, body, body_len);
  else if (p == "/search") r = handle_search(svc, m, body, body_len);
  else r = error_text("404 page not found", 404);
  *status = r.status;
  *resp = dup_bytes(r.body);
  if (resp_len) *resp_len = r.body.size();
  if (content_type) *content_type = r.type == kTextType ? kTextType : kJsonType;
  return *resp ? VS_OK : VS_ERR_OOM;
}

void vsvc_free(char* p) { std::free(p); }

int vsvc_reencode(const char* json, size_t len, char** out) {
  Json v;
  std::string err;
  if (!vsjson::parse(json, len, &v, &err)) {
    *out = dup_bytes(err);
    return -1;
  }
  std::string s;
  vsjson::encode(v, &s);
  s.push_back('\n');
  *out = dup_bytes(s);
  return 0;
}

// Test hook (not in the public header): the /search decode through the fast
// path only (path 1: "declined" when it falls back) or the generic decoder
// only (path 0), as JSON {"collection","query":[float32 bits],"top_k"} or
// {"error"}, so the tests can hold the two decoders equal.
int vsvc_debug_decode_search(const char* body, size_t len, int path, char** out) {
  if (!out) return VS_ERR_INVALID_ARG;
  SearchRequest r;
  std::string err;
  if (path == 1) {
    if (!decode_search_fast(body ? body : "", len, &r)) err = "declined";
  } else {
    err = decode_search_generic(body ? body : "", len, &r);
  }
  Json o = Json::object();
  if (!err.empty()) {
    o.obj.emplace_back("error", Json::string(err));
  } else {
    o.obj.emplace_back("collection", Json::string(r.collection));
    Json q = Json::array();
    for (float f : r.query) {
      uint32_t u;
      std::memcpy(&u, &f, 4);
      q.arr.push_back(Json::number((double)u));
    }
    o.obj.emplace_back("query", std::move(q));
    o.obj.emplace_back("top_k", Json::number((double)r.top_k));
  }
  std::string s;
  vsjson::encode(o, &s, false);
  *out = dup_bytes(s);
  return *out ? VS_OK : VS_ERR_OOM;
}

int vsvc_validate(const char* path, const char* body, size_t len, char** msg) {
  std::string p = path ? path : "", err;
  if (p == "/search") {
    SearchRequest r;
    err = decode_search(body ? body : "", len, &r);
  } else if (p == "/upsert") {
    UpsertRequest r;
    err = decode_upsert(body ? body : "", len, &r);
  }
  if (msg) *msg = dup_bytes(err);
  return err.empty() ? 0 : 400;
}

}  // extern "C"
