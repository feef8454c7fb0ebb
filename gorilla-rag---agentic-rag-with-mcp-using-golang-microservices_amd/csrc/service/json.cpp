// json.cpp — see json.h. Go toolchain behaviour mirrored: encoding/json of
// Go >= 1.22 (the repository root pins go 1.24.3, go.mod:3).
#include "json.h"

#include <algorithm>
#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace vsjson {

namespace {

bool ieq(const std::string& a, const std::string& b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i) {
    char x = a[i], y = b[i];
    if (x >= 'A' && x <= 'Z') x = (char)(x - 'A' + 'a');
    if (y >= 'A' && y <= 'Z') y = (char)(y - 'A' + 'a');
    if (x != y) return false;
  }
  return true;
}

void put_utf8(uint32_t cp, std::string* o) {
  if (cp < 0x80) {
    o->push_back((char)cp);
  } else if (cp < 0x800) {
    o->push_back((char)(0xC0 | (cp >> 6)));
    o->push_back((char)(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    o->push_back((char)(0xE0 | (cp >> 12)));
    o->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    o->push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    o->push_back((char)(0xF0 | (cp >> 18)));
    o->push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    o->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    o->push_back((char)(0x80 | (cp & 0x3F)));
  }
}

// Decodes one UTF-8 rune at s[i] (n bytes available). Returns its length and
// sets *cp; invalid sequences return 1 with *cp = 0xFFFD (Go's RuneError).
int next_rune(const unsigned char* s, size_t n, uint32_t* cp) {
  unsigned char c = s[0];
  if (c < 0x80) { *cp = c; return 1; }
  int len = (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : (c & 0xF8) == 0xF0 ? 4 : 0;
  if (len == 0 || (size_t)len > n) { *cp = 0xFFFD; return 1; }
  uint32_t v = c & (0xFF >> (len + 1));
  for (int i = 1; i < len; ++i) {
    if ((s[i] & 0xC0) != 0x80) { *cp = 0xFFFD; return 1; }
    v = (v << 6) | (s[i] & 0x3F);
  }
  static const uint32_t minv[5] = {0, 0, 0x80, 0x800, 0x10000};
  if (v < minv[len] || v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) { *cp = 0xFFFD; return 1; }
  *cp = v;
  return len;
}

struct Parser {
  const char* s;
  size_t n, i = 0;
  std::string err;
  int depth = 0;

  void ws() {
    while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
  }
  bool fail(const char* m) {
    if (err.empty()) err = std::string(m) + " at offset " + std::to_string(i);
    return false;
  }
  bool lit(const char* w) {
    size_t L = std::strlen(w);
    if (n - i < L || std::memcmp(s + i, w, L) != 0) return fail("invalid literal");
    i += L;
    return true;
  }
  int hex4(size_t at) {
    if (n - at < 4) return -1;
    int v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = s[at + k];
      int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10
              : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
      if (d < 0) return -1;
      v = v * 16 + d;
    }
    return v;
  }
  bool string(std::string* out) {
    ++i;  // opening quote
    while (true) {
      if (i >= n) return fail("unterminated string");
      unsigned char c = (unsigned char)s[i];
      if (c == '"') { ++i; return true; }
      if (c < 0x20) return fail("control character in string");
      if (c == '\\') {
        if (i + 1 >= n) return fail("bad escape");
        char e = s[i + 1];
        i += 2;
        switch (e) {
          case '"': out->push_back('"'); break;
          case '\\': out->push_back('\\'); break;
          case '/': out->push_back('/'); break;
          case 'b': out->push_back('\b'); break;
          case 'f': out->push_back('\f'); break;
          case 'n': out->push_back('\n'); break;
          case 'r': out->push_back('\r'); break;
          case 't': out->push_back('\t'); break;
          case 'u': {
            int v = hex4(i);
            if (v < 0) return fail("bad \\u escape");
            i += 4;
            uint32_t cp = (uint32_t)v;
            if (cp >= 0xD800 && cp < 0xDC00) {  // surrogate pair
              int lo = (i + 1 < n && s[i] == '\\' && s[i + 1] == 'u') ? hex4(i + 2) : -1;
              if (lo >= 0xDC00 && lo < 0xE000) {
                cp = 0x10000 + ((cp - 0xD800) << 10) + ((uint32_t)lo - 0xDC00);
                i += 6;
              } else {
                cp = 0xFFFD;
              }
            } else if (cp >= 0xDC00 && cp < 0xE000) {
              cp = 0xFFFD;
            }
            put_utf8(cp, out);
            break;
          }
          default:
            return fail("bad escape");
        }
        continue;
      }
      uint32_t cp;
      int len = next_rune((const unsigned char*)s + i, n - i, &cp);
      if (cp == 0xFFFD && len == 1 && c >= 0x80)
        put_utf8(0xFFFD, out);  // invalid UTF-8 becomes U+FFFD, as Go does
      else
        out->append(s + i, len);
      i += len;
    }
  }
  bool number(Json* out) {
    size_t st = i;
    if (s[i] == '-') ++i;
    if (i >= n) return fail("bad number");
    if (s[i] == '0') {
      ++i;
    } else if (s[i] >= '1' && s[i] <= '9') {
      while (i < n && s[i] >= '0' && s[i] <= '9') ++i;
    } else {
      return fail("bad number");
    }
    if (i < n && s[i] == '.') {
      ++i;
      if (i >= n || !(s[i] >= '0' && s[i] <= '9')) return fail("bad number");
      while (i < n && s[i] >= '0' && s[i] <= '9') ++i;
    }
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
      ++i;
      if (i < n && (s[i] == '+' || s[i] == '-')) ++i;
      if (i >= n || !(s[i] >= '0' && s[i] <= '9')) return fail("bad number");
      while (i < n && s[i] >= '0' && s[i] <= '9') ++i;
    }
    out->kind = Json::Number;
    out->str.assign(s + st, i - st);
    // correctly rounded either way; from_chars is ~4x faster than strtod
    // (no locale), which matters for 768-number query bodies. Out of range
    // (overflow to inf, underflow) keeps strtod's IEEE result.
    const auto r = std::from_chars(s + st, s + i, out->num);
    if (r.ec != std::errc() || r.ptr != s + i) out->num = std::strtod(out->str.c_str(), nullptr);
    return true;
  }
  bool value(Json* out) {
    if (++depth > 10000) return fail("exceeded max depth");
    ws();
    if (i >= n) return fail("unexpected end of JSON input");
    bool ok;
    switch (s[i]) {
      case '{': {
        out->kind = Json::Object;
        ++i;
        ws();
        if (i < n && s[i] == '}') { ++i; ok = true; break; }
        while (true) {
          ws();
          if (i >= n || s[i] != '"') { ok = fail("expected object key"); break; }
          std::string key;
          if (!string(&key)) { ok = false; break; }
          ws();
          if (i >= n || s[i] != ':') { ok = fail("expected ':'"); break; }
          ++i;
          Json v;
          if (!value(&v)) { ok = false; break; }
          out->obj.emplace_back(std::move(key), std::move(v));
          ws();
          if (i < n && s[i] == ',') { ++i; continue; }
          if (i < n && s[i] == '}') { ++i; ok = true; break; }
          ok = fail("expected ',' or '}'");
          break;
        }
        break;
      }
      case '[': {
        out->kind = Json::Array;
        ++i;
        ws();
        if (i < n && s[i] == ']') { ++i; ok = true; break; }
        while (true) {
          out->arr.emplace_back();  // parsed in place: no element copy per value
          if (!value(&out->arr.back())) { ok = false; break; }
          ws();
          if (i < n && s[i] == ',') { ++i; continue; }
          if (i < n && s[i] == ']') { ++i; ok = true; break; }
          ok = fail("expected ',' or ']'");
          break;
        }
        break;
      }
      case '"':
        out->kind = Json::String;
        ok = string(&out->str);
        break;
      case 't': out->kind = Json::Bool; out->b = true; ok = lit("true"); break;
      case 'f': out->kind = Json::Bool; out->b = false; ok = lit("false"); break;
      case 'n': out->kind = Json::Null; ok = lit("null"); break;
      default:
        ok = (s[i] == '-' || (s[i] >= '0' && s[i] <= '9')) ? number(out) : fail("invalid character");
    }
    --depth;
    return ok;
  }
};

const char kHex[] = "0123456789abcdef";

}  // namespace

const Json* Json::field(const std::string& key) const {
  const Json* exact = nullptr;
  const Json* fold = nullptr;
  for (const auto& kv : obj) {
    if (kv.first == key) exact = &kv.second;
    else if (ieq(kv.first, key)) fold = &kv.second;
  }
  // Go assigns every matching key in document order; the last one wins.
  if (exact && fold) {
    const Json* last = nullptr;
    for (const auto& kv : obj)
      if (kv.first == key || ieq(kv.first, key)) last = &kv.second;
    return last;
  }
  return exact ? exact : fold;
}

const Json* Json::get(const std::string& key) const {
  const Json* last = nullptr;
  for (const auto& kv : obj)
    if (kv.first == key) last = &kv.second;
  return last;
}

bool parse(const char* s, size_t n, Json* out, std::string* err) {
  Parser p{s, n};
  *out = Json();
  if (!p.value(out)) {
    if (err) *err = p.err;
    return false;
  }
  return true;
}

void encode_string(const std::string& s, std::string* o) {
  o->push_back('"');
  const unsigned char* p = (const unsigned char*)s.data();
  size_t n = s.size(), i = 0;
  while (i < n) {
    unsigned char c = p[i];
    if (c < 0x80) {
      switch (c) {
        case '"': o->append("\\\""); break;
        case '\\': o->append("\\\\"); break;
        case '\b': o->append("\\b"); break;
        case '\f': o->append("\\f"); break;
        case '\n': o->append("\\n"); break;
        case '\r': o->append("\\r"); break;
        case '\t': o->append("\\t"); break;
        case '<': case '>': case '&':
          o->append("\\u00");
          o->push_back(kHex[c >> 4]);
          o->push_back(kHex[c & 15]);
          break;
        default:
          if (c < 0x20) {
            o->append("\\u00");
            o->push_back(kHex[c >> 4]);
            o->push_back(kHex[c & 15]);
          } else {
            o->push_back((char)c);
          }
      }
      ++i;
      continue;
    }
    uint32_t cp;
    int len = next_rune(p + i, n - i, &cp);
    if (cp == 0xFFFD && len == 1) {
      o->append("\\ufffd");
    } else if (cp == 0x2028 || cp == 0x2029) {
      o->append(cp == 0x2028 ? "\\u2028" : "\\u2029");
    } else {
      o->append((const char*)p + i, len);
    }
    i += len;
  }
  o->push_back('"');
}

void encode_float64(double v, std::string* o) {
  char buf[64];
  double a = std::fabs(v);
  bool sci = a != 0 && (a < 1e-6 || a >= 1e21);
  auto r = std::to_chars(buf, buf + sizeof(buf), v,
                         sci ? std::chars_format::scientific : std::chars_format::fixed);
  size_t len = (size_t)(r.ptr - buf);
  if (sci && len >= 4 && buf[len - 4] == 'e' && buf[len - 3] == '-' && buf[len - 2] == '0') {
    buf[len - 2] = buf[len - 1];
    --len;
  }
  o->append(buf, len);
}

void encode(const Json& v, std::string* o, bool sort_keys) {
  switch (v.kind) {
    case Json::Null: o->append("null"); break;
    case Json::Bool: o->append(v.b ? "true" : "false"); break;
    case Json::Number: encode_float64(v.num, o); break;
    case Json::String: encode_string(v.str, o); break;
    case Json::Array:
      o->push_back('[');
      for (size_t i = 0; i < v.arr.size(); ++i) {
        if (i) o->push_back(',');
        encode(v.arr[i], o, sort_keys);
      }
      o->push_back(']');
      break;
    case Json::Object: {
      // a decoded Go map: duplicate keys collapse to the last value, keys sorted
      std::vector<std::pair<std::string, const Json*>> kv;
      for (const auto& e : v.obj) {
        auto it = std::find_if(kv.begin(), kv.end(), [&](const auto& x) { return x.first == e.first; });
        if (it != kv.end()) it->second = &e.second;
        else kv.emplace_back(e.first, &e.second);
      }
      if (sort_keys)
        std::sort(kv.begin(), kv.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
      o->push_back('{');
      for (size_t i = 0; i < kv.size(); ++i) {
        if (i) o->push_back(',');
        encode_string(kv[i].first, o);
        o->push_back(':');
        encode(*kv[i].second, o, sort_keys);
      }
      o->push_back('}');
      break;
    }
  }
}

bool parse_float32(const std::string& lit, float* out) {
  // Go's ParseFloat(s, 32): the correctly rounded float32. Fast path
  // from_chars; anything it does not take cleanly (out of range either way)
  // goes through strtof, which tells overflow (an error in Go) from
  // underflow (not one).
  float f;
  const auto r = std::from_chars(lit.data(), lit.data() + lit.size(), f);
  if (r.ec == std::errc() && r.ptr == lit.data() + lit.size()) {
    *out = f;
    return true;
  }
  errno = 0;
  char* end = nullptr;
  float v = std::strtof(lit.c_str(), &end);
  if (end != lit.c_str() + lit.size()) return false;
  if (std::isinf(v)) return false;  // more than 1/2 ulp beyond FLT_MAX: ErrRange
  *out = v;                         // underflow to 0/denormal is not an error in Go
  return true;
}

bool parse_int64(const std::string& lit, int64_t* out) {
  const char* b = lit.data();
  const char* e = b + lit.size();
  if (b != e && *b == '+') return false;
  auto r = std::from_chars(b, e, *out, 10);
  return r.ec == std::errc() && r.ptr == e;
}

}  // namespace vsjson
