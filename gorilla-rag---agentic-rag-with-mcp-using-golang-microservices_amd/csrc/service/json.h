// json.h — the JSON dialect of rag/vector-service (Go encoding/json).
//
// Decoding keeps each number's literal so a field can be parsed the way Go
// parses it for its target type: float32 fields (SearchRequest.Query,
// rag/vector-service/main.go:28) straight from decimal, interface{} values
// (UpsertRequest points, main.go:22) as float64, int fields (TopK) as a
// base-10 integer literal. Encoding follows json.Encoder: object keys of maps
// sorted, float64 in the shortest round-trip form ('e' only below 1e-6 or from
// 1e21, "e-07" cleaned to "e-7"), <, >, & and U+2028/9 escaped, trailing '\n'
// added by the caller.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace vsjson {

struct Json {
  enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
  bool b = false;
  double num = 0.0;      // float64 value of a Number (Go interface{} decoding)
  std::string str;       // String value, or the literal text of a Number
  std::vector<Json> arr;
  std::vector<std::pair<std::string, Json>> obj;  // in document order

  static Json null() { return Json(); }
  static Json boolean(bool v) { Json j; j.kind = Bool; j.b = v; return j; }
  static Json number(double v) { Json j; j.kind = Number; j.num = v; return j; }
  static Json string(std::string s) { Json j; j.kind = String; j.str = std::move(s); return j; }
  static Json array() { Json j; j.kind = Array; return j; }
  static Json object() { Json j; j.kind = Object; return j; }

  // last value of `key` (exact match preferred, else ASCII case-insensitive,
  // as Go matches struct fields); nullptr if absent
  const Json* field(const std::string& key) const;
  // exact-key lookup (Go map[string]interface{} semantics: last duplicate wins)
  const Json* get(const std::string& key) const;
};

// Parses the first JSON value of `s` (trailing bytes are ignored, like
// json.Decoder.Decode). Returns false with a message on a syntax error.
bool parse(const char* s, size_t n, Json* out, std::string* err);

// Go-style encoders. `sort_keys` = the value came from a Go map.
void encode(const Json& v, std::string* out, bool sort_keys = true);
void encode_string(const std::string& s, std::string* out);
void encode_float64(double v, std::string* out);

// strconv-equivalent literal parsers. Return false on a syntax/range error.
bool parse_float32(const std::string& lit, float* out);   // ParseFloat(s, 32)
bool parse_int64(const std::string& lit, int64_t* out);   // ParseInt(s, 10, 64)

}  // namespace vsjson
