// Compact arena JSON DOM used by the policy compiler and the resource ingest.
// Number typing follows the two decoders the reference uses:
//   NUM_FLOAT        encoding/json into interface{} (policies / patterns)
//   NUM_UNSTRUCTURED k8s unstructured.UnmarshalJSON: int64 if the literal parses
//                    as int64, else float64 (resources)
// Strings are decoded with encoding/json's rules: invalid UTF-8 and lone
// surrogates become U+FFFD. Duplicate object keys: last one wins.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace kvh {

enum JT : uint8_t { J_NULL = 0, J_BOOL, J_INT, J_FLOAT, J_STR, J_MAP, J_ARR };
enum NumMode { NUM_FLOAT, NUM_UNSTRUCTURED };

struct JNode {
  uint8_t t = J_NULL;
  bool b = false;
  uint32_t key_off = 0, key_len = 0;  // key in parent map (strs)
  uint32_t s_off = 0, s_len = 0;      // J_STR value (strs)
  uint32_t first = 0, count = 0;      // J_MAP / J_ARR children in nodes[]
  int64_t i = 0;
  double f = 0;
};

struct JDoc {
  std::vector<JNode> nodes;
  std::string strs;
  uint32_t root = 0;

  std::string_view str(uint32_t off, uint32_t len) const { return std::string_view(strs.data() + off, len); }
  std::string_view key(const JNode& n) const { return str(n.key_off, n.key_len); }
  std::string_view sval(const JNode& n) const { return str(n.s_off, n.s_len); }
  const JNode& at(uint32_t i) const { return nodes[i]; }
  // map lookup, -1 if absent
  int64_t get(uint32_t map, std::string_view k) const {
    const JNode& m = nodes[map];
    if (m.t != J_MAP) return -1;
    for (uint32_t c = m.first; c < m.first + m.count; c++)
      if (key(nodes[c]) == k) return c;
    return -1;
  }
};

// Parse one JSON value. Throws std::runtime_error.
void parse_json(const char* p, size_t n, NumMode mode, JDoc* doc);
// Parse a stream of JSON values: a top-level array (each element one value) or
// whitespace/newline separated values (NDJSON). Calls cb(doc) per value, reusing doc.
template <class F>
void parse_json_stream(const char* p, size_t n, NumMode mode, F&& cb);

// Go-compatible helpers (gocompat.cpp)
bool go_parse_int(std::string_view s, int64_t* out);
bool go_parse_float(std::string_view s, double* out);
std::string go_format_E(double v);
std::string go_format_f6(double v);
std::string go_json_float(double v);  // encoding/json float64
std::string go_format_g(double v);  // fmt %v of a float64
bool utf8_ascii(std::string_view s);

// k8s resource.Quantity canonical form (quantity.cpp)
struct QCanon {
  bool valid = false, neg = false, zero = false;
  int32_t exp = 0;  // order of magnitude: number of digits + exp10 of the normalized value
  uint64_t hi = 0, lo = 0;
};
QCanon parse_quantity(std::string_view s);

// Go `\d*(\.\d+)?` helpers etc. live with the compiler.

// internal: parser entry that parses at most one value starting at p, returns consumed bytes
size_t parse_one(const char* p, size_t n, NumMode mode, JDoc* doc);

template <class F>
void parse_json_stream(const char* p, size_t n, NumMode mode, F&& cb) {
  size_t i = 0;
  auto ws = [&]() {
    while (i < n && (p[i] == ' ' || p[i] == '\t' || p[i] == '\n' || p[i] == '\r')) i++;
  };
  ws();
  JDoc doc;
  if (i < n && p[i] == '[') {
    i++;
    ws();
    if (i < n && p[i] == ']') return;
    while (true) {
      doc.nodes.clear();
      doc.strs.clear();
      i += parse_one(p + i, n - i, mode, &doc);
      cb(doc);
      ws();
      if (i < n && p[i] == ',') { i++; ws(); continue; }
      if (i < n && p[i] == ']') { i++; break; }
      throw std::runtime_error("json: expected , or ] in resource list");
    }
    ws();
    if (i != n) throw std::runtime_error("json: trailing data after resource list");
    return;
  }
  while (i < n) {
    doc.nodes.clear();
    doc.strs.clear();
    i += parse_one(p + i, n - i, mode, &doc);
    cb(doc);
    ws();
  }
}

}  // namespace kvh
