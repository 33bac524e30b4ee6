// ORACLE — test infrastructure only. CPU restatement of the reference's
// validate.pattern path (isabella232/kyverno v1.5.x). Nothing under kyverno_amd/
// may include or link this code; only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg use it, as the checker.
//
// JSON value model mirroring Go's decoded `interface{}` trees:
//   - encoding/json into interface{}           (numbers always float64)
//     used for patterns: pkg/utils/loadpolicy.go:28-31 (apiextensions.JSON)
//   - k8s unstructured.UnmarshalJSON           (int64 if the literal parses as
//     int64, else float64): pkg/engine/utils/utils.go:93-100, fetch.go:266
// Invalid UTF-8 / lone surrogates in strings are replaced by U+FFFD, as
// encoding/json does when unmarshaling quoted strings.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace orc {

enum class T : uint8_t { Null = 0, Bool, Int, Float, Str, Map, Arr };

struct Value {
  T t = T::Null;
  bool b = false;
  int64_t i = 0;
  double f = 0.0;
  std::string s;
  // Map entries: key, value. `order` is the canonical iteration key (normally
  // the key itself; ExpandInMetadata sets it to the pre-expansion pattern key).
  struct Entry {
    std::string key;
    std::string order;
    Value* val;  // owned
  };
  std::vector<Entry> m;
  std::vector<Value*> a;  // owned

  Value() = default;
  Value(const Value& o) { copy_from(o); }
  Value& operator=(const Value& o) {
    if (this != &o) { clear(); copy_from(o); }
    return *this;
  }
  ~Value() { clear(); }

  void clear();
  void copy_from(const Value& o);

  bool is_nil() const { return t == T::Null; }
  const Value* get(const std::string& k) const;  // nullptr if absent
  Value* get_mut(const std::string& k);
  bool has(const std::string& k) const { return get(k) != nullptr; }
  void set(const std::string& k, const Value& v, const std::string& order);
  void erase(const std::string& k);

  static Value mk_str(const std::string& s) { Value v; v.t = T::Str; v.s = s; return v; }
  static Value mk_float(double f) { Value v; v.t = T::Float; v.f = f; return v; }
  static Value mk_int(int64_t i) { Value v; v.t = T::Int; v.i = i; return v; }
  static Value mk_bool(bool b) { Value v; v.t = T::Bool; v.b = b; return v; }
  static Value mk_map() { Value v; v.t = T::Map; return v; }
  static Value mk_arr() { Value v; v.t = T::Arr; return v; }
};

enum class NumMode { Float, Unstructured };

// Parses JSON text. Throws std::runtime_error on malformed input.
Value parse_json(const std::string& text, NumMode mode);
// Serializes (used for test plumbing; numbers: int64 decimal, float via %.17g).
std::string to_json(const Value& v);

// Go-compatible helpers (gofmt.cpp)
std::string go_format_E(double v);       // strconv.FormatFloat(v,'E',-1,64)
std::string go_format_f6(double v);      // fmt.Sprintf("%f", v)
std::string go_format_g(double v);       // fmt %v of float64 (FormatFloat 'g' -1, eprec 6)
std::string go_format_v(const Value* v); // fmt %v of an interface{} value
std::string go_type_name(const Value* v);// fmt %T of an interface{} value
bool go_parse_float(const std::string& s, double* out);   // strconv.ParseFloat(s,64) err==nil
bool go_parse_int(const std::string& s, int64_t* out);    // strconv.ParseInt(s,10,64) err==nil
std::string utf8_sanitize(const std::string& s);

// minio/pkg v1.1.3 wildcard.Match (glob.cpp)
bool wildcard_match(const std::string& pattern, const std::string& name);

// k8s.io/apimachinery v0.21.4 resource.ParseQuantity / Quantity.Cmp (quantity.cpp)
struct Quantity {
  bool neg = false;
  std::string digits;  // magnitude digits, no leading zeros ("" == zero)
  int64_t exp10 = 0;   // value = digits * 10^exp10
};
bool parse_quantity(const std::string& s, Quantity* q);
int quantity_cmp(const Quantity& a, const Quantity& b);
std::string quantity_debug(const Quantity& q);

}  // namespace orc
