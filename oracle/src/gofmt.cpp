// ORACLE — test infrastructure only (see ovalue.hpp header).
// Restatements of the Go stdlib formatting/parsing the reference path relies on:
//   strconv.FormatFloat(v,'E',-1,64)  (pkg/engine/validate/pattern.go:228)
//   fmt.Sprintf("%f", v)              (pkg/engine/validate/common.go:18)
//   fmt %v / %T of interface{} values (pkg/engine/validate/validate.go:83,89)
//   strconv.ParseFloat / ParseInt     (pkg/engine/validate/pattern.go:83,116)
#include <algorithm>
#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "ovalue.hpp"

namespace orc {

namespace {

// Shortest round-trip decimal digits of |v| (v finite, nonzero) and the decimal
// point position dp such that value = 0.d1d2d3... * 10^dp.
void shortest_digits(double v, std::string* digits, int* dp) {
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof buf, std::fabs(v), std::chars_format::scientific);
  std::string s(buf, r.ptr);
  size_t e = s.find('e');
  std::string mant = s.substr(0, e);
  int ex = atoi(s.c_str() + e + 1);
  std::string d;
  for (char c : mant)
    if (c != '.') d.push_back(c);
  while (d.size() > 1 && d.back() == '0') d.pop_back();
  *digits = d;
  *dp = ex + 1;
}

std::string fmt_e(bool neg, const std::string& d, int dp, char echar) {
  // %e with all digits of d: d0.d1d2...e±XX
  std::string out;
  if (neg) out.push_back('-');
  out.push_back(d.empty() ? '0' : d[0]);
  if (d.size() > 1) {
    out.push_back('.');
    out.append(d.begin() + 1, d.end());
  }
  out.push_back(echar);
  int ex = d.empty() ? 0 : dp - 1;
  if (ex < 0) { out.push_back('-'); ex = -ex; } else out.push_back('+');
  char b[16];
  if (ex < 10) snprintf(b, sizeof b, "0%d", ex);
  else snprintf(b, sizeof b, "%d", ex);
  out += b;
  return out;
}

std::string fmt_f(bool neg, const std::string& d, int dp) {
  // %f with max(nd-dp,0) decimals, digits d (no rounding needed: exact digits)
  std::string out;
  if (neg) out.push_back('-');
  int nd = (int)d.size();
  if (dp > 0) {
    for (int k = 0; k < dp; k++) out.push_back(k < nd ? d[k] : '0');
  } else {
    out.push_back('0');
  }
  int frac = std::max(nd - dp, 0);
  if (frac > 0) {
    out.push_back('.');
    for (int k = 0; k < frac; k++) {
      int idx = dp + k;
      out.push_back(idx >= 0 && idx < nd ? d[idx] : '0');
    }
  }
  return out;
}

}  // namespace

std::string go_format_E(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  bool neg = std::signbit(v);
  if (v == 0) return neg ? "-0E+00" : "0E+00";
  std::string d;
  int dp;
  shortest_digits(v, &d, &dp);
  return fmt_e(neg, d, dp, 'E');
}

std::string go_format_f6(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  char buf[512];
  snprintf(buf, sizeof buf, "%f", v);
  return buf;
}

std::string go_format_g(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  bool neg = std::signbit(v);
  if (v == 0) return neg ? "-0" : "0";
  std::string d;
  int dp;
  shortest_digits(v, &d, &dp);
  int ex = dp - 1;
  if (ex < -4 || ex >= 6 /* eprec = 6 when shortest */) return fmt_e(neg, d, dp, 'e');
  return fmt_f(neg, d, dp);
}

std::string go_type_name(const Value* v) {
  if (!v) return "<nil>";
  switch (v->t) {
    case T::Null: return "<nil>";
    case T::Bool: return "bool";
    case T::Int: return "int64";
    case T::Float: return "float64";
    case T::Str: return "string";
    case T::Map: return "map[string]interface {}";
    case T::Arr: return "[]interface {}";
  }
  return "?";
}

std::string go_format_v(const Value* v) {
  if (!v) return "<nil>";
  switch (v->t) {
    case T::Null: return "<nil>";
    case T::Bool: return v->b ? "true" : "false";
    case T::Int: return std::to_string(v->i);
    case T::Float: return go_format_g(v->f);
    case T::Str: return v->s;
    case T::Map: {
      std::vector<const Value::Entry*> es;
      for (const auto& e : v->m) es.push_back(&e);
      std::sort(es.begin(), es.end(), [](const Value::Entry* x, const Value::Entry* y) { return x->key < y->key; });
      std::string out = "map[";
      for (size_t k = 0; k < es.size(); k++) {
        if (k) out.push_back(' ');
        out += es[k]->key;
        out.push_back(':');
        out += go_format_v(es[k]->val);
      }
      out.push_back(']');
      return out;
    }
    case T::Arr: {
      std::string out = "[";
      for (size_t k = 0; k < v->a.size(); k++) {
        if (k) out.push_back(' ');
        out += go_format_v(v->a[k]);
      }
      out.push_back(']');
      return out;
    }
  }
  return "?";
}

bool go_parse_int(const std::string& s, int64_t* out) {
  size_t k = 0, n = s.size();
  bool neg = false;
  if (k < n && (s[k] == '+' || s[k] == '-')) { neg = s[k] == '-'; k++; }
  if (k >= n) return false;
  unsigned __int128 acc = 0;
  for (; k < n; k++) {
    char c = s[k];
    if (c < '0' || c > '9') return false;
    acc = acc * 10 + (unsigned)(c - '0');
    if (acc > ((unsigned __int128)1 << 64)) return false;
  }
  if (neg) {
    if (acc > ((unsigned __int128)1 << 63)) return false;
    *out = (int64_t)(-(__int128)acc);
  } else {
    if (acc > (((unsigned __int128)1 << 63) - 1)) return false;
    *out = (int64_t)acc;
  }
  return true;
}

bool go_parse_float(const std::string& s, double* out) {
  size_t k = 0, n = s.size();
  if (n == 0) return false;
  bool neg = false;
  if (s[k] == '+' || s[k] == '-') { neg = s[k] == '-'; k++; }
  std::string rest = s.substr(k);
  std::string low;
  for (char c : rest) low.push_back((char)tolower((unsigned char)c));
  if (low == "inf" || low == "infinity") { *out = neg ? -INFINITY : INFINITY; return true; }
  if (low == "nan") { *out = NAN; return true; }
  // syntax check
  size_t j = 0, m = rest.size();
  bool hex = m >= 2 && rest[0] == '0' && (rest[1] == 'x' || rest[1] == 'X');
  if (hex) {
    j = 2;
    bool digits = false, sawdot = false;
    for (; j < m; j++) {
      char c = rest[j];
      if (isxdigit((unsigned char)c)) digits = true;
      else if (c == '.' && !sawdot) sawdot = true;
      else break;
    }
    if (!digits) return false;
    if (j >= m || (rest[j] != 'p' && rest[j] != 'P')) return false;
    j++;
    if (j < m && (rest[j] == '+' || rest[j] == '-')) j++;
    if (j >= m) return false;
    for (; j < m; j++)
      if (!isdigit((unsigned char)rest[j])) return false;
  } else {
    bool digits = false, sawdot = false;
    for (; j < m; j++) {
      char c = rest[j];
      if (c >= '0' && c <= '9') digits = true;
      else if (c == '.' && !sawdot) sawdot = true;
      else break;
    }
    if (!digits) return false;
    if (j < m && (rest[j] == 'e' || rest[j] == 'E')) {
      j++;
      if (j < m && (rest[j] == '+' || rest[j] == '-')) j++;
      if (j >= m) return false;
      for (; j < m; j++)
        if (!isdigit((unsigned char)rest[j])) return false;
    }
    if (j != m) return false;
  }
  errno = 0;
  char* endp = nullptr;
  double d = strtod(rest.c_str(), &endp);
  if (endp != rest.c_str() + rest.size()) return false;
  if (errno == ERANGE && std::isinf(d)) return false;
  *out = neg ? -d : d;
  return true;
}

}  // namespace orc
