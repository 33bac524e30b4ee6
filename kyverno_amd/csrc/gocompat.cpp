// Go-compatible scalar conversions precomputed at ingest/compile time so the
// device compares canonical integers and bytes only:
//   strconv.FormatFloat(v,'E',-1,64)   pkg/engine/validate/pattern.go:228
//   fmt.Sprintf("%f", v)               pkg/engine/validate/common.go:18
//   strconv.ParseInt / ParseFloat      pkg/engine/validate/pattern.go:83,116
//   resource.ParseQuantity (k8s.io/apimachinery v0.21.4) -> canonical decimal
#include <algorithm>
#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "kvjson.hpp"

namespace kvh {

bool go_parse_int(std::string_view s, int64_t* out) {
  size_t k = 0, n = s.size();
  bool neg = false;
  if (k < n && (s[k] == '+' || s[k] == '-')) { neg = s[k] == '-'; k++; }
  if (k >= n) return false;
  uint64_t acc = 0;
  const uint64_t lim = neg ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1;
  for (; k < n; k++) {
    unsigned d = (unsigned)(s[k] - '0');
    if (d > 9) return false;
    if (acc > (lim - d) / 10) return false;
    acc = acc * 10 + d;
  }
  *out = neg ? (int64_t)(0 - acc) : (int64_t)acc;
  return true;
}

bool go_parse_float(std::string_view s, double* out) {
  size_t n = s.size();
  if (n == 0) return false;
  size_t k = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; k = 1; }
  // every form below starts with a digit, '.', "inf" / "infinity" or "nan" (any case): reject the
  // rest (most strings: image names, resource names) before building the copies
  if (k >= n) return false;
  const char c0 = s[k];
  if (!((c0 >= '0' && c0 <= '9') || c0 == '.' || c0 == 'i' || c0 == 'I' || c0 == 'n' || c0 == 'N')) return false;
  std::string rest(s.substr(k));
  std::string low = rest;
  for (auto& c : low) c = (char)tolower((unsigned char)c);
  if (low == "inf" || low == "infinity") { *out = neg ? -INFINITY : INFINITY; return true; }
  if (low == "nan") { *out = NAN; return true; }
  size_t j = 0, m = rest.size();
  bool hex = m >= 2 && rest[0] == '0' && (rest[1] == 'x' || rest[1] == 'X');
  bool digits = false, dot = false;
  if (hex) {
    for (j = 2; j < m; j++) {
      char c = rest[j];
      if (isxdigit((unsigned char)c)) digits = true;
      else if (c == '.' && !dot) dot = true;
      else break;
    }
    if (!digits || j >= m || (rest[j] != 'p' && rest[j] != 'P')) return false;
    j++;
    if (j < m && (rest[j] == '+' || rest[j] == '-')) j++;
    if (j >= m) return false;
    for (; j < m; j++)
      if (!isdigit((unsigned char)rest[j])) return false;
  } else {
    for (; j < m; j++) {
      char c = rest[j];
      if (c >= '0' && c <= '9') digits = true;
      else if (c == '.' && !dot) dot = true;
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
  char* e = nullptr;
  double d = strtod(rest.c_str(), &e);
  if (e != rest.c_str() + m) return false;
  if (errno == ERANGE && std::isinf(d)) return false;
  *out = neg ? -d : d;
  return true;
}

std::string go_format_E(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);
  std::string s(buf, r.ptr);
  // to_chars shortest scientific: d[.ddd]e±XX ; Go 'E': same digits, 'E', >= 2 exp digits
  size_t e = s.find('e');
  std::string mant = s.substr(0, e);
  if (mant.find('.') != std::string::npos) {
    while (mant.back() == '0') mant.pop_back();
    if (mant.back() == '.') mant.pop_back();
  }
  std::string ex = s.substr(e + 1);
  char sign = ex[0];
  std::string digs = ex.substr(1);
  while (digs.size() > 2 && digs[0] == '0') digs.erase(0, 1);
  if (digs.size() < 2) digs = "0" + digs;
  return mant + "E" + sign + digs;
}

// fmt's %v of a float64: strconv.FormatFloat(v, 'g', -1, 64) — shortest
// round-trip digits; strconv/ftoa.go %g rule with shortest precision: eprec = 6,
// exponent form when exp < -4 || exp >= eprec, exponent written e±dd.
std::string go_format_g(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  if (v == 0) return std::signbit(v) ? "-0" : "0";
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);
  std::string s(buf, r.ptr);
  bool neg = s[0] == '-';
  if (neg) s.erase(0, 1);
  size_t e = s.find('e');
  std::string digs;
  for (size_t i = 0; i < e; i++)
    if (s[i] != '.') digs += s[i];
  while (digs.size() > 1 && digs.back() == '0') digs.pop_back();
  const int exp = std::stoi(s.substr(e + 1));  // value = d.ddd x 10^exp
  const int nd = (int)digs.size(), dp = exp + 1;
  std::string out = neg ? "-" : "";
  if (exp < -4 || exp >= 6) {
    out += digs[0];
    if (nd > 1) { out += '.'; out += digs.substr(1); }
    out += 'e';
    out += exp < 0 ? '-' : '+';
    int ax = exp < 0 ? -exp : exp;
    if (ax < 10) out += '0';
    out += std::to_string(ax);
    return out;
  }
  if (dp <= 0) {
    out += "0.";
    out += std::string((size_t)-dp, '0');
    out += digs;
  } else if (dp >= nd) {
    out += digs;
    out += std::string((size_t)(dp - nd), '0');
  } else {
    out += digs.substr(0, (size_t)dp);
    out += '.';
    out += digs.substr((size_t)dp);
  }
  return out;
}

// encoding/json's float64 encoding (floatEncoder): strconv 'f' -1, or 'e' -1 when
// |v| < 1e-6 || |v| >= 1e21 (v != 0), with "e-0d" shortened to "e-d"
std::string go_json_float(double v) {
  const double a = std::fabs(v);
  if (a != 0 && (a < 1e-6 || a >= 1e21)) {
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);
    std::string s(buf, r.ptr);  // shortest d[.ddd]e±XX
    const size_t e = s.find('e');
    std::string ex = s.substr(e + 1);
    const char sign = ex[0];
    std::string digs = ex.substr(1);
    while (digs.size() > 2 && digs[0] == '0') digs.erase(0, 1);
    if (digs.size() < 2) digs = "0" + digs;
    if (sign == '-' && digs.size() == 2 && digs[0] == '0') digs.erase(0, 1);
    return s.substr(0, e) + "e" + sign + digs;
  }
  char buf[400];
  auto r = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::fixed);
  return std::string(buf, r.ptr);
}

std::string go_format_f6(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  char buf[400];
  snprintf(buf, sizeof buf, "%f", v);
  return buf;
}

bool utf8_ascii(std::string_view s) {
  for (unsigned char c : s)
    if (c >= 0x80) return false;
  return true;
}

// ---------------------------------------------------------------- quantity
namespace {

bool isd(char c) { return c >= '0' && c <= '9'; }

// Exact decimal: value = digits * 10^e (digits without leading zeros; "" == 0)
struct Dec {
  std::string d;
  int64_t e = 0;
  void norm() {
    size_t k = 0;
    while (k < d.size() && d[k] == '0') k++;
    d.erase(0, k);
    while (!d.empty() && d.back() == '0') { d.pop_back(); e++; }
    if (d.empty()) e = 0;
  }
};

int dec_mag_cmp(const Dec& a, const Dec& b) {
  if (a.d.empty() || b.d.empty()) return a.d.empty() ? (b.d.empty() ? 0 : -1) : 1;
  int64_t oa = (int64_t)a.d.size() + a.e, ob = (int64_t)b.d.size() + b.e;
  if (oa != ob) return oa < ob ? -1 : 1;
  size_t n = std::max(a.d.size(), b.d.size());
  for (size_t k = 0; k < n; k++) {
    char x = k < a.d.size() ? a.d[k] : '0', y = k < b.d.size() ? b.d[k] : '0';
    if (x != y) return x < y ? -1 : 1;
  }
  return 0;
}

std::string dmul2(const std::string& d) {
  std::string out;
  int carry = 0;
  for (size_t k = d.size(); k-- > 0;) {
    int v = (d[k] - '0') * 2 + carry;
    out.push_back((char)('0' + v % 10));
    carry = v / 10;
  }
  if (carry) out.push_back((char)('0' + carry));
  std::reverse(out.begin(), out.end());
  return out;
}

std::string dinc(std::string d) {
  size_t k = d.size();
  while (k > 0) {
    k--;
    if (d[k] == '9') { d[k] = '0'; continue; }
    d[k]++;
    return d;
  }
  return "1" + d;
}

// Returns false if not a quantity. On success sets neg and magnitude.
bool quantity(std::string_view str, bool* neg, Dec* mag) {
  *neg = false;
  *mag = Dec();
  if (str.empty()) return false;
  if (str == "0") return true;
  // parseQuantityString
  bool positive = true;
  size_t pos = 0, end = str.size();
  if (str[0] == '-') { positive = false; pos++; }
  else if (str[0] == '+') pos++;
  std::string_view value, num, denom, suffix;
  bool done = false;
  for (size_t i = pos;; i++) {
    if (i >= end) { num = "0"; value = num; done = true; break; }
    if (str[i] == '0') pos++;
    else break;
  }
  if (!done) {
    size_t i = pos;
    for (;; i++) {
      if (i >= end) { num = str.substr(pos, end - pos); value = str.substr(0, end); done = true; break; }
      if (!isd(str[i])) { num = str.substr(pos, i - pos); pos = i; break; }
    }
  }
  if (!done) {
    if (num.empty()) num = "0";
    if (pos < end && str[pos] == '.') {
      pos++;
      size_t i = pos;
      for (;; i++) {
        if (i >= end) { denom = str.substr(pos, end - pos); value = str.substr(0, end); done = true; break; }
        if (!isd(str[i])) { denom = str.substr(pos, i - pos); pos = i; break; }
      }
    }
  }
  if (!done) {
    value = str.substr(0, pos);
    size_t ss = pos;
    bool ended = false;
    for (size_t i = pos;; i++) {
      if (i >= end) { suffix = str.substr(ss, end - ss); ended = true; break; }
      if (!strchr("eEinumkKMGTP", str[i])) { pos = i; break; }
    }
    if (!ended) {
      if (pos < end && (str[pos] == '-' || str[pos] == '+')) pos++;
      for (size_t i = pos;; i++) {
        if (i >= end) { suffix = str.substr(ss, end - ss); ended = true; break; }
        if (!isd(str[i])) break;
      }
      if (!ended) return false;  // ErrFormatWrong
    }
  }
  // interpret suffix
  int base = 0, exponent = 0;
  int fmt = 0;  // 0 DecimalExponent, 1 BinarySI, 2 DecimalSI
  static const char* ds[] = {"n", "u", "m", "", "k", "M", "G", "T", "P", "E"};
  static const int de[] = {-9, -6, -3, 0, 3, 6, 9, 12, 15, 18};
  static const char* bs[] = {"Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
  bool found = false;
  for (int k = 0; k < 10 && !found; k++)
    if (suffix == ds[k]) { base = 10; exponent = de[k]; fmt = 2; found = true; }
  for (int k = 0; k < 6 && !found; k++)
    if (suffix == bs[k]) { base = 2; exponent = 10 * (k + 1); fmt = 1; found = true; }
  if (!found) {
    if (suffix.size() > 1 && (suffix[0] == 'E' || suffix[0] == 'e')) {
      int64_t v;
      if (!go_parse_int(suffix.substr(1), &v)) return false;
      base = 10;
      exponent = (int32_t)v;
      fmt = 0;
    } else {
      return false;
    }
  }
  int precision = 0, scale = 0;
  int64_t mantissa = 1;
  if (fmt != 1) {
    scale = exponent;
    precision = 18 - (int)(num.size() + denom.size());
  } else {
    if (exponent >= 0 && denom.empty()) {
      mantissa = (int64_t)1 << exponent;
      precision = 15 - (int)num.size() - (int)((float)exponent * 3 / 10) - 1;
    } else {
      precision = -1;
    }
  }
  if (precision >= 0) {
    scale -= (int)denom.size();
    if (scale >= -9) {
      std::string shifted = std::string(num) + std::string(denom);
      int64_t v;
      if (!go_parse_int(shifted, &v)) return false;
      __int128 r = (__int128)v * mantissa;
      if (r <= (__int128)INT64_MAX && r >= (__int128)INT64_MIN) {
        int64_t res = (int64_t)r;
        if (!positive) res = -res;
        uint64_t m = res < 0 ? (uint64_t)(-(__int128)res) : (uint64_t)res;
        mag->d = m ? std::to_string(m) : "";
        mag->e = scale;
        mag->norm();
        *neg = res < 0;
        return true;
      }
    }
  }
  // slow path: inf.Dec over `value`
  std::string digs;
  bool vneg = false;
  int dp = -1;
  bool anyd = false;
  for (size_t k = 0; k < value.size(); k++) {
    char c = value[k];
    if (c == '+' || c == '-') {
      if (!digs.empty() || dp >= 0) return false;
      vneg = c == '-';
    } else if (c == '.') {
      if (dp >= 0) return false;
      dp = (int)digs.size();
    } else if (isd(c)) {
      digs.push_back(c);
      anyd = true;
    } else {
      return false;
    }
  }
  if (!anyd) return false;
  Dec m;
  m.d = digs;
  m.e = dp >= 0 ? -((int64_t)digs.size() - dp) : 0;
  if (base == 10) m.e += exponent;
  else for (int k = 0; k < exponent; k++) m.d = dmul2(m.d);
  m.norm();
  if (!m.d.empty() && m.e < -9) {  // round magnitude up to nano
    int64_t cut = -9 - m.e;
    std::string keep, drop;
    if ((int64_t)m.d.size() > cut) { keep = m.d.substr(0, m.d.size() - cut); drop = m.d.substr(m.d.size() - cut); }
    else { keep = "0"; drop = m.d; }
    if (drop.find_first_not_of('0') != std::string::npos) keep = dinc(keep);
    m.d = keep;
    m.e = -9;
    m.norm();
  }
  Dec mx;
  mx.d = "9223372036854775807";
  if (dec_mag_cmp(m, mx) > 0) m = mx;
  *neg = vneg && !m.d.empty();
  *mag = m;
  return true;
}

}  // namespace

QCanon parse_quantity(std::string_view s) {
  QCanon q;
  bool neg;
  Dec m;
  if (!quantity(s, &neg, &m)) return q;
  q.valid = true;
  if (m.d.empty()) { q.zero = true; return q; }
  q.neg = neg;
  q.exp = (int32_t)std::max<int64_t>(std::min<int64_t>((int64_t)m.d.size() + m.e, INT32_MAX), INT32_MIN);
  std::string d = m.d;
  if (d.size() > 38) d.resize(38);  // cannot happen for k8s quantities (<= 28 significant digits)
  d.resize(38, '0');
  q.hi = std::stoull(d.substr(0, 19));
  q.lo = std::stoull(d.substr(19, 19));
  return q;
}

}  // namespace kvh
