// ORACLE — test infrastructure only (see ovalue.hpp header).
// Restatement of k8s.io/apimachinery v0.21.4 (go.mod:46; not vendored under
// /root/reference) api/resource: ParseQuantity / parseQuantityString /
// suffixHandler.interpret / Quantity.Cmp, as called from
// pkg/engine/validate/pattern.go:264-309 (validateNumberWithStr, compareQuantity).
// Exact decimal arithmetic on digit strings; the value of a Quantity is
// sign * digits * 10^exp10. Pinned by pkg/engine/validate/pattern_test.go:313-379.
#include <cstring>

#include "ovalue.hpp"

namespace orc {

namespace {

bool is_digit(char c) { return c >= '0' && c <= '9'; }

// parseQuantityString (quantity.go). Returns false on ErrFormatWrong.
bool parse_quantity_string(const std::string& str, bool* positive, std::string* value,
                           std::string* num, std::string* denom, std::string* suffix) {
  *positive = true;
  size_t pos = 0, end = str.size();
  if (pos < end) {
    if (str[0] == '-') { *positive = false; pos++; }
    else if (str[0] == '+') { pos++; }
  }
  // strip leading zeros
  for (size_t i = pos;; i++) {
    if (i >= end) { *num = "0"; *value = *num; return true; }
    if (str[i] == '0') pos++;
    else break;
  }
  // numerator
  for (size_t i = pos;; i++) {
    if (i >= end) { *num = str.substr(pos, end - pos); *value = str.substr(0, end); return true; }
    if (!is_digit(str[i])) { *num = str.substr(pos, i - pos); pos = i; break; }
  }
  if (num->empty()) *num = "0";
  // denominator
  if (pos < end && str[pos] == '.') {
    pos++;
    for (size_t i = pos;; i++) {
      if (i >= end) { *denom = str.substr(pos, end - pos); *value = str.substr(0, end); return true; }
      if (!is_digit(str[i])) { *denom = str.substr(pos, i - pos); pos = i; break; }
    }
  }
  *value = str.substr(0, pos);
  size_t suffix_start = pos;
  for (size_t i = pos;; i++) {
    if (i >= end) { *suffix = str.substr(suffix_start, end - suffix_start); return true; }
    if (!strchr("eEinumkKMGTP", str[i])) { pos = i; break; }
  }
  if (pos < end && (str[pos] == '-' || str[pos] == '+')) pos++;
  for (size_t i = pos;; i++) {
    if (i >= end) { *suffix = str.substr(suffix_start, end - suffix_start); return true; }
    if (!is_digit(str[i])) break;
  }
  return false;  // ErrFormatWrong
}

enum Fmt { DecimalExponent, BinarySI, DecimalSI };

bool interpret(const std::string& s, int* base, int* exponent, Fmt* fmt) {
  static const struct { const char* s; int e; } dec[] = {
      {"n", -9}, {"u", -6}, {"m", -3}, {"", 0}, {"k", 3}, {"M", 6}, {"G", 9}, {"T", 12}, {"P", 15}, {"E", 18}};
  static const struct { const char* s; int e; } bin[] = {
      {"Ki", 10}, {"Mi", 20}, {"Gi", 30}, {"Ti", 40}, {"Pi", 50}, {"Ei", 60}};
  for (auto& d : dec)
    if (s == d.s) { *base = 10; *exponent = d.e; *fmt = DecimalSI; return true; }
  for (auto& b : bin)
    if (s == b.s) { *base = 2; *exponent = b.e; *fmt = BinarySI; return true; }
  if (s.size() > 1 && (s[0] == 'E' || s[0] == 'e')) {
    int64_t v;
    if (!go_parse_int(s.substr(1), &v)) return false;
    *base = 10;
    *exponent = (int)(int32_t)v;  // int32(parsed)
    *fmt = DecimalExponent;
    return true;
  }
  return false;
}

std::string strip_lead(const std::string& d) {
  size_t k = 0;
  while (k < d.size() && d[k] == '0') k++;
  return d.substr(k);
}

void normalize(Quantity* q) {
  q->digits = strip_lead(q->digits);
  while (!q->digits.empty() && q->digits.back() == '0') { q->digits.pop_back(); q->exp10++; }
  if (q->digits.empty()) { q->neg = false; q->exp10 = 0; }
}

std::string mul_small(const std::string& d, int m) {
  std::string out(d.size() + 4, '0');
  int carry = 0;
  size_t o = out.size();
  for (size_t k = d.size(); k-- > 0;) {
    int v = (d[k] - '0') * m + carry;
    out[--o] = (char)('0' + v % 10);
    carry = v / 10;
  }
  while (carry) { out[--o] = (char)('0' + carry % 10); carry /= 10; }
  return strip_lead(out);
}

std::string add_one(const std::string& d) {
  std::string out = d;
  size_t k = out.size();
  while (k > 0) {
    k--;
    if (out[k] == '9') { out[k] = '0'; continue; }
    out[k]++;
    return out;
  }
  return "1" + out;
}

// magnitude compare of normalized quantities
int mag_cmp(const Quantity& a, const Quantity& b) {
  if (a.digits.empty() && b.digits.empty()) return 0;
  if (a.digits.empty()) return -1;
  if (b.digits.empty()) return 1;
  int64_t oa = (int64_t)a.digits.size() + a.exp10, ob = (int64_t)b.digits.size() + b.exp10;
  if (oa != ob) return oa < ob ? -1 : 1;
  size_t n = std::max(a.digits.size(), b.digits.size());
  for (size_t k = 0; k < n; k++) {
    char ca = k < a.digits.size() ? a.digits[k] : '0';
    char cb = k < b.digits.size() ? b.digits[k] : '0';
    if (ca != cb) return ca < cb ? -1 : 1;
  }
  return 0;
}

}  // namespace

bool parse_quantity(const std::string& str, Quantity* q) {
  *q = Quantity();
  if (str.empty()) return false;
  if (str == "0") return true;
  bool positive;
  std::string value, num, denom, suf;
  if (!parse_quantity_string(str, &positive, &value, &num, &denom, &suf)) return false;
  int base = 0, exponent = 0;
  Fmt format;
  if (!interpret(suf, &base, &exponent, &format)) return false;

  const int maxInt64Factors = 18;
  int precision = 0, scale = 0;
  int64_t mantissa = 1;
  if (format == DecimalExponent || format == DecimalSI) {
    scale = exponent;
    precision = maxInt64Factors - (int)(num.size() + denom.size());
  } else {
    scale = 0;
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
      std::string shifted = num + denom;
      int64_t v;
      if (!go_parse_int(shifted, &v)) return false;  // ErrNumeric
      __int128 r = (__int128)v * mantissa;
      if (r <= (__int128)INT64_MAX && r >= (__int128)INT64_MIN) {
        int64_t res = (int64_t)r;
        if (!positive) res = -res;
        q->neg = res < 0;
        unsigned __int128 mag = res < 0 ? (unsigned __int128)(-(__int128)res) : (unsigned __int128)res;
        std::string d;
        if (mag == 0) d = "";
        else {
          while (mag) { d.insert(d.begin(), (char)('0' + (int)(mag % 10))); mag /= 10; }
        }
        q->digits = d;
        q->exp10 = scale;
        normalize(q);
        return true;
      }
    }
  }
  // Slow path: inf.Dec from `value`.
  {
    size_t k = 0;
    bool neg = false;
    std::string digs;
    int dp = -1, dg = -1;
    for (; k < value.size(); k++) {
      char c = value[k];
      if (c == '+' || c == '-') {
        if (!digs.empty() || dp >= 0) break;
        neg = c == '-';
        continue;  // sign is not a digit
      } else if (c == '.') {
        if (dp >= 0) break;
        dp = (int)digs.size();
        continue;
      } else if (is_digit(c)) {
        if (dg == -1) dg = (int)digs.size();
      } else {
        break;
      }
      digs.push_back(c);
    }
    if (k != value.size() || dg == -1) return false;  // ErrNumeric
    int64_t s = dp >= 0 ? (int64_t)digs.size() - dp : 0;  // inf scale
    std::string D = strip_lead(digs);
    int64_t e10 = -s;
    if (base == 10) {
      e10 += exponent;
    } else if (base == 2) {
      for (int j = 0; j < exponent; j++) D = mul_small(D, 2);
    }
    Quantity m;
    m.neg = false;
    m.digits = D;
    m.exp10 = e10;
    if (!strip_lead(D).empty()) {
      // Round up (away from zero) to nano scale.
      if (m.exp10 < -9) {
        int64_t cut = -9 - m.exp10;
        std::string keep, dropped;
        if ((int64_t)m.digits.size() > cut) {
          keep = m.digits.substr(0, m.digits.size() - cut);
          dropped = m.digits.substr(m.digits.size() - cut);
        } else {
          keep = "";
          dropped = m.digits;
        }
        bool nz = dropped.find_first_not_of('0') != std::string::npos;
        if (keep.empty()) keep = "0";
        if (nz) keep = add_one(keep);
        m.digits = keep;
        m.exp10 = -9;
      }
    }
    normalize(&m);
    Quantity maxq;
    maxq.digits = "9223372036854775807";
    maxq.exp10 = 0;
    normalize(&maxq);
    if (mag_cmp(m, maxq) > 0) m = maxq;
    m.neg = neg && !m.digits.empty();
    *q = m;
    return true;
  }
}

int quantity_cmp(const Quantity& a, const Quantity& b) {
  bool az = a.digits.empty(), bz = b.digits.empty();
  int sa = az ? 0 : (a.neg ? -1 : 1), sb = bz ? 0 : (b.neg ? -1 : 1);
  if (sa != sb) return sa < sb ? -1 : 1;
  if (sa == 0) return 0;
  int m = mag_cmp(a, b);
  return sa > 0 ? m : -m;
}

std::string quantity_debug(const Quantity& q) {
  if (q.digits.empty()) return "0";
  return std::string(q.neg ? "-" : "") + q.digits + "e" + std::to_string(q.exp10);
}

}  // namespace orc
