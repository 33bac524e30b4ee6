// ORACLE — test infrastructure only (see ovalue.hpp header).
// Restatement of github.com/minio/pkg v1.1.3 wildcard.Match (go.mod:28; not
// vendored under /root/reference). Published algorithm: Match(pattern, name):
//   pattern == "" -> name == "";  pattern == "*" -> true;
//   otherwise deepMatchRune([]rune(name), []rune(pattern), simple=false):
//   '*' matches any run of runes (including empty), '?' exactly one rune,
//   every other rune literally; the whole name must be consumed.
// Call sites: pkg/engine/validate/pattern.go:250,284; pkg/engine/utils.go:59,69,85;
// pkg/engine/wildcards/wildcards.go:40,43. The recursive backtracking of the
// reference is replaced here by the equivalent iterative star-backtrack walk.
// Pinned by pkg/engine/validate/pattern_test.go:19-59 and wildcards tests.
#include "ovalue.hpp"

namespace orc {

namespace {
std::vector<uint32_t> runes(const std::string& s) {
  std::vector<uint32_t> out;
  const unsigned char* p = (const unsigned char*)s.data();
  size_t n = s.size(), k = 0;
  while (k < n) {
    unsigned c = p[k];
    if (c < 0x80) { out.push_back(c); k++; continue; }
    // decode; invalid -> U+FFFD width 1 (Go []rune conversion)
    uint32_t cp = 0xFFFD;
    size_t w = 1;
    auto cont = [&](size_t j) { return k + j < n && (p[k + j] & 0xC0) == 0x80; };
    if (c >= 0xC2 && c <= 0xDF && cont(1)) { cp = ((c & 0x1F) << 6) | (p[k + 1] & 0x3F); w = 2; }
    else if (c >= 0xE0 && c <= 0xEF && k + 1 < n) {
      unsigned c1 = p[k + 1];
      bool ok = (c == 0xE0) ? (c1 >= 0xA0 && c1 <= 0xBF) : (c == 0xED) ? (c1 >= 0x80 && c1 <= 0x9F) : (c1 >= 0x80 && c1 <= 0xBF);
      if (ok && cont(2)) { cp = ((c & 0x0F) << 12) | ((c1 & 0x3F) << 6) | (p[k + 2] & 0x3F); w = 3; }
    } else if (c >= 0xF0 && c <= 0xF4 && k + 1 < n) {
      unsigned c1 = p[k + 1];
      bool ok = (c == 0xF0) ? (c1 >= 0x90 && c1 <= 0xBF) : (c == 0xF4) ? (c1 >= 0x80 && c1 <= 0x8F) : (c1 >= 0x80 && c1 <= 0xBF);
      if (ok && cont(2) && cont(3)) { cp = ((c & 0x07) << 18) | ((c1 & 0x3F) << 12) | ((p[k + 2] & 0x3F) << 6) | (p[k + 3] & 0x3F); w = 4; }
    }
    out.push_back(cp);
    k += w;
  }
  return out;
}
}  // namespace

bool wildcard_match(const std::string& pattern, const std::string& name) {
  if (pattern.empty()) return name.empty();
  if (pattern == "*") return true;
  std::vector<uint32_t> s = runes(name), p = runes(pattern);
  size_t si = 0, pi = 0, star = (size_t)-1, mark = 0;
  while (si < s.size()) {
    if (pi < p.size() && p[pi] == '*') {
      star = pi++;
      mark = si;
    } else if (pi < p.size() && (p[pi] == '?' || p[pi] == s[si])) {
      pi++;
      si++;
    } else if (star != (size_t)-1) {
      pi = star + 1;
      si = ++mark;
    } else {
      return false;
    }
  }
  while (pi < p.size() && p[pi] == '*') pi++;
  return pi == p.size();
}

}  // namespace orc
