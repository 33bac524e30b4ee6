// Arena JSON parser (see kvjson.hpp).
#include "kvjson.hpp"

#include <algorithm>
#include <cstring>
#include <emmintrin.h>

namespace kvh {

namespace {

// UTF-8 bytes of code point cp at out (returns the count, 1..4)
inline size_t put_utf8(char* out, uint32_t cp) {
  if (cp < 0x80) {
    out[0] = (char)cp;
    return 1;
  } else if (cp < 0x800) {
    out[0] = (char)(0xC0 | (cp >> 6));
    out[1] = (char)(0x80 | (cp & 0x3F));
    return 2;
  } else if (cp < 0x10000) {
    out[0] = (char)(0xE0 | (cp >> 12));
    out[1] = (char)(0x80 | ((cp >> 6) & 0x3F));
    out[2] = (char)(0x80 | (cp & 0x3F));
    return 3;
  }
  out[0] = (char)(0xF0 | (cp >> 18));
  out[1] = (char)(0x80 | ((cp >> 12) & 0x3F));
  out[2] = (char)(0x80 | ((cp >> 6) & 0x3F));
  out[3] = (char)(0x80 | (cp & 0x3F));
  return 4;
}

// Width of a valid UTF-8 sequence at p (1..4), or 0 if invalid.
inline size_t valid_utf8(const unsigned char* p, size_t n) {
  unsigned c = p[0];
  if (c < 0x80) return 1;
  auto cont = [&](size_t k) { return k < n && (p[k] & 0xC0) == 0x80; };
  if (c >= 0xC2 && c <= 0xDF) return cont(1) ? 2 : 0;
  if (c >= 0xE0 && c <= 0xEF) {
    if (n < 2) return 0;
    unsigned c1 = p[1];
    bool ok = c == 0xE0 ? (c1 >= 0xA0 && c1 <= 0xBF) : c == 0xED ? (c1 >= 0x80 && c1 <= 0x9F) : (c1 >= 0x80 && c1 <= 0xBF);
    return ok && cont(2) ? 3 : 0;
  }
  if (c >= 0xF0 && c <= 0xF4) {
    if (n < 2) return 0;
    unsigned c1 = p[1];
    bool ok = c == 0xF0 ? (c1 >= 0x90 && c1 <= 0xBF) : c == 0xF4 ? (c1 >= 0x80 && c1 <= 0x8F) : (c1 >= 0x80 && c1 <= 0xBF);
    return ok && cont(2) && cont(3) ? 4 : 0;
  }
  return 0;
}

struct P {
  const char* s;
  size_t n;
  size_t i = 0;
  NumMode mode;
  JDoc* d;
  std::vector<JNode>& scratch;  // children staging (stack discipline), reused per thread
  // decoded string bytes go to d->strs[o..] through a raw cursor (strs is kept longer than
  // o and grown on demand; parse_one trims it to o at the end)
  char* sb = nullptr;
  size_t o = 0;
  inline void room(size_t k) {
    if (o + k > d->strs.size()) {
      d->strs.resize(std::max(2 * d->strs.size(), o + k + 256));
      sb = &d->strs[0];
    }
  }
  inline void put1(char c) { room(1); sb[o++] = c; }
  inline void putn(const char* p, size_t k) { room(k); memcpy(sb + o, p, k); o += k; }

  [[noreturn]] void fail(const char* w) { throw std::runtime_error(std::string("json: ") + w); }
  inline void ws() {
    while (i < n) {
      char c = s[i];
      if (c == ' ' || c == '\n' || c == '\r' || c == '\t') i++;
      else break;
    }
  }
  uint32_t hex4() {
    if (n - i < 4) fail("bad \\u");
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) {
      char c = s[i + k];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex");
    }
    i += 4;
    return v;
  }
  // appends decoded string to d->strs, returns (off, len)
  void str(uint32_t* off, uint32_t* len) {
    if (i >= n || s[i] != '"') fail("expected string");
    i++;
    const size_t start = o;
    // fast path: plain ASCII run (16 bytes per step: quote, backslash, control or non-ASCII)
    while (true) {
      size_t j = i;
      const __m128i q = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\'), lim = _mm_set1_epi8(0x20);
      while (j + 16 <= n) {
        const __m128i x = _mm_loadu_si128((const __m128i*)(s + j));
        // c < 0x20 or c >= 0x80: one signed compare, c < 0x20 as signed bytes, covers both
        const __m128i stop = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(x, q), _mm_cmpeq_epi8(x, bs)),
                                          _mm_cmpgt_epi8(lim, x));
        const int m = _mm_movemask_epi8(stop);
        if (m) { j += (size_t)__builtin_ctz((unsigned)m); goto found; }
        j += 16;
      }
      while (j < n) {
        unsigned char c = (unsigned char)s[j];
        if (c == '"' || c == '\\' || c < 0x20 || c >= 0x80) break;
        j++;
      }
    found:
      putn(s + i, j - i);
      i = j;
      if (i >= n) fail("unterminated string");
      unsigned char c = (unsigned char)s[i];
      if (c == '"') { i++; break; }
      if (c < 0x20) fail("control character in string");
      if (c == '\\') {
        i++;
        if (i >= n) fail("bad escape");
        char e = s[i++];
        switch (e) {
          case '"': put1('"'); break;
          case '\\': put1('\\'); break;
          case '/': put1('/'); break;
          case 'b': put1('\b'); break;
          case 'f': put1('\f'); break;
          case 'n': put1('\n'); break;
          case 'r': put1('\r'); break;
          case 't': put1('\t'); break;
          case 'u': {
            uint32_t cp = hex4();
            if (cp >= 0xD800 && cp < 0xDC00) {
              if (n - i >= 6 && s[i] == '\\' && s[i + 1] == 'u') {
                size_t save = i;
                i += 2;
                uint32_t lo = hex4();
                if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                else { i = save; cp = 0xFFFD; }
              } else {
                cp = 0xFFFD;
              }
            } else if (cp >= 0xDC00 && cp < 0xE000) {
              cp = 0xFFFD;
            }
            room(4);
            o += put_utf8(sb + o, cp);
            break;
          }
          default: fail("bad escape");
        }
        continue;
      }
      // non-ASCII
      size_t w = valid_utf8((const unsigned char*)s + i, n - i);
      if (w == 0) { room(4); o += put_utf8(sb + o, 0xFFFD); i++; }
      else { putn(s + i, w); i += w; }
    }
    *off = (uint32_t)start;
    *len = (uint32_t)(o - start);
  }
  void num(JNode& v) {
    size_t st = i;
    if (i < n && s[i] == '-') i++;
    if (i >= n) fail("bad number");
    if (s[i] == '0') i++;
    else if (s[i] >= '1' && s[i] <= '9') { while (i < n && s[i] >= '0' && s[i] <= '9') i++; }
    else fail("bad number");
    bool isint = true;
    if (i < n && s[i] == '.') {
      isint = false;
      i++;
      if (i >= n || s[i] < '0' || s[i] > '9') fail("bad fraction");
      while (i < n && s[i] >= '0' && s[i] <= '9') i++;
    }
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
      isint = false;
      i++;
      if (i < n && (s[i] == '+' || s[i] == '-')) i++;
      if (i >= n || s[i] < '0' || s[i] > '9') fail("bad exponent");
      while (i < n && s[i] >= '0' && s[i] <= '9') i++;
    }
    std::string_view lit(s + st, i - st);
    if (mode == NUM_UNSTRUCTURED && isint) {
      int64_t iv;
      if (go_parse_int(lit, &iv)) { v.t = J_INT; v.i = iv; return; }
    }
    double f;
    if (!go_parse_float(lit, &f)) fail("number out of range");
    v.t = J_FLOAT;
    v.f = f;
  }
  // parse a value into `v` (children placed into d->nodes)
  void value(JNode& v, int depth) {
    if (depth > 2000) fail("nesting too deep");
    ws();
    if (i >= n) fail("unexpected end");
    char c = s[i];
    if (c == '{') {
      i++;
      v.t = J_MAP;
      size_t base = scratch.size();
      ws();
      if (i < n && s[i] == '}') { i++; v.first = (uint32_t)d->nodes.size(); v.count = 0; return; }
      uint64_t seen = 0;  // keys of this map so far by (length, first byte, last byte) signature bit
      while (true) {
        ws();
        JNode ch;
        str(&ch.key_off, &ch.key_len);
        ws();
        if (i >= n || s[i] != ':') fail("expected :");
        i++;
        value(ch, depth + 1);
        // duplicate key: last one wins (replace in place); the earlier keys are compared only
        // when one of them has the same signature
        const std::string_view k(sb + ch.key_off, ch.key_len);
        const uint64_t sig = 1ull << ((k.size() * 7u + (k.empty() ? 0u : (unsigned char)k[0] * 3u +
                                                                        (unsigned char)k.back())) & 63u);
        bool dup = false;
        if (seen & sig)
          for (size_t q = base; q < scratch.size(); q++) {
            if (std::string_view(sb + scratch[q].key_off, scratch[q].key_len) == k) { scratch[q] = ch; dup = true; break; }
          }
        seen |= sig;
        if (!dup) scratch.push_back(ch);
        ws();
        if (i < n && s[i] == ',') { i++; continue; }
        if (i < n && s[i] == '}') { i++; break; }
        fail("expected , or }");
      }
      v.first = (uint32_t)d->nodes.size();
      v.count = (uint32_t)(scratch.size() - base);
      d->nodes.insert(d->nodes.end(), scratch.begin() + base, scratch.end());
      scratch.resize(base);
      return;
    }
    if (c == '[') {
      i++;
      v.t = J_ARR;
      size_t base = scratch.size();
      ws();
      if (i < n && s[i] == ']') { i++; v.first = (uint32_t)d->nodes.size(); v.count = 0; return; }
      while (true) {
        JNode ch;
        value(ch, depth + 1);
        scratch.push_back(ch);
        ws();
        if (i < n && s[i] == ',') { i++; continue; }
        if (i < n && s[i] == ']') { i++; break; }
        fail("expected , or ]");
      }
      v.first = (uint32_t)d->nodes.size();
      v.count = (uint32_t)(scratch.size() - base);
      d->nodes.insert(d->nodes.end(), scratch.begin() + base, scratch.end());
      scratch.resize(base);
      return;
    }
    if (c == '"') { v.t = J_STR; str(&v.s_off, &v.s_len); return; }
    if (c == 't') { if (n - i >= 4 && !memcmp(s + i, "true", 4)) { i += 4; v.t = J_BOOL; v.b = true; return; } fail("bad literal"); }
    if (c == 'f') { if (n - i >= 5 && !memcmp(s + i, "false", 5)) { i += 5; v.t = J_BOOL; v.b = false; return; } fail("bad literal"); }
    if (c == 'n') { if (n - i >= 4 && !memcmp(s + i, "null", 4)) { i += 4; v.t = J_NULL; return; } fail("bad literal"); }
    num(v);
  }
};

}  // namespace

size_t parse_one(const char* s, size_t n, NumMode mode, JDoc* doc) {
  static thread_local std::vector<JNode> scratch;
  scratch.clear();
  P p{s, n, 0, mode, doc, scratch};
  const size_t base = doc->strs.size();
  doc->strs.resize(std::max(doc->strs.capacity(), base + 1024));
  p.sb = &doc->strs[0];
  p.o = base;
  JNode root;
  try {
    p.value(root, 0);
  } catch (...) {
    doc->strs.resize(base);
    throw;
  }
  doc->strs.resize(p.o);
  doc->root = (uint32_t)doc->nodes.size();
  doc->nodes.push_back(root);
  return p.i;
}

void parse_json(const char* s, size_t n, NumMode mode, JDoc* doc) {
  doc->nodes.clear();
  doc->strs.clear();
  size_t used = parse_one(s, n, mode, doc);
  while (used < n && (s[used] == ' ' || s[used] == '\n' || s[used] == '\r' || s[used] == '\t')) used++;
  if (used != n) throw std::runtime_error("json: trailing data");
}

}  // namespace kvh
