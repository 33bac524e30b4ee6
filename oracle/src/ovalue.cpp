// ORACLE — test infrastructure only (see ovalue.hpp header).
#include "ovalue.hpp"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>

namespace orc {

void Value::clear() {
  for (auto& e : m) delete e.val;
  m.clear();
  for (auto* p : a) delete p;
  a.clear();
}

void Value::copy_from(const Value& o) {
  t = o.t; b = o.b; i = o.i; f = o.f; s = o.s;
  m.reserve(o.m.size());
  for (const auto& e : o.m) m.push_back({e.key, e.order, new Value(*e.val)});
  a.reserve(o.a.size());
  for (const auto* p : o.a) a.push_back(new Value(*p));
}

const Value* Value::get(const std::string& k) const {
  for (const auto& e : m)
    if (e.key == k) return e.val;
  return nullptr;
}

Value* Value::get_mut(const std::string& k) {
  for (auto& e : m)
    if (e.key == k) return e.val;
  return nullptr;
}

void Value::set(const std::string& k, const Value& v, const std::string& order) {
  for (auto& e : m) {
    if (e.key == k) {
      delete e.val;
      e.val = new Value(v);
      e.order = order;
      return;
    }
  }
  m.push_back({k, order, new Value(v)});
}

void Value::erase(const std::string& k) {
  for (size_t j = 0; j < m.size(); j++) {
    if (m[j].key == k) {
      delete m[j].val;
      m.erase(m.begin() + j);
      return;
    }
  }
}

namespace {

void append_utf8(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out.push_back((char)cp);
  } else if (cp < 0x800) {
    out.push_back((char)(0xC0 | (cp >> 6)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    out.push_back((char)(0xE0 | (cp >> 12)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    out.push_back((char)(0xF0 | (cp >> 18)));
    out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  }
}

// Decodes one UTF-8 rune like Go's utf8.DecodeRune: invalid -> (0xFFFD, 1).
uint32_t decode_rune(const unsigned char* p, size_t n, size_t* width) {
  if (n == 0) { *width = 0; return 0xFFFD; }
  unsigned c = p[0];
  if (c < 0x80) { *width = 1; return c; }
  auto cont = [&](size_t k) { return k < n && (p[k] & 0xC0) == 0x80; };
  if (c >= 0xC2 && c <= 0xDF) {
    if (cont(1)) { *width = 2; return ((c & 0x1F) << 6) | (p[1] & 0x3F); }
  } else if (c >= 0xE0 && c <= 0xEF) {
    if (n >= 2) {
      unsigned c1 = p[1];
      bool ok1 = (c == 0xE0) ? (c1 >= 0xA0 && c1 <= 0xBF)
               : (c == 0xED) ? (c1 >= 0x80 && c1 <= 0x9F)
                             : (c1 >= 0x80 && c1 <= 0xBF);
      if (ok1 && cont(2)) {
        *width = 3;
        return ((c & 0x0F) << 12) | ((c1 & 0x3F) << 6) | (p[2] & 0x3F);
      }
    }
  } else if (c >= 0xF0 && c <= 0xF4) {
    if (n >= 2) {
      unsigned c1 = p[1];
      bool ok1 = (c == 0xF0) ? (c1 >= 0x90 && c1 <= 0xBF)
               : (c == 0xF4) ? (c1 >= 0x80 && c1 <= 0x8F)
                             : (c1 >= 0x80 && c1 <= 0xBF);
      if (ok1 && cont(2) && cont(3)) {
        *width = 4;
        return ((c & 0x07) << 18) | ((c1 & 0x3F) << 12) | ((p[2] & 0x3F) << 6) | (p[3] & 0x3F);
      }
    }
  }
  *width = 1;
  return 0xFFFD;
}

struct Parser {
  const char* p;
  const char* end;
  NumMode mode;

  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json: ") + what);
  }
  void ws() {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
  }
  uint32_t hex4() {
    if (end - p < 4) fail("bad \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) {
      char c = p[k];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex");
    }
    p += 4;
    return v;
  }
  std::string str() {
    if (p >= end || *p != '"') fail("expected string");
    p++;
    std::string out;
    while (true) {
      if (p >= end) fail("unterminated string");
      unsigned char c = (unsigned char)*p;
      if (c == '"') { p++; break; }
      if (c < 0x20) fail("control char in string");
      if (c == '\\') {
        p++;
        if (p >= end) fail("bad escape");
        char e = *p++;
        switch (e) {
          case '"': out.push_back('"'); break;
          case '\\': out.push_back('\\'); break;
          case '/': out.push_back('/'); break;
          case 'b': out.push_back('\b'); break;
          case 'f': out.push_back('\f'); break;
          case 'n': out.push_back('\n'); break;
          case 'r': out.push_back('\r'); break;
          case 't': out.push_back('\t'); break;
          case 'u': {
            uint32_t cp = hex4();
            if (cp >= 0xD800 && cp < 0xDC00) {
              // surrogate pair?
              if (end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                const char* save = p;
                p += 2;
                uint32_t lo = hex4();
                if (lo >= 0xDC00 && lo < 0xE000) {
                  cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                } else {
                  p = save;
                  cp = 0xFFFD;
                }
              } else {
                cp = 0xFFFD;
              }
            } else if (cp >= 0xDC00 && cp < 0xE000) {
              cp = 0xFFFD;
            }
            append_utf8(out, cp);
            break;
          }
          default: fail("bad escape char");
        }
        continue;
      }
      if (c < 0x80) { out.push_back((char)c); p++; continue; }
      size_t w;
      uint32_t cp = decode_rune((const unsigned char*)p, end - p, &w);
      if (cp == 0xFFFD && w == 1) { append_utf8(out, 0xFFFD); p++; continue; }
      out.append(p, w);
      p += w;
    }
    return out;
  }
  Value num() {
    const char* st = p;
    if (p < end && *p == '-') p++;
    if (p >= end) fail("bad number");
    if (*p == '0') {
      p++;
    } else if (*p >= '1' && *p <= '9') {
      while (p < end && *p >= '0' && *p <= '9') p++;
    } else {
      fail("bad number");
    }
    if (p < end && *p == '.') {
      p++;
      if (p >= end || !(*p >= '0' && *p <= '9')) fail("bad fraction");
      while (p < end && *p >= '0' && *p <= '9') p++;
    }
    if (p < end && (*p == 'e' || *p == 'E')) {
      p++;
      if (p < end && (*p == '+' || *p == '-')) p++;
      if (p >= end || !(*p >= '0' && *p <= '9')) fail("bad exponent");
      while (p < end && *p >= '0' && *p <= '9') p++;
    }
    std::string lit(st, p - st);
    Value v;
    if (mode == NumMode::Unstructured) {
      int64_t iv;
      if (go_parse_int(lit, &iv)) { v.t = T::Int; v.i = iv; return v; }
    }
    double d;
    if (!go_parse_float(lit, &d)) fail("number out of range");
    v.t = T::Float;
    v.f = d;
    return v;
  }
  Value value(int depth) {
    if (depth > 10000) fail("too deep");
    ws();
    if (p >= end) fail("unexpected end");
    char c = *p;
    Value v;
    if (c == '{') {
      p++;
      v.t = T::Map;
      ws();
      if (p < end && *p == '}') { p++; return v; }
      while (true) {
        ws();
        std::string k = str();
        ws();
        if (p >= end || *p != ':') fail("expected :");
        p++;
        Value x = value(depth + 1);
        v.set(k, x, k);
        ws();
        if (p < end && *p == ',') { p++; continue; }
        if (p < end && *p == '}') { p++; break; }
        fail("expected , or }");
      }
      return v;
    }
    if (c == '[') {
      p++;
      v.t = T::Arr;
      ws();
      if (p < end && *p == ']') { p++; return v; }
      while (true) {
        v.a.push_back(new Value(value(depth + 1)));
        ws();
        if (p < end && *p == ',') { p++; continue; }
        if (p < end && *p == ']') { p++; break; }
        fail("expected , or ]");
      }
      return v;
    }
    if (c == '"') { v.t = T::Str; v.s = str(); return v; }
    if (c == 't') { if (end - p >= 4 && !memcmp(p, "true", 4)) { p += 4; v.t = T::Bool; v.b = true; return v; } fail("bad literal"); }
    if (c == 'f') { if (end - p >= 5 && !memcmp(p, "false", 5)) { p += 5; v.t = T::Bool; v.b = false; return v; } fail("bad literal"); }
    if (c == 'n') { if (end - p >= 4 && !memcmp(p, "null", 4)) { p += 4; return v; } fail("bad literal"); }
    return num();
  }
};

void esc(std::string& out, const std::string& s) {
  out.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof b, "\\u%04x", c);
          out += b;
        } else {
          out.push_back((char)c);
        }
    }
  }
  out.push_back('"');
}

void ser(std::string& out, const Value& v) {
  switch (v.t) {
    case T::Null: out += "null"; break;
    case T::Bool: out += v.b ? "true" : "false"; break;
    case T::Int: out += std::to_string(v.i); break;
    case T::Float: {
      char b[64];
      snprintf(b, sizeof b, "%.17g", v.f);
      std::string s = b;
      if (s.find_first_of(".eEn") == std::string::npos) s += ".0";
      out += s;
      break;
    }
    case T::Str: esc(out, v.s); break;
    case T::Map: {
      out.push_back('{');
      bool first = true;
      for (const auto& e : v.m) {
        if (!first) out.push_back(',');
        first = false;
        esc(out, e.key);
        out.push_back(':');
        ser(out, *e.val);
      }
      out.push_back('}');
      break;
    }
    case T::Arr: {
      out.push_back('[');
      for (size_t k = 0; k < v.a.size(); k++) {
        if (k) out.push_back(',');
        ser(out, *v.a[k]);
      }
      out.push_back(']');
      break;
    }
  }
}

}  // namespace

std::string utf8_sanitize(const std::string& s) {
  std::string out;
  const unsigned char* p = (const unsigned char*)s.data();
  size_t n = s.size(), k = 0;
  while (k < n) {
    if (p[k] < 0x80) { out.push_back((char)p[k]); k++; continue; }
    size_t w;
    uint32_t cp = decode_rune(p + k, n - k, &w);
    if (cp == 0xFFFD && w == 1) append_utf8(out, 0xFFFD);
    else out.append((const char*)p + k, w);
    k += w;
  }
  return out;
}

Value parse_json(const std::string& text, NumMode mode) {
  Parser ps{text.data(), text.data() + text.size(), mode};
  Value v = ps.value(0);
  ps.ws();
  if (ps.p != ps.end) throw std::runtime_error("json: trailing data");
  return v;
}

std::string to_json(const Value& v) {
  std::string out;
  ser(out, v);
  return out;
}

}  // namespace orc
