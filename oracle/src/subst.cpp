// ORACLE — test infrastructure only (see ovalue.hpp header).
// Restatement of the reference's pattern-relative `$(...)` reference resolution
// and escape handling, which runs per (policy, resource) before matching:
//   pkg/engine/variables/vars.go:20-28   RegexVariables / RegexReferences / escapes
//   pkg/engine/variables/vars.go:253-309 substituteReferencesIfAny
//   pkg/engine/variables/vars.go:450-554 resolveReference / formAbsolutePath /
//                                        getValueFromReference / valFromReferenceToString
//   pkg/engine/jsonutils/traverse.go:58-130 traversal (keys and leafs, path strings)
// Map iteration order: canonical byte-lex by key.
#include <algorithm>
#include <vector>

#include "matcher.hpp"

namespace orc {

namespace {

// Extent of `.[^\ ]*\)` starting at position k (the '.' char). Returns end
// (exclusive) of the greedy match or npos.
size_t ref_tail(const std::string& s, size_t k) {
  if (k >= s.size() || s[k] == '\n') return std::string::npos;
  // '.' consumes one rune
  size_t w = 1;
  unsigned char c = (unsigned char)s[k];
  if (c >= 0xF0) w = 4; else if (c >= 0xE0) w = 3; else if (c >= 0xC0) w = 2;
  size_t st = k + w;
  size_t runend = st;
  while (runend < s.size() && s[runend] != ' ') runend++;
  // last ')' in [st, runend)
  for (size_t p = runend; p-- > st;) {
    if (s[p] == ')') return p + 1;
  }
  return std::string::npos;
}

struct Match {
  size_t b, e;
};

// RegexReferences = ^\$\(.[^\ ]*\)|[^\\]\$\(.[^\ ]*\)
std::vector<Match> find_references(const std::string& s) {
  std::vector<Match> out;
  size_t i = 0;
  while (i < s.size()) {
    if (i == 0 && s.compare(0, 2, "$(") == 0) {
      size_t e = ref_tail(s, 2);
      if (e != std::string::npos) { out.push_back({0, e}); i = e; continue; }
    }
    if (s[i] != '\\' && i + 2 < s.size() + 0 && s.compare(i + 1, 2, "$(") == 0) {
      // [^\\] consumes one rune at i
      size_t e = ref_tail(s, i + 3);
      if (e != std::string::npos) { out.push_back({i, e}); i = e; continue; }
    }
    i++;
  }
  return out;
}

// RegexEscpReferences = \\\$\(.[^\ ]*\)
std::vector<std::string> find_escaped_references(const std::string& s) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i < s.size()) {
    if (s[i] == '\\' && s.compare(i + 1, 2, "$(") == 0) {
      size_t e = ref_tail(s, i + 3);
      if (e != std::string::npos) { out.push_back(s.substr(i, e - i)); i = e; continue; }
    }
    i++;
  }
  return out;
}

// RegexEscpVariables = \\\{\{[^{}]*\}\}
std::vector<std::string> find_escaped_vars(const std::string& s) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i < s.size()) {
    if (s[i] == '\\' && s.compare(i + 1, 2, "{{") == 0) {
      size_t k = i + 3;
      while (k < s.size() && s[k] != '{' && s[k] != '}') k++;
      if (s.compare(k, 2, "}}") == 0) { out.push_back(s.substr(i, k + 2 - i)); i = k + 2; continue; }
    }
    i++;
  }
  return out;
}

std::string replace_n(const std::string& s, const std::string& from, const std::string& to, int n) {
  if (from.empty()) return s;
  std::string out;
  size_t i = 0;
  int done = 0;
  while (true) {
    size_t j = (n < 0 || done < n) ? s.find(from, i) : std::string::npos;
    if (j == std::string::npos) { out += s.substr(i); break; }
    out += s.substr(i, j - i);
    out += to;
    i = j + from.size();
    done++;
  }
  return out;
}

std::string trim_set(const std::string& s, const std::string& set) {
  size_t b = 0, e = s.size();
  while (b < e && set.find(s[b]) != std::string::npos) b++;
  while (e > b && set.find(s[e - 1]) != std::string::npos) e--;
  return s.substr(b, e - b);
}

std::string path_clean(const std::string& p) {
  if (p.empty()) return ".";
  bool rooted = p[0] == '/';
  std::vector<std::string> parts;
  size_t i = 0;
  while (i <= p.size()) {
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    std::string c = p.substr(i, j - i);
    if (c.empty() || c == ".") {
    } else if (c == "..") {
      if (!parts.empty() && parts.back() != "..") parts.pop_back();
      else if (!rooted) parts.push_back("..");
    } else {
      parts.push_back(c);
    }
    i = j + 1;
  }
  std::string out = rooted ? "/" : "";
  for (size_t k = 0; k < parts.size(); k++) {
    if (k) out += "/";
    out += parts[k];
  }
  return out.empty() ? "." : out;
}

// path.Join(a, b)
std::string path_join2(const std::string& a, const std::string& b) {
  if (a.empty() && b.empty()) return "";
  if (a.empty()) return path_clean(b);
  if (b.empty()) return path_clean(a);
  return path_clean(a + "/" + b);
}

std::vector<const Value::Entry*> sorted_entries(const Value& m) {
  std::vector<const Value::Entry*> es;
  for (const auto& e : m.m) es.push_back(&e);
  std::sort(es.begin(), es.end(), [](const Value::Entry* a, const Value::Entry* b) { return a->order < b->order; });
  return es;
}

// getValueFromReference: last matching key/leaf in traversal order.
void find_by_path(const Value& v, const std::string& path, const std::string& target, const Value** found,
                  std::string* found_key, bool* found_is_key) {
  switch (v.t) {
    case T::Map:
      for (const auto* e : sorted_entries(v)) {
        if (RemoveAnchorsFromPath(path) == target) { *found = nullptr; *found_key = e->key; *found_is_key = true; }
        find_by_path(*e->val, path + "/" + e->key, target, found, found_key, found_is_key);
      }
      break;
    case T::Arr:
      for (size_t k = 0; k < v.a.size(); k++) find_by_path(*v.a[k], path + "/" + std::to_string(k), target, found, found_key, found_is_key);
      break;
    default:
      if (RemoveAnchorsFromPath(path) == target) { *found = &v; *found_is_key = false; }
  }
}

struct Ctx {
  const Value* doc;
};

// Returns true (value updated), else false with the error message. *keep (optional) is set
// when the reference's action returns the unchanged element together with the error
// (vars.go:278-279,292-295: a reference resolving to nil, or to a non-string without an
// operator) rather than nil (an empty path or an operator on a missing value).
bool subst_string(const Ctx& cx, std::string& value, const std::string& dpath, std::string* err,
                  bool* keep = nullptr) {
  std::string orig = value;
  for (const auto& m : find_references(orig)) {
    std::string v = orig.substr(m.b, m.e - m.b);
    bool initial = v.compare(0, 2, "$(") == 0;
    std::string old = v;
    if (!initial) v = v.substr(1);
    // resolveReference
    std::string p = trim_set(v, "$()");
    std::string op = GetOperatorFromStringPattern(p);
    p = p.substr(op.size());
    if (p.empty()) {
      *err = "failed to resolve " + v + " at path " + dpath + ": expected path, found empty reference";
      return false;
    }
    std::string abs = (!p.empty() && p[0] == '/') ? p : path_join2(dpath, p);
    const Value* found = nullptr;
    std::string fkey;
    bool is_key = false;
    find_by_path(*cx.doc, "", abs, &found, &fkey, &is_key);
    Value keyval;
    if (is_key) { keyval = Value::mk_str(fkey); found = &keyval; }
    std::string resolved;
    bool resolved_is_string = false;
    if (op.empty()) {
      if (!found || found->t == T::Null) {
        *err = "failed to resolve " + v + " at path " + dpath + ": <nil>";
        if (keep) *keep = true;
        return false;
      }
      if (found->t == T::Str) { resolved = found->s; resolved_is_string = true; }
    } else {
      std::string fv;
      if (found && found->t == T::Str) fv = found->s;
      else if (found && found->t == T::Int) fv = std::to_string(found->i);
      else if (found && found->t == T::Float) fv = go_format_f6(found->f);
      else {
        *err = "failed to resolve " + v + " at path " + dpath + ": incorrect expression: operator " + op +
               " does not match with value " + go_format_v(found);
        return false;
      }
      resolved = op + fv;
      resolved_is_string = true;
    }
    if (resolved_is_string) {
      std::string repl = initial ? "" : old.substr(0, 1);
      repl += resolved;
      value = replace_n(value, old, repl, 1);
      continue;
    }
    *err = "NotResolvedReferenceErr,reference " + v + " not resolved at path " + dpath;
    if (keep) *keep = true;
    return false;
  }
  for (const auto& e : find_escaped_references(value)) value = replace_n(value, e, e.substr(1), -1);
  return true;
}

bool traverse(const Ctx& cx, Value& v, const std::string& path, std::string* err) {
  if (v.t == T::Map) {
    // keys first (per entry: key action, then value), canonical order
    std::vector<std::string> keys;
    for (const auto* e : sorted_entries(v)) keys.push_back(e->key);
    for (const auto& k : keys) {
      std::string nk = k;
      if (!subst_string(cx, nk, path, err)) return false;
      Value* child = v.get_mut(k);
      if (!traverse(cx, *child, path + "/" + k, err)) return false;
      if (nk != k) {
        Value copy = *child;
        std::string order;
        for (auto& e : v.m)
          if (e.key == k) order = e.order;
        v.erase(k);
        v.set(nk, copy, order);
      }
    }
    return true;
  }
  if (v.t == T::Arr) {
    for (size_t k = 0; k < v.a.size(); k++)
      if (!traverse(cx, *v.a[k], path + "/" + std::to_string(k), err)) return false;
    return true;
  }
  if (v.t == T::Str) return subst_string(cx, v.s, path, err);
  return true;
}

void unescape_vars(Value& v) {
  if (v.t == T::Map) {
    std::vector<std::string> keys;
    for (const auto& e : v.m) keys.push_back(e.key);
    for (const auto& k : keys) {
      std::string nk = k;
      for (const auto& e : find_escaped_vars(k)) nk = replace_n(nk, e, e.substr(1), -1);
      Value* child = v.get_mut(k);
      unescape_vars(*child);
      if (nk != k) {
        Value copy = *child;
        std::string order;
        for (auto& e : v.m)
          if (e.key == k) order = e.order;
        v.erase(k);
        v.set(nk, copy, order);
      }
    }
  } else if (v.t == T::Arr) {
    for (auto* x : v.a) unescape_vars(*x);
  } else if (v.t == T::Str) {
    for (const auto& e : find_escaped_vars(v.s)) v.s = replace_n(v.s, e, e.substr(1), -1);
  }
}

}  // namespace

bool HasVariable(const std::string& s) {
  // RegexVariables = ^\{\{[^{}]*\}\}|[^\\]\{\{[^{}]*\}\}
  for (size_t j = 0; j + 1 < s.size(); j++) {
    if (s[j] == '{' && s[j + 1] == '{') {
      if (j > 0 && s[j - 1] == '\\') continue;
      size_t k = j + 2;
      while (k < s.size() && s[k] != '{' && s[k] != '}') k++;
      if (s.compare(k, 2, "}}") == 0) return true;
    }
  }
  return false;
}

bool DocHasVariable(const Value& v) {
  switch (v.t) {
    case T::Str: return HasVariable(v.s);
    case T::Map:
      for (const auto& e : v.m)
        if (HasVariable(e.key) || DocHasVariable(*e.val)) return true;
      return false;
    case T::Arr:
      for (const auto* x : v.a)
        if (DocHasVariable(*x)) return true;
      return false;
    default: return false;
  }
}

bool SubstituteReferences(Value& document, std::string* err, bool unescape) {
  Value original = document;  // references resolve against the unmodified document
  Ctx cx{&original};
  if (!traverse(cx, document, "", err)) return false;
  if (unescape) unescape_vars(document);  // (documents with variables: per string, after substitution)
  return true;
}


// ---------------------------------------------------------------- message variables
// buildErrorMessage (pkg/engine/validation.go:510-532) -> variables.SubstituteAll on the
// message: substituteReferences, then substituteVariablesIfAny (vars.go:319-398) with the
// CLI context {"request":{"object": resource}} read back by encoding/json (float64 numbers),
// then RegexEscpVariables unescaping. Returns false where the reference panics (an
// unresolvable variable or a non-string whole-message value: msgRaw.(string), :519-524).
namespace {

// RegexVariables.FindAllString: ^\{\{[^{}]*\}\}|[^\\]\{\{[^{}]*\}\}, leftmost-first
std::vector<std::string> find_vars(const std::string& s) {
  std::vector<std::string> out;
  auto close = [&](size_t j) -> size_t {
    if (s.compare(j, 2, "{{") != 0) return std::string::npos;
    size_t k = j + 2;
    while (k < s.size() && s[k] != '{' && s[k] != '}') k++;
    return s.compare(k, 2, "}}") == 0 ? k + 2 : std::string::npos;
  };
  size_t i = 0;
  while (i < s.size()) {
    if (i == 0) {
      size_t e = close(0);
      if (e != std::string::npos) { out.push_back(s.substr(0, e)); i = e; continue; }
    }
    if (s[i] != '\\' && i + 1 < s.size()) {
      size_t e = close(i + 1);
      if (e != std::string::npos) { out.push_back(s.substr(i, e - i)); i = e; continue; }
    }
    i++;
  }
  return out;
}

// encoding/json float64: strconv 'f' -1, or 'e' -1 outside [1e-6, 1e21) with "e-07" -> "e-7"
std::string json_float(double f) {
  char buf[64];
  int p = 1;
  for (; p <= 17; p++) {
    snprintf(buf, sizeof buf, "%.*e", p - 1, f);
    if (strtod(buf, nullptr) == f) break;
  }
  std::string e(buf);  // d.ddde[+-]XX
  size_t ep = e.find('e');
  std::string mant = e.substr(0, ep);
  int ex = atoi(e.c_str() + ep + 1);
  double a = f < 0 ? -f : f;
  if (a != 0 && (a < 1e-6 || a >= 1e21)) {
    char eb[16];
    snprintf(eb, sizeof eb, "e%c%02d", ex < 0 ? '-' : '+', ex < 0 ? -ex : ex);
    std::string es(eb);
    if (es.size() == 4 && es[1] == '-' && es[2] == '0') es.erase(2, 1);
    return mant + es;
  }
  bool neg = mant[0] == '-';
  std::string digs;
  for (char c : mant) if (c >= '0' && c <= '9') digs += c;
  while (digs.size() > 1 && digs.back() == '0') digs.pop_back();
  // value = 0.digs * 10^(ex+1)
  int point = ex + 1;
  std::string out;
  if (point <= 0) out = "0." + std::string(-point, '0') + digs;
  else if ((size_t)point >= digs.size()) out = digs + std::string(point - digs.size(), '0');
  else out = digs.substr(0, point) + "." + digs.substr(point);
  if (out == "0" || f == 0) out = "0";
  return (neg ? "-" : "") + out;
}

std::string json_string(const std::string& s) {
  std::string o = "\"";
  for (size_t i = 0; i < s.size(); i++) {
    unsigned char c = (unsigned char)s[i];
    if (c == '"') o += "\\\"";
    else if (c == '\\') o += "\\\\";
    else if (c == '\n') o += "\\n";
    else if (c == '\r') o += "\\r";
    else if (c == '\t') o += "\\t";
    else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", c);
      o += b;
    } else if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
               ((unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9)) {
      o += (unsigned char)s[i + 2] == 0xA8 ? "\\u2028" : "\\u2029";
      i += 2;
    } else {
      o += (char)c;
    }
  }
  return o + "\"";
}

std::string json_marshal(const Value* v) {
  if (!v) return "null";
  switch (v->t) {
    case T::Null: return "null";
    case T::Bool: return v->b ? "true" : "false";
    case T::Int: return json_float((double)v->i);
    case T::Float: return json_float(v->f);
    case T::Str: return json_string(v->s);
    case T::Arr: {
      std::string o = "[";
      for (size_t k = 0; k < v->a.size(); k++) o += (k ? "," : "") + json_marshal(v->a[k]);
      return o + "]";
    }
    case T::Map: {
      std::vector<const Value::Entry*> es;
      for (const auto& e : v->m) es.push_back(&e);
      std::sort(es.begin(), es.end(), [](const Value::Entry* x, const Value::Entry* y) { return x->key < y->key; });
      std::string o = "{";
      for (size_t k = 0; k < es.size(); k++) o += (k ? "," : "") + json_string(es[k]->key) + ":" + json_marshal(es[k]->val);
      return o + "}";
    }
  }
  return "null";
}

// ctx.Query (context/evaluate.go:15-50) for request.object field / "quoted" / [index] chains.
// Returns false on an unknown key or an unsupported expression.
bool query_object(const std::string& q, const Value& resource, const Value** out) {
  const std::string root = "request.object";
  if (q.compare(0, root.size(), root) != 0) return false;
  const Value* cur = &resource;
  size_t i = root.size();
  while (i < q.size()) {
    if (q[i] == '[') {
      size_t e = q.find(']', i);
      if (e == std::string::npos || e == i + 1) return false;
      std::string num = q.substr(i + 1, e - i - 1);
      for (size_t k = 0; k < num.size(); k++)
        if (!(isdigit((unsigned char)num[k]) || (k == 0 && num[k] == '-' && num.size() > 1))) return false;
      long idx = atol(num.c_str());
      if (cur && cur->t == T::Arr) {
        long n = (long)cur->a.size();
        if (idx < 0) idx += n;
        cur = (idx >= 0 && idx < n) ? cur->a[idx] : nullptr;
      } else {
        cur = nullptr;
      }
      i = e + 1;
      continue;
    }
    if (q[i] != '.') return false;
    i++;
    std::string key;
    if (i < q.size() && q[i] == '"') {
      i++;
      while (i < q.size() && q[i] != '"') {
        if (q[i] == '\\' && i + 1 < q.size()) i++;
        key += q[i++];
      }
      if (i >= q.size()) return false;
      i++;
    } else {
      size_t s = i;
      while (i < q.size() && (isalnum((unsigned char)q[i]) || q[i] == '_')) i++;
      if (i == s || isdigit((unsigned char)q[s])) return false;
      key = q.substr(s, i - s);
    }
    if (cur && cur->t == T::Map) {
      cur = cur->get(key);
      if (!cur) return false;  // NotFoundError: Unknown key
    } else {
      cur = nullptr;
    }
  }
  *out = cur;
  return true;
}

}  // namespace

bool SubstituteMessage(const std::string& msg, const Value& resource, std::string* out) {
  // substituteReferences over the string document (its only leaf, at path ""): a reference that
  // returns the element with an error leaves the message as it is (SubstituteAll returns it,
  // buildErrorMessage logs the error, validation.go:519-522); one that returns nil panics
  std::string value = msg;
  {
    const Value original = Value::mk_str(msg);
    Ctx cx{&original};
    std::string err;
    bool keep = false;
    if (!subst_string(cx, value, "", &err, &keep)) {
      if (!keep) return false;
      *out = msg;
      return true;
    }
  }
  auto vars = find_vars(value);
  while (!vars.empty()) {
    std::string original = value;
    for (std::string v : vars) {
      bool initial = v.compare(0, 2, "{{") == 0;
      std::string old = v;
      if (!initial) v = v.substr(1);
      std::string var = replace_n(replace_n(v, "{{", "", -1), "}}", "", -1);
      size_t b = var.find_first_not_of(" \t\n\r\v\f"), e = var.find_last_not_of(" \t\n\r\v\f");
      var = b == std::string::npos ? "" : var.substr(b, e - b + 1);
      const Value* got = nullptr;
      if (!query_object(var, resource, &got)) return false;
      if (original == v) {
        if (!got || got->t != T::Str) return false;
        *out = got->s;
        return true;
      }
      std::string prefix = initial ? "" : old.substr(0, 1);
      std::string sub = got && got->t == T::Str ? got->s : json_marshal(got);
      value = replace_n(original, prefix + v, prefix + sub, 1);
    }
    vars = find_vars(value);
  }
  for (const auto& e : find_escaped_vars(value)) value = replace_n(value, e, e.substr(1), -1);
  *out = value;
  return true;
}


// ---------------------------------------------------------------- pattern variables
// substituteVars over a validate.pattern / anyPattern document (vars.go:319-398, traversal
// jsonutils/traverse.go:58-130: the action runs on an element first, then the traversal
// descends into what it returned; per map entry the key, then the value; canonical key
// order) with the CLI / admission JSON context {"request":{"object": resource}} (numbers
// read back as float64). Device scope: variables `request.object<path>`
// (fields, "quoted" fields, [index]) and `@`; anything else is outside it.
namespace {

// regexVariableInit = ^\{\{[^{}]*\}\}
bool var_initial(const std::string& v) {
  if (v.compare(0, 2, "{{") != 0) return false;
  size_t k = 2;
  while (k < v.size() && v[k] != '{' && v[k] != '}') k++;
  return v.compare(k, 2, "}}") == 0;
}

std::string trim_space(const std::string& s) {
  size_t b = s.find_first_not_of(" \t\n\r\v\f"), e = s.find_last_not_of(" \t\n\r\v\f");
  return b == std::string::npos ? "" : s.substr(b, e - b + 1);
}

// getJMESPath (vars.go:416-422): tokens [3:] of the traversal path joined with '.', then
// regexPathDigit `\.?([\d])\.?` -> "[$1]." and '.' trimmed. false where the reference's
// slice expression panics (fewer than 3 tokens).
bool jmes_path_of(const std::string& raw, std::string* out) {
  std::vector<std::string> tok;
  size_t i = 0;
  while (true) {
    size_t j = raw.find('/', i);
    tok.push_back(raw.substr(i, j == std::string::npos ? std::string::npos : j - i));
    if (j == std::string::npos) break;
    i = j + 1;
  }
  if (tok.size() < 3) return false;
  std::string path;
  for (size_t k = 3; k < tok.size(); k++) path += (k > 3 ? "." : "") + tok[k];
  std::string b;
  for (size_t k = 0; k < path.size();) {
    size_t d = k;
    if (path[d] == '.' && d + 1 < path.size() && isdigit((unsigned char)path[d + 1])) d++;
    if (isdigit((unsigned char)path[d])) {
      size_t e = d + 1;
      if (e < path.size() && path[e] == '.') e++;
      b += "[";
      b += path[d];
      b += "].";
      k = e;
      continue;
    }
    b += path[k++];
  }
  size_t s0 = b.find_first_not_of('.'), s1 = b.find_last_not_of('.');
  *out = s0 == std::string::npos ? "" : b.substr(s0, s1 - s0 + 1);
  return true;
}

// the query of one variable (after brace removal and trimming); false: outside the scope
bool var_query(const std::string& var, const std::string& path, std::string* q) {
  if (var == "@") {
    std::string p;
    if (!jmes_path_of(path, &p)) return false;
    *q = (!p.empty() && p[0] == '[') ? "request.object" + p : "request.object." + p;
    return true;
  }
  *q = var;
  return true;
}

// a resource value as the JSON context returns it (numbers float64)
void to_context(Value& v) {
  if (v.t == T::Int) {
    v = Value::mk_float((double)v.i);
  } else if (v.t == T::Map) {
    for (auto& e : v.m) to_context(*e.val);
  } else if (v.t == T::Arr) {
    for (auto* x : v.a) to_context(*x);
  }
}
Value as_context(const Value* v) {
  if (!v) return Value();
  Value c = *v;
  to_context(c);
  return c;
}

// substituteVariablesIfAny on one string: 0 ok (*out = the new element), 1 error, 2 outside scope
int subst_var_string(const std::string& s, const std::string& path, const Value& resource, Value* out,
                     std::string* err, bool* structural) {
  std::string value = s;
  auto vars = find_vars(value);
  while (!vars.empty()) {
    std::string original = value;
    for (std::string v : vars) {
      const bool initial = var_initial(v);
      const std::string old = v;
      if (!initial) {
        if ((unsigned char)old[0] >= 0x80) return 2;  // a rune split by v[1:]: "failed to resolve" (outside scope)
        v = v.substr(1);
      }
      const std::string var = trim_space(replace_n(replace_n(v, "{{", "", -1), "}}", "", -1));
      std::string q;
      if (!var_query(var, path, &q)) return 2;
      const Value* got = nullptr;
      std::string missing;
      int r = QueryObject(q, resource, &got, &missing);
      if (r == 2) return 2;
      if (r == 1) {
        *err = "Unknown key \"" + missing + "\" in path";
        return 1;
      }
      if (original == v) {
        if (got && (got->t == T::Map || got->t == T::Arr)) *structural = true;
        *out = as_context(got);
        return 0;
      }
      const std::string prefix = initial ? "" : old.substr(0, 1);
      const Value cv = as_context(got);
      const std::string sub = got && got->t == T::Str ? got->s : json_marshal(got ? &cv : nullptr);
      value = replace_n(original, prefix + v, prefix + sub, 1);
    }
    vars = find_vars(value);
  }
  for (const auto& e : find_escaped_vars(value)) value = replace_n(value, e, e.substr(1), -1);
  *out = Value::mk_str(value);
  return 0;
}

int traverse_vars(Value& v, const std::string& path, const Value& resource, std::string* err, bool* structural) {
  if (v.t == T::Str) {
    Value nv;
    int r = subst_var_string(v.s, path, resource, &nv, err, structural);
    if (r) return r;
    v = nv;
    if (v.t != T::Map && v.t != T::Arr) return 0;
    // the traversal descends into what the action returned (traverse.go:63-76)
  }
  if (v.t == T::Map) {
    std::vector<std::string> keys;
    for (const auto* e : sorted_entries(v)) keys.push_back(e->key);
    for (const auto& k : keys) {
      if (HasVariable(k)) return 2;  // variables in keys: outside scope
      std::string nk = k;
      for (const auto& e : find_escaped_vars(k)) nk = replace_n(nk, e, e.substr(1), -1);
      Value* child = v.get_mut(k);
      int r = traverse_vars(*child, path + "/" + k, resource, err, structural);
      if (r) return r;
      if (nk != k) {
        Value copy = *child;
        std::string order;
        for (auto& e : v.m)
          if (e.key == k) order = e.order;
        v.erase(k);
        v.set(nk, copy, order);
      }
    }
    return 0;
  }
  if (v.t == T::Arr) {
    for (size_t k = 0; k < v.a.size(); k++) {
      int r = traverse_vars(*v.a[k], path + "/" + std::to_string(k), resource, err, structural);
      if (r) return r;
    }
  }
  return 0;
}

bool vars_in_scope(const Value& v, const std::string& path) {
  if (v.t == T::Str) {
    for (std::string x : find_vars(v.s)) {
      if (!var_initial(x)) {
        if ((unsigned char)x[0] >= 0x80) return false;
        x = x.substr(1);
      }
      const std::string var = trim_space(replace_n(replace_n(x, "{{", "", -1), "}}", "", -1));
      std::string q;
      if (!var_query(var, path, &q) || QueryObject(q, Value::mk_map(), nullptr, nullptr) == 2) return false;
    }
    return true;
  }
  if (v.t == T::Map) {
    for (const auto& e : v.m)
      if (HasVariable(e.key) || !vars_in_scope(*e.val, path + "/" + e.key)) return false;
    return true;
  }
  if (v.t == T::Arr)
    for (size_t k = 0; k < v.a.size(); k++)
      if (!vars_in_scope(*v.a[k], path + "/" + std::to_string(k))) return false;
  return true;
}

}  // namespace

int QueryObject(const std::string& q, const Value& resource, const Value** out, std::string* missing) {
  // grammar check first (out == nullptr: check only)
  const std::string root = "request.object";
  if (q.compare(0, root.size(), root) != 0) return 2;
  const Value* cur = &resource;
  bool lost = false;  // a missing key was met (the search stops there with NotFoundError)
  std::string miss;
  size_t i = root.size();
  while (i < q.size()) {
    if (q[i] == '[') {
      size_t e = q.find(']', i);
      if (e == std::string::npos || e == i + 1) return 2;
      std::string num = q.substr(i + 1, e - i - 1);
      for (size_t k = 0; k < num.size(); k++)
        if (!(isdigit((unsigned char)num[k]) || (k == 0 && num[k] == '-' && num.size() > 1))) return 2;
      long idx = atol(num.c_str());
      if (!lost) {
        if (cur && cur->t == T::Arr) {
          long n = (long)cur->a.size();
          if (idx < 0) idx += n;
          cur = (idx >= 0 && idx < n) ? cur->a[idx] : nullptr;
        } else {
          cur = nullptr;
        }
      }
      i = e + 1;
      continue;
    }
    if (q[i] != '.') return 2;
    i++;
    std::string key;
    if (i < q.size() && q[i] == '"') {
      i++;
      while (i < q.size() && q[i] != '"') {
        if (q[i] == '\\' && i + 1 < q.size()) i++;
        key += q[i++];
      }
      if (i >= q.size()) return 2;
      i++;
    } else {
      size_t s = i;
      while (i < q.size() && (isalnum((unsigned char)q[i]) || q[i] == '_')) i++;
      if (i == s || isdigit((unsigned char)q[s])) return 2;
      key = q.substr(s, i - s);
    }
    if (!lost) {
      if (cur && cur->t == T::Map) {
        const Value* nx = cur->get(key);
        if (!nx) { lost = true; miss = key; }
        cur = nx;
      } else {
        cur = nullptr;
      }
    }
  }
  if (!out) return 0;
  if (lost) {
    if (missing) *missing = miss;
    return 1;
  }
  *out = cur;
  return 0;
}

bool PatternVarsInScope(const Value& doc) { return vars_in_scope(doc, ""); }

int SubstitutePatternVars(Value& doc, const Value& resource, std::string* err, bool* structural) {
  bool st = false;
  int r = traverse_vars(doc, "", resource, err, &st);
  if (structural) *structural = st;
  return r;
}

}  // namespace orc
