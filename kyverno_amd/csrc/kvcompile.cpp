// Policy compiler: lowers validate.pattern / validate.anyPattern rules and their
// match/exclude blocks into the structured program executed by the HIP pattern
// VM (kv_validate_kernel) and the prefilter tables.
//
// Reference semantics compiled here (isabella232/kyverno v1.5.x):
//   pkg/engine/validation.go:26-547       rule dispatch, anyPattern, routing
//   pkg/engine/validate/validate.go:29-194 MatchPattern / validateMap / validateArray
//   pkg/engine/validate/utils.go:10-60    key order tiers
//   pkg/engine/anchor/anchor.go:21-277    handlers; common/common.go anchor syntax
//   pkg/engine/common/anchorKey.go        AnchorKey registration
//   pkg/engine/validate/pattern.go:153-318, operator/operator.go:33-67  string predicates
//   pkg/engine/wildcards/wildcards.go:13-161 ExpandInMetadata / ReplaceInSelector
//   pkg/engine/variables/vars.go:20-28,253-309,450-554  $() references (resolved here, once)
//   pkg/engine/utils.go:37-369            match/exclude blocks
// Go map iteration order is replaced by the canonical order of DESIGN.md.
#include <cmath>
#include <algorithm>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <stdexcept>

#include "kvinternal.hpp"

namespace kvh {

using namespace kv;

// ---------------------------------------------------------------- anchors
bool is_condition_anchor(const std::string& s) { return s.size() >= 2 && s[0] == '(' && s.back() == ')'; }
static bool pfx_anchor(const std::string& s, char a) { return s.size() >= 3 && s[0] == a && s[1] == '(' && s.back() == ')'; }
bool is_global_anchor(const std::string& s) { return pfx_anchor(s, '<'); }
bool is_negation_anchor(const std::string& s) { return pfx_anchor(s, 'X'); }
static bool is_adding_anchor(const std::string& s) { return pfx_anchor(s, '+'); }
bool is_equality_anchor(const std::string& s) { return pfx_anchor(s, '='); }
bool is_existence_anchor(const std::string& s) { return pfx_anchor(s, '^'); }

std::string remove_anchor(const std::string& key, std::string* prefix) {
  if (is_condition_anchor(key)) {
    if (prefix) *prefix = "(";
    return key.substr(1, key.size() - 2);
  }
  if (is_existence_anchor(key) || is_adding_anchor(key) || is_equality_anchor(key) || is_negation_anchor(key) ||
      is_global_anchor(key)) {
    if (prefix) *prefix = key.substr(0, 2);
    return key.substr(2, key.size() - 3);
  }
  if (prefix) prefix->clear();
  return key;
}

static bool has_wild(const std::string& s) { return s.find_first_of("*?") != std::string::npos; }

// Go fmt of a decoded pattern value (encoding/json into interface{}), for the
// error messages of validate.go / anchor.go: %T and %v (map keys sorted).
static std::string go_T(const PV& p) {
  switch (p.t) {
    case J_MAP: return "map[string]interface {}";
    case J_ARR: return "[]interface {}";
    case J_STR: return "string";
    case J_BOOL: return "bool";
    case J_INT: return "int64";
    case J_FLOAT: return "float64";
    default: return "<nil>";
  }
}
static std::string go_v(const PV& p) {
  switch (p.t) {
    case J_MAP: {
      std::vector<size_t> ix(p.mk.size());
      for (size_t i = 0; i < ix.size(); i++) ix[i] = i;
      std::sort(ix.begin(), ix.end(), [&](size_t a, size_t b) { return p.mk[a] < p.mk[b]; });
      std::string o = "map[";
      for (size_t k = 0; k < ix.size(); k++) o += (k ? " " : "") + p.mk[ix[k]] + ":" + go_v(p.mv[ix[k]]);
      return o + "]";
    }
    case J_ARR: {
      std::string o = "[";
      for (size_t k = 0; k < p.a.size(); k++) o += (k ? " " : "") + go_v(p.a[k]);
      return o + "]";
    }
    case J_STR: return p.s;
    case J_BOOL: return p.b ? "true" : "false";
    case J_INT: return std::to_string((long long)p.f);
    case J_FLOAT: return go_format_g(p.f);
    default: return "<nil>";
  }
}

// ---------------------------------------------------------------- glob compilation
void PolicySet::compile_glob(Atom& a, const std::string& p) {
  a.gflags = 0;
  a.gfirst = (uint32_t)gsegs.size();
  a.gcount = 0;
  a.gmin = 0;
  if (p.empty()) { a.gflags = G_EMPTY; return; }
  if (p.find_first_not_of('*') == std::string::npos) { a.gflags = G_ALL; return; }
  if (p[0] == '*') a.gflags |= G_LEAD;
  if (p.back() == '*') a.gflags |= G_TRAIL;
  size_t i = 0;
  while (i < p.size()) {
    size_t j = p.find('*', i);
    if (j == std::string::npos) j = p.size();
    if (j > i) {
      std::string seg = p.substr(i, j - i);
      GSeg g{(uint32_t)gwords.size(), (uint32_t)seg.size()};
      for (size_t w = 0; w < seg.size(); w += 4) {
        GWord gw{0, 0};
        for (size_t b = 0; b < 4 && w + b < seg.size(); b++) {
          unsigned char c = (unsigned char)seg[w + b];
          if (c == '?') { a.gflags |= G_HASQ; continue; }
          gw.w |= (uint32_t)c << (8 * b);
          gw.mask |= 0xFFu << (8 * b);
        }
        gwords.push_back(gw);
      }
      gsegs.push_back(g);
      a.gcount++;
      a.gmin += (uint32_t)seg.size();
    }
    i = j + 1;
  }
}

// ---------------------------------------------------------------- glob (host)
bool wildcard_match_host(std::string_view p, std::string_view s) {
  if (p.empty()) return s.empty();
  if (p == "*") return true;
  auto rl = [](unsigned char c) -> size_t { return c < 0x80 ? 1 : c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 1; };
  size_t si = 0, pi = 0, star = std::string::npos, mark = 0;
  while (si < s.size()) {
    if (pi < p.size() && p[pi] == '*') { star = pi++; mark = si; continue; }
    if (pi < p.size() && p[pi] == '?') {
      si += rl((unsigned char)s[si]);
      pi++;
      continue;
    }
    if (pi < p.size()) {
      size_t w = rl((unsigned char)p[pi]);
      if (si + w <= s.size() && memcmp(p.data() + pi, s.data() + si, w) == 0) { pi += w; si += w; continue; }
    }
    if (star != std::string::npos) {
      pi = star + 1;
      mark += rl((unsigned char)s[mark]);
      si = mark;
      continue;
    }
    return false;
  }
  while (pi < p.size() && p[pi] == '*') pi++;
  return pi == p.size() && si == s.size();
}

// ---------------------------------------------------------------- label validation
static bool re_qname(const std::string& n) {
  auto an = [](char c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
  if (n.empty() || !an(n[0]) || !an(n.back())) return false;
  for (char c : n)
    if (!(an(c) || c == '-' || c == '_' || c == '.')) return false;
  return true;
}
static bool re_dns_sub(const std::string& s) {
  if (s.empty() || s.size() > 253) return false;
  size_t i = 0;
  while (true) {
    size_t j = s.find('.', i);
    std::string lab = s.substr(i, j == std::string::npos ? std::string::npos : j - i);
    auto ok = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
    if (lab.empty() || !ok(lab[0]) || !ok(lab.back())) return false;
    for (char c : lab)
      if (!(ok(c) || c == '-')) return false;
    if (j == std::string::npos) return true;
    i = j + 1;
  }
}
bool valid_label_key(const std::string& k) {
  size_t c = std::count(k.begin(), k.end(), '/');
  std::string name;
  if (c == 0) name = k;
  else if (c == 1) {
    size_t p = k.find('/');
    std::string pre = k.substr(0, p);
    if (pre.empty() || !re_dns_sub(pre)) return false;
    name = k.substr(p + 1);
  } else return false;
  return !name.empty() && name.size() <= 63 && re_qname(name);
}
bool valid_label_value(const std::string& v) { return v.size() <= 63 && (v.empty() || re_qname(v)); }

int selector_eval_host(const SelectorHost& sel, std::vector<std::pair<std::string, std::string>> labels) {
  std::sort(labels.begin(), labels.end());
  std::vector<std::pair<std::string, std::string>> ml = sel.matchLabels;
  std::sort(ml.begin(), ml.end());
  std::map<std::string, std::string> result;
  for (auto& kv : ml) {
    if (has_wild(kv.first) || has_wild(kv.second)) {
      std::string mk = kv.first, mv = kv.second;
      for (auto& c : mk) if (c == '*' || c == '?') c = '0';
      for (auto& c : mv) if (c == '*' || c == '?') c = '0';
      for (auto& r : labels)
        if (wildcard_match_host(kv.first, r.first) && wildcard_match_host(kv.second, r.second)) { mk = r.first; mv = r.second; break; }
      result[mk] = mv;
    } else {
      result[kv.first] = kv.second;
    }
  }
  if (result.empty() && sel.exprs.empty()) return 1;
  for (auto& kv : result)
    if (!valid_label_key(kv.first) || !valid_label_value(kv.second)) return -1;
  for (auto& e : sel.exprs) {
    if (e.op != "In" && e.op != "NotIn" && e.op != "Exists" && e.op != "DoesNotExist") return -1;
    if (!valid_label_key(e.key)) return -1;
    if ((e.op == "In" || e.op == "NotIn") && e.values.empty()) return -1;
    if ((e.op == "Exists" || e.op == "DoesNotExist") && !e.values.empty()) return -1;
    for (auto& v : e.values) if (!valid_label_value(v)) return -1;
  }
  auto get = [&](const std::string& k, std::string* v) {
    for (auto& r : labels) if (r.first == k) { *v = r.second; return true; }
    return false;
  };
  for (auto& kv : result) {
    std::string v;
    if (!get(kv.first, &v) || v != kv.second) return 0;
  }
  for (auto& e : sel.exprs) {
    std::string v;
    bool h = get(e.key, &v);
    bool in = h && std::find(e.values.begin(), e.values.end(), v) != e.values.end();
    if ((e.op == "In" && !in) || (e.op == "NotIn" && in) || (e.op == "Exists" && !h) || (e.op == "DoesNotExist" && h)) return 0;
  }
  return 1;
}

// ---------------------------------------------------------------- PV
PV to_pv(const JDoc& d, uint32_t node) {
  const JNode& n = d.at(node);
  PV v;
  v.t = n.t;
  switch (n.t) {
    case J_BOOL: v.b = n.b; break;
    case J_INT: v.t = J_FLOAT; v.f = (double)n.i; break;
    case J_FLOAT: v.f = n.f; break;
    case J_STR: v.s = std::string(d.sval(n)); break;
    case J_MAP:
      for (uint32_t c = n.first; c < n.first + n.count; c++) {
        v.mk.emplace_back(d.key(d.at(c)));
        v.mo.push_back(v.mk.back());
        v.mv.push_back(to_pv(d, c));
      }
      break;
    case J_ARR:
      for (uint32_t c = n.first; c < n.first + n.count; c++) v.a.push_back(to_pv(d, c));
      break;
    default: break;
  }
  return v;
}

// ---------------------------------------------------------------- $() references
namespace {

std::string fmt_f6(double v) { return go_format_f6(v); }

size_t ref_tail(const std::string& s, size_t k) {
  if (k >= s.size() || s[k] == '\n') return std::string::npos;
  unsigned char c = (unsigned char)s[k];
  size_t w = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 1;
  size_t st = k + w, run = st;
  while (run < s.size() && s[run] != ' ') run++;
  for (size_t p = run; p-- > st;)
    if (s[p] == ')') return p + 1;
  return std::string::npos;
}

std::vector<std::pair<size_t, size_t>> find_refs(const std::string& s) {
  std::vector<std::pair<size_t, size_t>> out;
  size_t i = 0;
  while (i < s.size()) {
    if (i == 0 && s.compare(0, 2, "$(") == 0) {
      size_t e = ref_tail(s, 2);
      if (e != std::string::npos) { out.push_back({0, e}); i = e; continue; }
    }
    if (s[i] != '\\' && s.compare(i + 1, 2, "$(") == 0) {
      size_t e = ref_tail(s, i + 3);
      if (e != std::string::npos) { out.push_back({i, e}); i = e; continue; }
    }
    i++;
  }
  return out;
}

std::string replace_n(const std::string& s, const std::string& from, const std::string& to, int n) {
  if (from.empty()) return s;
  std::string out;
  size_t i = 0;
  int k = 0;
  while (true) {
    size_t j = (n < 0 || k < n) ? s.find(from, i) : std::string::npos;
    if (j == std::string::npos) { out += s.substr(i); return out; }
    out += s.substr(i, j - i) + to;
    i = j + from.size();
    k++;
  }
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
    if (c == "..") {
      if (!parts.empty() && parts.back() != "..") parts.pop_back();
      else if (!rooted) parts.push_back("..");
    } else if (!c.empty() && c != ".") parts.push_back(c);
    i = j + 1;
  }
  std::string out = rooted ? "/" : "";
  for (size_t k = 0; k < parts.size(); k++) out += (k ? "/" : "") + parts[k];
  return out.empty() ? "." : out;
}

std::string remove_anchors_from_path(const std::string& str) {
  std::vector<std::string> comps;
  size_t i = 0;
  while (true) {
    size_t j = str.find('/', i);
    if (j == std::string::npos) { comps.push_back(str.substr(i)); break; }
    comps.push_back(str.substr(i, j - i));
    i = j + 1;
  }
  if (!comps.empty() && comps[0].empty()) comps.erase(comps.begin());
  std::string joined;
  bool any = false;
  for (auto& c : comps) {
    std::string r = remove_anchor(c, nullptr);
    if (!any && r.empty()) continue;
    joined += (any ? "/" : "") + r;
    any = true;
  }
  std::string np = any ? path_clean(joined) : "";
  if (!str.empty() && str[0] == '/') np = "/" + np;
  return np;
}

std::vector<size_t> sorted_idx(const PV& m) {
  std::vector<size_t> idx(m.mk.size());
  for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
  std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return m.mo[a] < m.mo[b]; });
  return idx;
}

struct Found {
  const PV* leaf = nullptr;
  bool is_key = false, any = false;
  std::string key;
};

void find_path(const PV& v, const std::string& path, const std::string& target, Found* f) {
  if (v.t == J_MAP) {
    for (size_t i : sorted_idx(v)) {
      if (remove_anchors_from_path(path) == target) { f->is_key = true; f->key = v.mk[i]; f->leaf = nullptr; f->any = true; }
      find_path(v.mv[i], path + "/" + v.mk[i], target, f);
    }
  } else if (v.t == J_ARR) {
    for (size_t i = 0; i < v.a.size(); i++) find_path(v.a[i], path + "/" + std::to_string(i), target, f);
  } else if (remove_anchors_from_path(path) == target) {
    f->leaf = &v;
    f->is_key = false;
    f->any = true;
  }
}

std::string go_operator(const std::string& p);  // fwd

bool subst_str(const PV& doc, std::string& value, const std::string& dpath, std::string* err) {
  std::string orig = value;
  for (auto& m : find_refs(orig)) {
    std::string v = orig.substr(m.first, m.second - m.first);
    bool initial = v.compare(0, 2, "$(") == 0;
    std::string old = v;
    if (!initial) v = v.substr(1);
    size_t b = 0, e = v.size();
    while (b < e && strchr("$()", v[b])) b++;
    while (e > b && strchr("$()", v[e - 1])) e--;
    std::string p = v.substr(b, e - b);
    std::string op = go_operator(p);
    p = p.substr(op.size());
    if (p.empty()) { *err = "failed to resolve " + v + " at path " + dpath + ": expected path, found empty reference"; return false; }
    std::string abs = p[0] == '/' ? p : (dpath.empty() ? path_clean(p) : path_clean(dpath + "/" + p));
    Found f;
    find_path(doc, "", abs, &f);
    bool is_str = false;
    std::string resolved;
    bool isnil = !f.any || (!f.is_key && f.leaf->t == J_NULL);
    if (op.empty()) {
      if (isnil) { *err = "failed to resolve " + v + " at path " + dpath + ": <nil>"; return false; }
      if (f.is_key) { resolved = f.key; is_str = true; }
      else if (f.leaf->t == J_STR) { resolved = f.leaf->s; is_str = true; }
    } else {
      std::string fv;
      if (f.any && f.is_key) fv = f.key;
      else if (f.any && f.leaf->t == J_STR) fv = f.leaf->s;
      else if (f.any && f.leaf->t == J_FLOAT) fv = fmt_f6(f.leaf->f);
      else {
        std::string vs = "<nil>";
        if (f.any && f.leaf->t == J_BOOL) vs = f.leaf->b ? "true" : "false";
        *err = "failed to resolve " + v + " at path " + dpath + ": incorrect expression: operator " + op +
               " does not match with value " + vs;
        return false;
      }
      resolved = op + fv;
      is_str = true;
    }
    if (!is_str) { *err = "NotResolvedReferenceErr,reference " + v + " not resolved at path " + dpath; return false; }
    value = replace_n(value, old, (initial ? "" : old.substr(0, 1)) + resolved, 1);
  }
  // RegexEscpReferences: \$(...) -> $(...)
  size_t i = 0;
  std::vector<std::string> escs;
  while (i < value.size()) {
    if (value[i] == '\\' && value.compare(i + 1, 2, "$(") == 0) {
      size_t e2 = ref_tail(value, i + 3);
      if (e2 != std::string::npos) { escs.push_back(value.substr(i, e2 - i)); i = e2; continue; }
    }
    i++;
  }
  for (auto& s : escs) value = replace_n(value, s, s.substr(1), -1);
  return true;
}

bool subst_tree(const PV& doc, PV& v, const std::string& path, std::string* err) {
  if (v.t == J_MAP) {
    for (size_t i : sorted_idx(v)) {
      std::string k = v.mk[i];
      std::string nk = k;
      if (!subst_str(doc, nk, path, err)) return false;
      if (!subst_tree(doc, v.mv[i], path + "/" + k, err)) return false;
      if (nk != k) {
        int other = v.find(nk);
        if (other >= 0 && (size_t)other != i) {
          v.mv[other] = v.mv[i];
          v.mo[other] = v.mo[i];
          v.mk.erase(v.mk.begin() + i); v.mo.erase(v.mo.begin() + i); v.mv.erase(v.mv.begin() + i);
          return subst_tree(doc, v, path, err);  // restart scan on the rebuilt map (rare)
        }
        v.mk[i] = nk;
      }
    }
    return true;
  }
  if (v.t == J_ARR) {
    for (size_t i = 0; i < v.a.size(); i++)
      if (!subst_tree(doc, v.a[i], path + "/" + std::to_string(i), err)) return false;
    return true;
  }
  if (v.t == J_STR) return subst_str(doc, v.s, path, err);
  return true;
}

// RegexEscpVariables: \{{...}} -> {{...}}
void unescape_vars_str(std::string& s) {
  size_t i = 0;
  std::vector<std::string> escs;
  while (i < s.size()) {
    if (s[i] == '\\' && s.compare(i + 1, 2, "{{") == 0) {
      size_t k = i + 3;
      while (k < s.size() && s[k] != '{' && s[k] != '}') k++;
      if (s.compare(k, 2, "}}") == 0) { escs.push_back(s.substr(i, k + 2 - i)); i = k + 2; continue; }
    }
    i++;
  }
  for (auto& e : escs) s = replace_n(s, e, e.substr(1), -1);
}
void unescape_vars(PV& v) {
  if (v.t == J_STR) unescape_vars_str(v.s);
  for (auto& k : v.mk) unescape_vars_str(k);
  for (auto& x : v.mv) unescape_vars(x);
  for (auto& x : v.a) unescape_vars(x);
}

bool has_variable(const std::string& s) {
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
bool doc_has_variable(const PV& v) {
  if (v.t == J_STR) return has_variable(v.s);
  for (size_t i = 0; i < v.mk.size(); i++)
    if (has_variable(v.mk[i]) || doc_has_variable(v.mv[i])) return true;
  for (auto& x : v.a)
    if (doc_has_variable(x)) return true;
  return false;
}
bool has_magic(const std::string& s) {
  return s.find("conditional anchor mismatch") != std::string::npos || s.find("global anchor mismatch") != std::string::npos;
}
bool doc_has_magic(const PV& v) {
  if (v.t == J_STR && has_magic(v.s)) return true;
  for (size_t i = 0; i < v.mk.size(); i++)
    if (has_magic(v.mk[i]) || doc_has_magic(v.mv[i])) return true;
  for (auto& x : v.a)
    if (doc_has_magic(x)) return true;
  return false;
}

// ---------------------------------------------------------------- operators / predicates
std::string go_operator(const std::string& p) {
  if (p.size() < 2) return "";
  if (p.compare(0, 2, ">=") == 0) return ">=";
  if (p.compare(0, 2, "<=") == 0) return "<=";
  if (p[0] == '>') return ">";
  if (p[0] == '<') return "<";
  if (p[0] == '!') return "!";
  size_t n = p.size();
  auto numnd = [&](size_t k, size_t* out) {
    size_t s = k;
    while (k < n && p[k] >= '0' && p[k] <= '9') k++;
    if (k == s) return false;
    while (k < n && p[k] != '-') k++;
    *out = k;
    return true;
  };
  size_t k, r;
  if (numnd(0, &k) && k < n && p[k] == '-') {
    if (p[k - 1] == '!' && numnd(k + 1, &r) && r == n) return "!-";
    if (numnd(k + 1, &r) && r == n) return "-";
  }
  return "";
}

uint32_t cmp_op(const std::string& op) {
  if (op.empty()) return CO_EQ;
  if (op == "!") return CO_NE;
  if (op == ">") return CO_GT;
  if (op == "<") return CO_LT;
  if (op == ">=") return CO_GE;
  return CO_LE;
}

std::string trim(const std::string& s, const char* set) {
  size_t b = 0, e = s.size();
  while (b < e && strchr(set, s[b])) b++;
  while (e > b && strchr(set, s[e - 1])) e--;
  return s.substr(b, e - b);
}

std::vector<std::string> split(const std::string& s, const std::string& sep) {
  std::vector<std::string> out;
  size_t i = 0;
  while (true) {
    size_t j = s.find(sep, i);
    if (j == std::string::npos) { out.push_back(s.substr(i)); return out; }
    out.push_back(s.substr(i, j - i));
    i = j + sep.size();
  }
}

}  // namespace

struct Compiler {
  PolicySet& ps;
  explicit Compiler(PolicySet& p) : ps(p) {}

  // one leaf atom: pattern text AFTER operator parsing, with its operator
  uint32_t atom(const std::string& op, const std::string& pat_after_op) {
    std::string pattern = trim(pat_after_op, " \t\n\v\f\r");
    // ^(\d*(\.\d+)?)(.*)
    size_t k = 0, n = pattern.size();
    while (k < n && pattern[k] >= '0' && pattern[k] <= '9') k++;
    size_t ne = k;
    if (k < n && pattern[k] == '.') {
      size_t j = k + 1;
      while (j < n && pattern[j] >= '0' && pattern[j] <= '9') j++;
      if (j > k + 1) ne = j;
    }
    Atom a{};
    a.op = cmp_op(op);
    if (ne == 0) {  // validateString: only Equal/NotEqual
      std::string str = pattern.substr(ne);
      if (a.op == CO_EQ || a.op == CO_NE) {
        a.kind = AT_GLOB_E;
        a.s_off = ps.add_str(str);
        a.s_len = (uint32_t)str.size() | (utf8_ascii(str) ? 0x80000000u : 0);
        ps.compile_glob(a, str);
      } else {
        a.kind = AT_FALSE;
      }
    } else {
      QCanon q = parse_quantity(pattern);
      if (q.valid) {
        a.kind = AT_QCMP;
        a.q_exp = q.exp;
        a.q_hi = q.hi;
        a.q_lo = q.lo;
        a.q_flags = (q.neg ? VF_Q_NEG : 0) | (q.zero ? VF_Q_ZERO : 0);
      } else {
        a.kind = AT_GLOB_N;
        a.s_off = ps.add_str(pattern);
        a.s_len = (uint32_t)pattern.size() | (utf8_ascii(pattern) ? 0x80000000u : 0);
        ps.compile_glob(a, pattern);
      }
    }
    ps.atoms.push_back(a);
    return (uint32_t)ps.atoms.size() - 1;
  }

  // validateValueWithStringPattern(value, pattern) for one '&' part
  Conj conj(const std::string& pattern) {
    std::string op = go_operator(pattern);
    Conj c{};
    if (op == "-") {
      auto ep = split(pattern, "-");
      std::string left = ">=" + ep[0];
      c.kind = CJ_INRANGE;
      c.a0 = atom(go_operator(left), left.substr(go_operator(left).size()));
      c.a1 = atom("<=", ep[1]);
      return c;
    }
    if (op == "!-") {
      auto ep = split(pattern, "!-");
      std::string left = "<" + ep[0];
      c.kind = CJ_NOTINRANGE;
      c.a0 = atom(go_operator(left), left.substr(go_operator(left).size()));
      c.a1 = atom(">", ep[1]);
      return c;
    }
    c.kind = CJ_ATOM;
    c.a0 = atom(op, pattern.substr(op.size()));
    return c;
  }

  uint32_t pred(const PV& p) {
    std::string key;
    switch (p.t) {
      case J_BOOL: key = p.b ? "b1" : "b0"; break;
      case J_FLOAT: { char b[64]; snprintf(b, sizeof b, "f%a", p.f); key = b; break; }
      case J_NULL: key = "n"; break;
      case J_STR: key = "s" + p.s; break;
      case J_MAP: key = "m"; break;
      default: key = "x"; break;
    }
    auto it = ps.pred_cache.find(key);
    if (it != ps.pred_cache.end()) return it->second;
    Pred pr{};
    switch (p.t) {
      case J_BOOL: pr.kind = PK_BOOL; pr.flags = p.b; break;
      case J_FLOAT: {
        pr.kind = PK_FLOAT;
        pr.f = p.f;
        pr.flags = (p.f == std::trunc(p.f)) ? 1 : 0;
        pr.fi = (p.f > -9223372036854775808.0 && p.f < 9223372036854775808.0) ? (int64_t)p.f : INT64_MIN;
        break;
      }
      case J_NULL: pr.kind = PK_NIL; break;
      case J_MAP: pr.kind = PK_MAPTYPE; break;
      case J_STR: {
        pr.kind = PK_STRING;
        std::vector<std::vector<Conj>> alts;
        for (auto& a : split(p.s, "|")) {
          std::vector<Conj> cs;
          for (auto& c : split(trim(a, " "), "&")) cs.push_back(conj(trim(c, " ")));
          alts.push_back(cs);
        }
        pr.first = (uint32_t)ps.alts.size();
        pr.count = (uint32_t)alts.size();
        for (auto& cs : alts) {
          Alt al{(uint32_t)ps.conjs.size(), (uint32_t)cs.size()};
          ps.alts.push_back(al);
          for (auto& c : cs) ps.conjs.push_back(c);
        }
        break;
      }
      default: pr.kind = PK_FALSE; break;
    }
    ps.preds.push_back(pr);
    uint32_t id = (uint32_t)ps.preds.size() - 1;
    ps.pred_cache.emplace(key, id);
    return id;
  }

  // ------------------------------------------------------------ program emission
  struct Scope { uint32_t end_pc = 0xFFFFFFFFu; };
  std::vector<Scope> scopes;
  std::vector<std::pair<uint32_t, uint32_t>> catch_fix;  // (inst, scope) -> c = scope end
  std::vector<std::pair<uint32_t, uint32_t>> skip_fix;   // (inst, scope) -> b = scope end
  std::string cpu_reason;
  uint32_t anchor_bits = 0;
  std::map<std::string, uint32_t> anchor_bit;
  uint32_t level = 0;
  uint32_t rule_flags = 0;
  uint32_t base_pc = 0;
  int array_ctx = 0;  // > 0 inside loops/existence (persistent-mutation semantics)

  uint32_t new_scope() { scopes.push_back(Scope()); return (uint32_t)scopes.size() - 1; }

  uint32_t emit(uint32_t op, uint32_t d, uint32_t aux, uint32_t a, uint32_t b, uint32_t catch_scope) {
    Inst in{op | (d << 8) | (aux << 16), a, b, 0};
    ps.prog.push_back(in);
    uint32_t pc = (uint32_t)ps.prog.size() - 1;
    if (catch_scope != 0xFFFFFFFFu) catch_fix.push_back({pc, catch_scope});
    if (d + 2 > ps.max_depth) ps.max_depth = d + 2;
    return pc;
  }
  void end_scope(uint32_t s, uint32_t pc) { scopes[s].end_pc = pc; }

  uint32_t pnode(uint32_t parent, uint8_t seg, uint32_t level_or_idx, const std::string& key) {
    ps.pnodes.push_back(PNodeInfo{parent, seg, level_or_idx, key});
    return (uint32_t)ps.pnodes.size() - 1;
  }

  uint32_t key(const std::string& k) { return ps.intern(k); }

  static bool hasNestedAnchors(const PV& p) {
    if (p.t == J_MAP) {
      for (auto& k : p.mk)
        if (is_condition_anchor(k) || is_existence_anchor(k) || is_equality_anchor(k) || is_negation_anchor(k) ||
            is_global_anchor(k))
          return true;
      for (auto& v : p.mv)
        if (hasNestedAnchors(v)) return true;
      return false;
    }
    if (p.t == J_ARR) {
      for (auto& v : p.a)
        if (hasNestedAnchors(v)) return true;
    }
    return false;
  }

  static int anchor_rank(const std::string& k) {
    if (is_condition_anchor(k)) return 0;
    if (is_existence_anchor(k)) return 1;
    if (is_equality_anchor(k)) return 2;
    if (is_negation_anchor(k)) return 3;
    return -1;
  }

  std::vector<size_t> canonical_children(const PV& P) {
    std::vector<size_t> anc, res;
    for (size_t i = 0; i < P.mk.size(); i++) (anchor_rank(P.mk[i]) >= 0 ? anc : res).push_back(i);
    std::sort(anc.begin(), anc.end(), [&](size_t a, size_t b) {
      int ra = anchor_rank(P.mk[a]), rb = anchor_rank(P.mk[b]);
      return ra != rb ? ra < rb : P.mo[a] < P.mo[b];
    });
    std::sort(res.begin(), res.end(), [&](size_t a, size_t b) {
      bool fa = is_global_anchor(P.mk[a]) || hasNestedAnchors(P.mv[a]);
      bool fb = is_global_anchor(P.mk[b]) || hasNestedAnchors(P.mv[b]);
      return fa != fb ? fa : P.mo[a] < P.mo[b];
    });
    anc.insert(anc.end(), res.begin(), res.end());
    return anc;
  }

  void trie_of(const PV& P, uint32_t t, bool under_metadata = false) {
    if (P.t == J_MAP) {
      for (size_t i = 0; i < P.mk.size(); i++) {
        std::string k = remove_anchor(P.mk[i], nullptr);
        uint32_t c = ps.trie.child(t, k);
        // labels/annotations below metadata: wildcard keys resolve against every resource key
        if (under_metadata && (k == "labels" || k == "annotations")) ps.trie.nodes[c].keep_all = true;
        trie_of(P.mv[i], c, k == "metadata");
      }
    } else if (P.t == J_ARR) {
      uint32_t e = ps.trie.elem(t);
      for (auto& x : P.a) trie_of(x, e);
    }
  }

  // validateResourceElement(cur[d], P) ; errors -> catch scope
  // slot fixups of this rule's key-lookup ops: (pc, trie node of the map, key)
  std::vector<std::tuple<uint32_t, uint32_t, std::string>> slot_fix;
  void lookup_fix(uint32_t pc, uint32_t t, const std::string& k) { slot_fix.emplace_back(pc, t, k); }

  // validateResourceElement(cur[d], P); t = projection-trie node of cur[d]
  // message operands of the pattern value compared at pnode pn
  void note_pattern(uint32_t pn, const PV& P) {
    PNodeInfo& n = ps.pnodes[pn];
    n.pat_t = go_T(P);
    n.pat_len = (uint32_t)P.a.size();
    n.pat_v = go_v(P.t == J_ARR && !P.a.empty() ? P.a[0] : P);
  }

  void elem(const PV& P, uint32_t d, uint32_t pn, uint32_t cs, uint32_t t, int expand_tag = 0) {
    if (d >= 30) { cpu_reason = "pattern too deep"; return; }
    note_pattern(pn, P);
    if (P.t == J_MAP) {
      emit(OP_MAPCHK, d, 0, pn, 0, cs);
      // CheckAnchorInResource: condition / existence / negation keys of this map
      for (size_t i = 0; i < P.mk.size(); i++) {
        const std::string& k = P.mk[i];
        if (is_condition_anchor(k) || is_existence_anchor(k) || is_negation_anchor(k)) {
          if (expand_tag && has_wild(k)) { cpu_reason = "anchored wildcard metadata key"; return; }
          auto it = anchor_bit.find(k);
          uint32_t bit;
          if (it == anchor_bit.end()) {
            bit = anchor_bits++;
            if (bit >= 64) { cpu_reason = "more than 64 anchor keys"; return; }
            anchor_bit[k] = bit;
          } else {
            bit = it->second;
          }
          uint32_t apc = emit(OP_AREG, d, bit, key(remove_anchor(k, nullptr)), 0, 0xFFFFFFFFu);
          lookup_fix(apc, t, remove_anchor(k, nullptr));
        }
      }
      // ExpandInMetadata site: this map has a key whose anchor-free form is "metadata"
      int meta = -1;
      for (size_t i = 0; i < P.mk.size(); i++)
        if (remove_anchor(P.mk[i], nullptr) == "metadata" && (meta < 0 || P.mo[i] < P.mo[meta])) meta = (int)i;
      std::set<size_t> expand_children;
      if (meta >= 0 && P.mv[meta].t != J_NULL) {
        const PV& md = P.mv[meta];
        if (md.t != J_MAP) { cpu_reason = "non-map metadata pattern (ExpandInMetadata panic)"; return; }
        for (const char* tag : {"labels", "annotations"}) {
          int lk = -1;
          for (size_t i = 0; i < md.mk.size(); i++)
            if (remove_anchor(md.mk[i], nullptr) == tag && (lk < 0 || md.mo[i] < md.mo[lk])) lk = (int)i;
          if (lk < 0 || md.mv[lk].t == J_NULL) continue;
          const PV& lm = md.mv[lk];
          if (lm.t != J_MAP) { cpu_reason = "non-map labels pattern (ExpandInMetadata panic)"; return; }
          for (auto& v : lm.mv)
            if (v.t != J_STR) { cpu_reason = "non-string label pattern value (ExpandInMetadata panic)"; return; }
          bool wild = false;
          for (auto& k : lm.mk) wild |= has_wild(k);
          if (wild && array_ctx > 0) { cpu_reason = "wildcard metadata keys under an array"; return; }
          rule_flags |= RR_META_EXPAND | (tag[0] == 'l' ? RR_META_LABELS : RR_META_ANN);
        }
        if (rule_flags & RR_META_EXPAND) emit(OP_METACHK, d, 0, 0, 0, cs);
      }
      children(P, d, pn, cs, meta, expand_tag, t);
      return;
    }
    if (P.t == J_ARR) {
      emit(OP_ARRCHK, d, 0, pn, 0, cs);
      if (P.a.empty()) {
        emit(OP_RAISE, d, 0, pn, E_EMPTY_PATARR, cs);
        return;
      }
      const PV& p0 = P.a[0];
      if (p0.t == J_MAP) {
        uint32_t L = level++;
        if (L >= 4) { cpu_reason = "more than 4 nested array levels"; return; }
        uint32_t s = new_scope();
        uint32_t epn = pnode(pn, SEG_LOOP, L, "");
        uint32_t b = emit(OP_LOOP_BEGIN, d, L, 0, 0, 0xFFFFFFFFu);
        array_ctx++;
        elem(p0, d + 1, epn, s, ps.trie.elem(t));
        array_ctx--;
        uint32_t e = emit(OP_LOOP_END, d, L, b, 0, cs);
        ps.prog[b].a = e;
        end_scope(s, e);
        level--;
        return;
      }
      if (p0.t != J_ARR) {  // scalar: every element
        leaf(p0, d, pn, cs);
        return;
      }
      // nested arrays: positional
      emit(OP_LENCHK, d, 0, (uint32_t)P.a.size(), pn, cs);
      for (size_t i = 0; i < P.a.size(); i++) {
        uint32_t s = new_scope();
        emit(OP_INDEX, d, 0, (uint32_t)i, 0, 0xFFFFFFFFu);
        uint32_t ipn = pnode(pn, SEG_CONST_INDEX, (uint32_t)i, "");
        array_ctx++;
        elem(P.a[i], d + 1, ipn, s, ps.trie.elem(t));
        array_ctx--;
        uint32_t e = emit(OP_POS_END, d, 0, 0, 0, cs);
        end_scope(s, e);
      }
      return;
    }
    leaf(P, d, pn, cs);
  }

  // scalar pattern leaf: a compiled predicate, or (a string holding variables) a dynamic
  // leaf whose predicate is the resource's substituted value (kvvars.cpp)
  void leaf(const PV& P, uint32_t d, uint32_t pn, uint32_t cs) {
    if (P.t == J_STR && P.vstr >= 0) {
      const uint32_t dl = (uint32_t)ps.dleaf_vstr.size();
      ps.dleaf_vstr.push_back((uint32_t)P.vstr);
      ps.pnodes[pn].dleaf = (int32_t)dl;
      emit(OP_VLEAF, d, 0, dl, pn, cs);
      return;
    }
    emit(OP_LEAF, d, 0, pred(P), pn, cs);
  }

  void children(const PV& P, uint32_t d, uint32_t pn, uint32_t cs, int meta_idx, int expand_tag, uint32_t t) {
    std::vector<size_t> order = canonical_children(P);
    // Label/annotation map below an ExpandInMetadata site: wildcard keys are
    // resolved per resource (OP_KEYGLOB) and a later canonical sibling that
    // resolves to the same result key overwrites (drops) an earlier one.
    bool label_map = expand_tag == 1;
    bool wild_any = false;
    if (label_map)
      for (auto& k : P.mk) wild_any |= has_wild(remove_anchor(k, nullptr));
    bool kg = label_map && wild_any;
    bool saved = in_label_map_with_wild;
    std::vector<uint32_t> saved_pending;
    saved_pending.swap(pending_keyglob);
    in_label_map_with_wild = kg;
    for (size_t oi : order) {
      const std::string& k = P.mk[oi];
      const PV& Pk = P.mv[oi];
      int child_tag = 0;
      if ((int)oi == meta_idx && Pk.t == J_MAP) child_tag = -1;  // metadata map: its labels/annotations expand
      if (expand_tag == -1) {
        std::string ak = remove_anchor(k, nullptr);
        if (ak == "labels" || ak == "annotations") child_tag = 1;
      }
      bool wildkey = label_map && has_wild(remove_anchor(k, nullptr));
      if (is_condition_anchor(k) || is_global_anchor(k)) {
        bool global = !is_condition_anchor(k);
        std::string ak = remove_anchor(k, nullptr);
        uint32_t cpn = pnode(pn, wildkey ? SEG_RESOLVED : SEG_KEY, 0, ak);
        ps.pnodes[cpn].wrap = global ? 2 : 1;
        uint32_t s = new_scope();
        uint32_t kpc = key_op(d, ak, wildkey, true, t);
        skip_fix.push_back({kpc, s});
        elem(Pk, d + 1, cpn, s, ps.trie.child(t, ak), child_tag);
        uint32_t e = emit(OP_SCOPE_END, d, global ? EF_GLOBAL : EF_COND, 0, 0, cs);
        end_scope(s, e);
      } else if (is_existence_anchor(k)) {
        std::string ak = remove_anchor(k, nullptr);
        if (wildkey) { cpu_reason = "anchored wildcard metadata key"; break; }
        uint32_t cpn = pnode(pn, SEG_KEY, 0, ak);
        note_pattern(cpn, Pk);
        uint32_t s = new_scope();
        uint32_t kpc = key_op(d, ak, false, true, t);
        skip_fix.push_back({kpc, s});
        emit(OP_EXISTCHK, d + 1, 0, cpn, 0, cs);
        const uint32_t et = ps.trie.elem(ps.trie.child(t, ak));
        if (Pk.t != J_ARR) {
          emit(OP_RAISE, d + 1, 0, cpn, E_EXIST_PATLIST, cs);
        } else {
          for (const PV& pm : Pk.a) {
            if (pm.t != J_MAP) {
              emit(OP_RAISE, d + 1, 0, cpn, E_EXIST_PATMAP, cs);
              break;
            }
            uint32_t L = level++;
            if (L >= 4) { cpu_reason = "more than 4 nested array levels"; break; }
            uint32_t es = new_scope();
            uint32_t epn = pnode(cpn, SEG_LOOP, L, "");
            uint32_t b = emit(OP_EXIST_BEGIN, d + 1, L, 0, cpn, cs);
            array_ctx++;
            elem(pm, d + 2, epn, es, et);
            array_ctx--;
            uint32_t e = emit(OP_EXIST_END, d + 1, L, b, cpn, cs);
            ps.prog[b].a = e;
            end_scope(es, e);
            level--;
          }
        }
        uint32_t e = emit(OP_SCOPE_END, d, 0, 0, 0, cs);
        end_scope(s, e);
      } else if (is_equality_anchor(k)) {
        std::string ak = remove_anchor(k, nullptr);
        uint32_t cpn = pnode(pn, wildkey ? SEG_RESOLVED : SEG_KEY, 0, ak);
        uint32_t s = new_scope();
        uint32_t kpc = key_op(d, ak, wildkey, true, t);
        skip_fix.push_back({kpc, s});
        elem(Pk, d + 1, cpn, cs, ps.trie.child(t, ak), child_tag);
        uint32_t e = emit(OP_SCOPE_END, d, 0, 0, 0, 0xFFFFFFFFu);
        end_scope(s, e);
      } else if (is_negation_anchor(k)) {
        std::string ak = remove_anchor(k, nullptr);
        if (wildkey) { cpu_reason = "anchored wildcard metadata key"; break; }
        uint32_t cpn = pnode(pn, SEG_KEY, 0, ak);
        lookup_fix(emit(OP_NEG, d, 0, key(ak), cpn, cs), t, ak);
        if (kg) pending_keyglob.push_back(0xFFFFFFFFu);  // keeps sibling numbering aligned
      } else {
        uint32_t cpn = pnode(pn, wildkey ? SEG_RESOLVED : SEG_KEY, 0, k);
        if (kg) {
          uint32_t s = new_scope();
          uint32_t kpc = key_op(d, k, wildkey, false, t);
          skip_fix.push_back({kpc, s});
          if (Pk.t == J_STR && Pk.s == "*") emit(OP_STAR, d, 0, 0, cpn, cs);  // path: parent of cpn
          else elem(Pk, d + 1, cpn, cs, ps.trie.child(t, k), child_tag);
          uint32_t e = emit(OP_SCOPE_END, d, 0, 0, 0, 0xFFFFFFFFu);
          end_scope(s, e);
        } else {
          lookup_fix(emit(OP_KEYV, d, 0, key(k), 0, 0xFFFFFFFFu), t, k);
          if (Pk.t == J_STR && Pk.s == "*") emit(OP_STAR, d, 0, 0, cpn, cs);  // path: parent of cpn
          else elem(Pk, d + 1, cpn, cs, ps.trie.child(t, k), child_tag);
        }
      }
      if (!cpu_reason.empty()) break;
    }
    if (kg && cpu_reason.empty()) {
      // sibling spec: per child (canonical order): [class | wild, atom (wild) or key id]
      // class = anchor prefix kind: 0 none, 1 "=(", 2 "<(", 3 other anchors
      std::vector<uint32_t> spec;
      for (size_t j = 0; j < order.size(); j++) {
        const std::string& k = P.mk[order[j]];
        std::string pre;
        std::string ak = remove_anchor(k, &pre);
        uint32_t cls = pre.empty() ? 0 : pre == "=(" ? 1 : pre == "<(" ? 2 : 3;
        uint32_t pc = pending_keyglob[j];
        bool w = has_wild(ak);
        spec.push_back((cls << 1) | (w ? 1u : 0u));
        spec.push_back(pc != 0xFFFFFFFFu ? (w ? ps.prog[pc].a : ps.prog[pc].c) : key(ak));
      }
      uint32_t off = (uint32_t)ps.kg_specs.size();
      ps.kg_specs.push_back((uint32_t)order.size());
      ps.kg_specs.insert(ps.kg_specs.end(), spec.begin(), spec.end());
      for (size_t j = 0; j < pending_keyglob.size(); j++) {
        uint32_t pc = pending_keyglob[j];
        if (pc == 0xFFFFFFFFu) continue;
        ps.prog[pc].op = (ps.prog[pc].op & 0x00FFFFFFu) | ((uint32_t)j << 24);
        ps.atoms[ps.prog[pc].a].q_hi = off;
        ps.atoms[ps.prog[pc].a].q_lo = spec[2 * j] >> 1;  // my class
      }
    }
    pending_keyglob.swap(saved_pending);
    in_label_map_with_wild = saved;
  }

  std::vector<uint32_t> pending_keyglob;  // pcs of key ops of the current wildcard label map

  uint32_t glob_atom(const std::string& g) {
    Atom a{};
    a.kind = AT_GLOB_E;
    a.op = CO_EQ;
    a.s_off = ps.add_str(g);
    a.s_len = (uint32_t)g.size() | (utf8_ascii(g) ? 0x80000000u : 0);
    ps.compile_glob(a, g);
    ps.atoms.push_back(a);
    return (uint32_t)ps.atoms.size() - 1;
  }

  // Key lookup op (absent -> skip target when skip_absent; patched by caller).
  uint32_t key_op(uint32_t d, const std::string& ak, bool wild, bool skip_absent, uint32_t t) {
    if (!in_label_map_with_wild) {
      uint32_t pc = emit(skip_absent ? OP_KEY : OP_KEYV, d, 0, key(ak), 0, 0xFFFFFFFFu);
      lookup_fix(pc, t, ak);
      return pc;
    }
    // OP_KEYGLOB: a = atom (glob, AT_FALSE for a literal sibling), b = skip target, c = literal key id
    uint32_t at = glob_atom(wild ? ak : std::string());
    if (!wild) ps.atoms[at].kind = AT_FALSE;
    uint32_t pc = emit(OP_KEYGLOB, d, skip_absent ? 1u : 0u, at, 0, 0xFFFFFFFFu);
    ps.prog[pc].c = key(ak);
    pending_keyglob.push_back(pc);
    return pc;
  }
  bool in_label_map_with_wild = false;
};

// ---------------------------------------------------------------- policies
namespace {

// Pattern strings holding variables, in the reference's traversal order (jsonutils/traverse.go:
// per map entry the key then the value, keys in canonical byte order; arrays in order), with
// their traversal paths: marks each with its VarStr and unescapes `\{{..}}` in every other
// string and key (substituteVariablesIfAny unescapes each leaf / key it visits, vars.go:393-395).
static void collect_var_strings(PolicySet& ps, PV& v, const std::string& path, uint32_t rule, bool label_value,
                                std::map<std::pair<std::string, std::string>, uint32_t>& keys) {
  if (v.t == J_STR) {
    if (!var_string(v.s)) {
      v.s = unescape_var_string(v.s);
      return;
    }
    VarStr vs;
    vs.rule = rule;
    vs.text = v.s;
    vs.path = path;
    vs.want_string = label_value;
    auto k = std::make_pair(v.s, path);
    auto it = keys.find(k);
    if (it == keys.end()) {
      it = keys.emplace(k, (uint32_t)ps.vkeys.size()).first;
      ps.vkeys.push_back(k);
    }
    vs.key = it->second;
    v.vstr = (int32_t)ps.vstrs.size();
    ps.vstrs.push_back(vs);
    return;
  }
  if (v.t == J_MAP) {
    std::vector<size_t> idx(v.mk.size());
    for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return v.mk[a] < v.mk[b]; });
    for (size_t i : idx) {
      const std::string k = v.mk[i];
      const std::string ak = remove_anchor(k, nullptr);
      // values of metadata.labels / annotations maps (ExpandInMetadata reads them as strings)
      const bool lbl = (ak == "labels" || ak == "annotations") && path.size() >= 9 &&
                       remove_anchor(path.substr(path.rfind('/') + 1), nullptr) == "metadata";
      collect_var_strings(ps, v.mv[i], path + "/" + k, rule, false, keys);
      if (lbl && v.mv[i].t == J_MAP)
        for (auto& x : v.mv[i].mv)
          if (x.t == J_STR && x.vstr >= 0) ps.vstrs[x.vstr].want_string = true;
      const std::string nk = unescape_var_string(k);
      if (nk != k) {
        v.mk[i] = nk;
        if (v.mo[i] == k) v.mo[i] = nk;
      }
    }
    return;
  }
  if (v.t == J_ARR)
    for (size_t i = 0; i < v.a.size(); i++)
      collect_var_strings(ps, v.a[i], path + "/" + std::to_string(i), rule, false, keys);
}

// every variable of the document is request.object<path> or @ (kvvars.cpp), none in a key
static bool pattern_vars_in_scope(const PV& v, const std::string& path) {
  if (v.t == J_STR) return !var_string(v.s) || var_string_in_scope(v.s, path);
  if (v.t == J_MAP) {
    for (size_t i = 0; i < v.mk.size(); i++)
      if (var_string(v.mk[i]) || !pattern_vars_in_scope(v.mv[i], path + "/" + v.mk[i])) return false;
    return true;
  }
  if (v.t == J_ARR)
    for (size_t i = 0; i < v.a.size(); i++)
      if (!pattern_vars_in_scope(v.a[i], path + "/" + std::to_string(i))) return false;
  return true;
}

std::string jstr(const JDoc& d, int64_t n) {
  if (n < 0 || d.at((uint32_t)n).t != J_STR) return "";
  return std::string(d.sval(d.at((uint32_t)n)));
}

bool jstrlist(const JDoc& d, int64_t n, std::vector<std::string>* out) {
  if (n < 0) return false;
  const JNode& v = d.at((uint32_t)n);
  if (v.t == J_NULL) return false;
  if (v.t != J_ARR) throw std::runtime_error("policy: expected a list");
  for (uint32_t c = v.first; c < v.first + v.count; c++) out->push_back(jstr(d, c));
  return true;
}

bool jstrmap(const JDoc& d, int64_t n, std::vector<std::pair<std::string, std::string>>* out) {
  if (n < 0) return false;
  const JNode& v = d.at((uint32_t)n);
  if (v.t == J_NULL) return false;
  if (v.t != J_MAP) throw std::runtime_error("policy: expected a map");
  for (uint32_t c = v.first; c < v.first + v.count; c++) out->push_back({std::string(d.key(d.at(c))), jstr(d, c)});
  return true;
}

std::string go_title(std::string s) {
  bool prev_sep = true;
  for (auto& c : s) {
    bool alnum = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_' ||
                 (unsigned char)c >= 0x80;
    if (prev_sep && c >= 'a' && c <= 'z') c = (char)(c - 'a' + 'A');
    prev_sep = !alnum;
  }
  return s;
}

}  // namespace

static void compile_filter(Compiler& C, const JDoc& d, int64_t fnode, int64_t rdnode, bool is_match, RuleHost& rh) {
  PolicySet& ps = C.ps;
  MFilter f{};
  UserInfoSpec ui;
  if (fnode >= 0 && d.at((uint32_t)fnode).t == J_MAP) {
    std::vector<std::string> tmp;
    bool r = jstrlist(d, d.get((uint32_t)fnode, "roles"), &ui.roles);
    bool c = jstrlist(d, d.get((uint32_t)fnode, "clusterRoles"), &ui.clusterRoles);
    int64_t sn = d.get((uint32_t)fnode, "subjects");
    bool s = false;
    if (sn >= 0 && d.at((uint32_t)sn).t == J_ARR) {
      s = true;
      const JNode& a = d.at((uint32_t)sn);
      for (uint32_t k = a.first; k < a.first + a.count; k++)
        ui.subjects.push_back({jstr(d, d.get(k, "kind")), jstr(d, d.get(k, "name")), jstr(d, d.get(k, "namespace"))});
    }
    ui.present = r || c || s;
  }
  bool rd_empty = true;
  std::vector<uint32_t> name_atoms;
  if (rdnode >= 0 && d.at((uint32_t)rdnode).t == J_MAP) {
    uint32_t rn = (uint32_t)rdnode;
    std::vector<std::string> kinds, names, nss;
    std::vector<std::pair<std::string, std::string>> ann;
    bool kp = jstrlist(d, d.get(rn, "kinds"), &kinds);
    std::string name = jstr(d, d.get(rn, "name"));
    bool np = jstrlist(d, d.get(rn, "names"), &names);
    bool nsp = jstrlist(d, d.get(rn, "namespaces"), &nss);
    bool ap = jstrmap(d, d.get(rn, "annotations"), &ann);
    int64_t sel = d.get(rn, "selector");
    int64_t nssel = d.get(rn, "namespaceSelector");
    bool selp = sel >= 0 && d.at((uint32_t)sel).t != J_NULL;
    bool nsselp = nssel >= 0 && d.at((uint32_t)nssel).t != J_NULL;
    rd_empty = !kp && name.empty() && !np && !nsp && !ap && !selp && !nsselp;
    if (!kinds.empty()) {
      f.flags |= MF_KINDS;
      f.kinds_first = (uint32_t)ps.kinds.size();
      for (auto& k : kinds) {
        std::vector<std::string> sp;
        size_t i = 0;
        while (true) {
          size_t j = k.find('/', i);
          if (j == std::string::npos) { sp.push_back(k.substr(i)); break; }
          sp.push_back(k.substr(i, j - i));
          i = j + 1;
        }
        KindSpec ks{};
        if (sp.size() == 1) {
          ks.form = k == "*" ? 3 : 0;
          ks.kind = ps.intern(go_title(k));
        } else if (sp.size() == 2) {
          ks.form = 1;
          ks.kind = ps.intern(go_title(sp[1]));
          ks.version = ps.intern(sp[0]);
        } else {
          ks.form = 2;
          ks.group = ps.intern(sp[0]);
          ks.version = ps.intern(sp[1]);
          ks.kind = ps.intern(go_title(sp[2]));
        }
        ps.kinds.push_back(ks);
      }
      f.kinds_count = (uint32_t)kinds.size();
    }
    // name globs are per resource (no interning): compiled word globs for the
    // specialized kernels (filter_name_atoms), strings for the bytecode VM
    if (!name.empty()) {
      f.flags |= MF_NAME;
      f.name_off = ps.add_str(name);
      f.name_len = (uint32_t)name.size();
      name_atoms.push_back(C.glob_atom(name));
    }
    if (!names.empty()) {
      f.flags |= MF_NAMES;
      f.names_first = (uint32_t)ps.strrefs.size();
      for (auto& n : names) ps.strrefs.push_back({ps.add_str(n), (uint32_t)n.size()});
      f.names_count = (uint32_t)names.size();
      for (auto& n : names) name_atoms.push_back(C.glob_atom(n));
    }
    if (!nss.empty()) {
      f.flags |= MF_NSS;
      f.nss_first = (uint32_t)ps.strrefs.size();
      for (auto& n : nss) ps.strrefs.push_back({ps.add_str(n), (uint32_t)n.size()});
      f.nss_count = (uint32_t)nss.size();
      f.nss_bit = ps.n_nss_bits++;
    }
    if (!ann.empty()) {
      f.flags |= MF_ANN;
      f.ann_first = (uint32_t)ps.strpairs.size();
      for (auto& kv : ann)
        ps.strpairs.push_back({ps.add_str(kv.first), (uint32_t)kv.first.size(), ps.add_str(kv.second), (uint32_t)kv.second.size()});
      f.ann_count = (uint32_t)ann.size();
      f.ann_bit = ps.n_ann_bits++;
    }
    auto parse_sel = [&](uint32_t sn, SelectorHost* sh) {
      jstrmap(d, d.get(sn, "matchLabels"), &sh->matchLabels);
      int64_t me = d.get(sn, "matchExpressions");
      if (me >= 0 && d.at((uint32_t)me).t == J_ARR) {
        const JNode& a = d.at((uint32_t)me);
        for (uint32_t k = a.first; k < a.first + a.count; k++) {
          SelectorHost::Expr e;
          e.key = jstr(d, d.get(k, "key"));
          e.op = jstr(d, d.get(k, "operator"));
          jstrlist(d, d.get(k, "values"), &e.values);
          sh->exprs.push_back(e);
        }
      }
    };
    if (selp) {
      SelectorHost sh;
      parse_sel((uint32_t)sel, &sh);
      Selector S{};
      std::sort(sh.matchLabels.begin(), sh.matchLabels.end());
      // duplicate JSON keys already resolved by the parser; canonical order = byte-lex
      S.ml_first = (uint32_t)ps.sellabels.size();
      bool static_invalid = false;
      for (auto& kv : sh.matchLabels) {
        SelLabel L{};
        bool wild = has_wild(kv.first) || has_wild(kv.second);
        L.k_off = ps.add_str(kv.first); L.k_len = (uint32_t)kv.first.size();
        L.v_off = ps.add_str(kv.second); L.v_len = (uint32_t)kv.second.size();
        if (wild) {
          std::string rk = kv.first, rv = kv.second;
          for (auto& c : rk) if (c == '*' || c == '?') c = '0';
          for (auto& c : rv) if (c == '*' || c == '?') c = '0';
          L.rk_off = ps.add_str(rk); L.rk_len = (uint32_t)rk.size();
          L.rv_off = ps.add_str(rv); L.rv_len = (uint32_t)rv.size();
          L.flags = SL_WILD | ((valid_label_key(rk) && valid_label_value(rv)) ? SL_VALID : 0);
        } else {
          L.flags = (valid_label_key(kv.first) && valid_label_value(kv.second)) ? SL_VALID : 0;
        }
        ps.sellabels.push_back(L);
      }
      S.ml_count = (uint32_t)sh.matchLabels.size();
      S.me_first = (uint32_t)ps.selexprs.size();
      for (auto& e : sh.exprs) {
        SelExpr E{};
        if (e.op == "In") E.op = 0;
        else if (e.op == "NotIn") E.op = 1;
        else if (e.op == "Exists") E.op = 2;
        else if (e.op == "DoesNotExist") E.op = 3;
        else static_invalid = true;
        if (!valid_label_key(e.key)) static_invalid = true;
        if ((E.op <= 1) && e.values.empty()) static_invalid = true;
        if ((E.op >= 2) && !e.values.empty()) static_invalid = true;
        for (auto& v : e.values) if (!valid_label_value(v)) static_invalid = true;
        E.k_off = ps.add_str(e.key); E.k_len = (uint32_t)e.key.size();
        E.v_first = (uint32_t)ps.strrefs.size();
        for (auto& v : e.values) ps.strrefs.push_back({ps.add_str(v), (uint32_t)v.size()});
        E.v_count = (uint32_t)e.values.size();
        ps.selexprs.push_back(E);
      }
      S.me_count = (uint32_t)sh.exprs.size();
      if (sh.matchLabels.empty() && sh.exprs.empty()) S.flags |= SF_EVERYTHING;
      if (static_invalid) S.flags |= SF_STATIC_INVALID;
      f.flags |= MF_SEL;
      f.sel = (uint32_t)ps.selectors.size();
      ps.selectors.push_back(S);
    }
    if (nsselp) {
      SelectorHost sh;
      parse_sel((uint32_t)nssel, &sh);
      f.flags |= MF_NSSEL;
      f.nssel_bit = (uint32_t)ps.nsselectors.size();
      ps.nsselectors.push_back(sh);
    }
  }
  if (rd_empty && !(ui.present && !is_match)) {
    // match: empty RD and (UserInfo emptied or empty) is decided at launch (user info
    // is cleared for an empty AdmissionInfo); exclude: empty RD + empty UI -> not applied
  }
  if (rd_empty) f.flags |= MF_EMPTY;  // refined with user info at launch time
  ps.filters.push_back(f);
  ps.filter_name_atoms.push_back(name_atoms);
  rh.filter_ui.push_back(ui);
  rh.filter_is_match.push_back(is_match);
}

static void compile_block(Compiler& C, const JDoc& d, int64_t blk, bool is_match, RuleRec& rr, RuleHost& rh) {
  uint32_t* mode = is_match ? &rr.m_mode : &rr.x_mode;
  uint32_t* first = is_match ? &rr.m_first : &rr.x_first;
  uint32_t* count = is_match ? &rr.m_count : &rr.x_count;
  *first = (uint32_t)C.ps.filters.size();
  *mode = 0;
  if (blk >= 0 && d.at((uint32_t)blk).t == J_MAP) {
    uint32_t b = (uint32_t)blk;
    int64_t any = d.get(b, "any"), all = d.get(b, "all");
    if (any >= 0 && d.at((uint32_t)any).t == J_ARR && d.at((uint32_t)any).count > 0) {
      *mode = 1;
      const JNode& a = d.at((uint32_t)any);
      for (uint32_t k = a.first; k < a.first + a.count; k++) compile_filter(C, d, k, d.get(k, "resources"), is_match, rh);
    } else if (all >= 0 && d.at((uint32_t)all).t == J_ARR && d.at((uint32_t)all).count > 0) {
      *mode = 2;
      const JNode& a = d.at((uint32_t)all);
      for (uint32_t k = a.first; k < a.first + a.count; k++) compile_filter(C, d, k, d.get(k, "resources"), is_match, rh);
    } else {
      compile_filter(C, d, b, d.get(b, "resources"), is_match, rh);
    }
  } else {
    compile_filter(C, d, -1, -1, is_match, rh);
  }
  *count = (uint32_t)C.ps.filters.size() - *first;
}

// Emits the full pattern program of one rule; returns false (with reason) if CPU-routed.
static bool compile_pattern_program(Compiler& C, const std::vector<PV>& patterns, bool any, RuleRec& rr, RuleHost& rh) {
  PolicySet& ps = C.ps;
  rr.prog = (uint32_t)ps.prog.size();
  C.scopes.clear();
  C.catch_fix.clear();
  C.skip_fix.clear();
  C.cpu_reason.clear();
  C.rule_flags = 0;
  C.slot_fix.clear();
  uint32_t root_scope = C.new_scope();
  for (size_t ai = 0; ai < patterns.size(); ai++) {
    C.anchor_bits = 0;
    C.anchor_bit.clear();
    C.level = 0;
    C.array_ctx = 0;
    uint32_t alt_scope = any ? C.new_scope() : root_scope;
    if (any) C.emit(OP_ALT_BEGIN, 0, 0, (uint32_t)ai, 0, 0xFFFFFFFFu);
    uint32_t root = C.pnode(0xFFFFFFFFu, SEG_ROOT, 0, "");
    if (any) rh.alt_roots.push_back(root);
    else rh.root_pnode = root;
    C.trie_of(patterns[ai], 0);  // before emission: key ops resolve their trie slots
    C.elem(patterns[ai], 0, root, alt_scope, 0);
    if (!C.cpu_reason.empty()) {
      ps.prog.resize(rr.prog);
      rh.route_reason = C.cpu_reason;
      return false;
    }
    if (any) {
      uint32_t e = C.emit(OP_ALT_END, 0, 0, (uint32_t)ai, ai + 1 == patterns.size() ? 1u : 0u, 0xFFFFFFFFu);
      C.end_scope(alt_scope, e);
    }
  }
  uint32_t done = C.emit(OP_DONE, 0, 0, 0, 0, 0xFFFFFFFFu);
  C.end_scope(root_scope, done);
  for (auto& f : C.catch_fix) ps.prog[f.first].c = C.scopes[f.second].end_pc;
  for (auto& f : C.skip_fix) ps.prog[f.first].b = C.scopes[f.second].end_pc;
  rr.flags |= C.rule_flags;
  for (auto& f : C.slot_fix) ps.slot_fix.push_back(f);
  return true;
}

void compile_policies(const char* json, size_t len, PolicySet* ps) {
  JDoc d;
  parse_json(json, len, NUM_FLOAT, &d);
  const JNode& root = d.at(d.root);
  std::vector<uint32_t> pols;
  if (root.t == J_ARR) {
    for (uint32_t c = root.first; c < root.first + root.count; c++) pols.push_back(c);
  } else if (root.t == J_MAP) {
    pols.push_back(d.root);
  } else {
    throw std::runtime_error("policies: expected a policy object or a list of policies");
  }
  ps->intern("");  // id 0: empty string
  Compiler C(*ps);
  std::map<std::pair<std::string, std::string>, uint32_t> var_keys;  // distinct (text, path) of VarStrs
  // keys always needed by match/ingest
  for (const char* k : {"metadata", "labels", "annotations", "name", "namespace", "kind", "apiVersion", "Namespace"})
    ps->intern(k);
  for (uint32_t pi = 0; pi < pols.size(); pi++) {
    uint32_t pn = pols[pi];
    int64_t md = d.get(pn, "metadata");
    ps->policy_names.push_back(md >= 0 ? jstr(d, d.get((uint32_t)md, "name")) : "");
    ps->policy_rule_first.push_back((uint32_t)ps->rules.size());
    int64_t spec = d.get(pn, "spec");
    int64_t rules = spec >= 0 ? d.get((uint32_t)spec, "rules") : -1;
    uint32_t nrules = 0;
    if (rules >= 0 && d.at((uint32_t)rules).t == J_ARR) {
      const JNode& rl = d.at((uint32_t)rules);
      for (uint32_t rn = rl.first; rn < rl.first + rl.count; rn++) {
        nrules++;
        RuleRec rr{};
        RuleHost rh;
        rh.policy = pi;
        rh.name = jstr(d, d.get(rn, "name"));
        compile_block(C, d, d.get(rn, "match"), true, rr, rh);
        compile_block(C, d, d.get(rn, "exclude"), false, rr, rh);
        int64_t val = d.get(rn, "validate");
        bool has_validate = false, patP = false, anyP = false, denyP = false, feP = false;
        int64_t pat = -1, ap = -1;
        std::string msg;
        if (val >= 0 && d.at((uint32_t)val).t == J_MAP) {
          uint32_t v = (uint32_t)val;
          msg = jstr(d, d.get(v, "message"));
          pat = d.get(v, "pattern");
          ap = d.get(v, "anyPattern");
          int64_t dn = d.get(v, "deny"), fe = d.get(v, "foreach");
          patP = pat >= 0 && d.at((uint32_t)pat).t != J_NULL;
          anyP = ap >= 0 && d.at((uint32_t)ap).t != J_NULL;
          denyP = dn >= 0 && d.at((uint32_t)dn).t != J_NULL;
          feP = fe >= 0 && d.at((uint32_t)fe).t != J_NULL;
          has_validate = !msg.empty() || patP || anyP || denyP || feP;
        }
        rh.message = msg;
        int64_t ctx = d.get(rn, "context"), pre = d.get(rn, "preconditions");
        bool ctxP = ctx >= 0 && d.at((uint32_t)ctx).t == J_ARR && d.at((uint32_t)ctx).count > 0;
        bool preP = pre >= 0 && d.at((uint32_t)pre).t != J_NULL;
        rr.route = 0;
        if (!has_validate) { rr.route = 2; rh.route_reason = "no validate"; }
        else if (feP) { rr.route = 1; rh.route_reason = "foreach"; }
        else if (ctxP) { rr.route = 1; rh.route_reason = "context"; }
        else if (preP) { rr.route = 1; rh.route_reason = "preconditions"; }
        else if (!patP && !anyP) {
          if (denyP) { rr.route = 1; rh.route_reason = "deny"; }
          else { rr.route = 2; rh.route_reason = "no pattern"; }  // validate() returns nil
        } else {
          PV doc = to_pv(d, patP ? (uint32_t)pat : (uint32_t)ap);
          const bool vars = doc_has_variable(doc);
          if (vars && !pattern_vars_in_scope(doc, "")) {
            rr.route = 1;
            rh.route_reason = "variables";
          } else if (doc_has_magic(doc) || has_magic(rh.name)) {
            rr.route = 1;
            rh.route_reason = "anchor-error phrase in pattern";
          } else {
            PV orig = doc;
            std::string err;
            if (!subst_tree(orig, doc, "", &err)) {
              rr.route = 3;
              rr.const_status = ST_ERROR;
              rh.const_message = "variable substitution failed: " + err;
            } else {
              const size_t vs0 = ps->vstrs.size();
              if (vars) {  // variables: resolved per resource (kvvars.cpp); other strings unescaped here
                collect_var_strings(*ps, doc, "", (uint32_t)ps->rules.size(), false, var_keys);
                ps->dyn_rules.push_back({(uint32_t)vs0, (uint32_t)(ps->vstrs.size() - vs0)});
                rr.dyn = (uint32_t)ps->dyn_rules.size();
              } else {
                unescape_vars(doc);
              }
              std::vector<PV> pats;
              bool ok = true;
              if (patP) {
                pats.push_back(doc);
              } else if (doc.t != J_ARR) {
                rr.route = 3;
                rr.const_status = ST_ERROR;
                const char* tn = doc.t == J_MAP ? "object" : doc.t == J_STR ? "string" : doc.t == J_BOOL ? "bool" : "number";
                rh.const_message = std::string("failed to deserialize anyPattern, expected type array: json: cannot unmarshal ") +
                                   tn + " into Go value of type []interface {}";
                ok = false;
              } else if (doc.a.empty()) {
                rr.route = 3;
                rr.const_status = ST_PASS;
                rh.const_message = msg;
                ok = false;
              } else {
                pats = doc.a;
                rh.anypattern = true;
                rr.n_alts = (uint32_t)pats.size();
              }
              if (ok) {
                if (!compile_pattern_program(C, pats, !patP, rr, rh)) rr.route = 1;
              }
            }
          }
        }
        ps->rules.push_back(rr);
        ps->rhost.push_back(rh);
      }
    }
    ps->policy_rule_count.push_back(nrules);
  }
  // Slot-addressed map layout: every non-keep-all trie node gets a byte-sorted
  // key list; key-lookup ops get the slot index (keep-all maps: key id + AUX_SCAN).
  for (auto& tn : ps->trie.nodes) {
    for (auto& kv : tn.kids) tn.slot_keys.push_back(kv.first);
    std::sort(tn.slot_keys.begin(), tn.slot_keys.end());
    for (uint32_t i = 0; i < tn.slot_keys.size(); i++) tn.slot.emplace(tn.slot_keys[i], i);
  }
  for (auto& f : ps->slot_fix) {
    Inst& in = ps->prog[std::get<0>(f)];
    const Trie::N& tn = ps->trie.nodes[std::get<1>(f)];
    if (tn.keep_all) {
      in.op |= AUX_SCAN << 16;
      continue;
    }
    auto it = tn.slot.find(std::get<2>(f));
    if (it == tn.slot.end()) throw std::runtime_error("compiler: key missing from projection trie: " + std::get<2>(f));
    in.a = it->second;
  }
}

std::string pattern_go_v(const PV& p) { return go_v(p); }

uint32_t compile_leaf_pred(PolicySet& tbl, const PV& value) {
  Compiler C(tbl);
  return C.pred(value);
}

}  // namespace kvh
