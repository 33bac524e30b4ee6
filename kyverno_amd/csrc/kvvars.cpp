// validate.pattern variables on the device: `{{request.object<path>}}` and
// `{{@}}` in pattern / anyPattern strings.
//
// The reference substitutes the whole pattern document per (rule, resource) before matching
// (pkg/engine/validation.go:181-189,549-571 -> variables.SubstituteAll, vars.go:172-179:
// references, then substituteVariablesIfAny, vars.go:319-398, over the traversal of
// jsonutils/traverse.go:58-130). Here:
//  * compile (kvcompile.cpp): every string of the pattern holding variables becomes a VarStr
//    (traversal order, canonical key order); a leaf predicate on one becomes OP_VLEAF (a
//    "dynamic leaf"). Rules whose variables are not all request.object paths / @, or that have
//    variables in keys, stay CPU-routed;
//  * ingest: each resource's JSON resolves every distinct VarStr once into an outcome (the
//    substituted string, a typed scalar, the substitution error, or "outside the device scope")
//    interned per batch;
//  * per batch (build_dyn): distinct outcomes are compiled into a batch predicate table (pred id
//    = outcome id); per (dynamic leaf, resource) the outcome id; per (rule, resource) the status
//    the substitution decides before matching (ERROR "variable substitution failed: ...", or CPU
//    for a value outside the scope: a map / array replacing a leaf, a nested variable).
// The device evaluates a dynamic leaf with the generic predicate evaluator on that table.
#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "kvinternal.hpp"

namespace kvh {

using namespace kv;

namespace {

// RegexVariables.FindAllString: ^\{\{[^{}]*\}\}|[^\\]\{\{[^{}]*\}\} (leftmost-first, non-overlapping)
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
      const size_t e = close(0);
      if (e != std::string::npos) { out.push_back(s.substr(0, e)); i = e; continue; }
    }
    if (s[i] != '\\' && i + 1 < s.size()) {
      // [^\\] is one rune
      const unsigned char c = (unsigned char)s[i];
      const size_t w = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 1;
      if (i + w < s.size()) {
        const size_t e = close(i + w);
        if (e != std::string::npos) { out.push_back(s.substr(i, e - i)); i = e; continue; }
      }
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

// regexVariableInit = ^\{\{[^{}]*\}\}
bool var_initial(const std::string& v) {
  if (v.compare(0, 2, "{{") != 0) return false;
  size_t k = 2;
  while (k < v.size() && v[k] != '{' && v[k] != '}') k++;
  return v.compare(k, 2, "}}") == 0;
}

std::string replace_all(std::string s, const std::string& from, const std::string& to) {
  if (from.empty()) return s;
  size_t p = 0;
  while ((p = s.find(from, p)) != std::string::npos) {
    s.replace(p, from.size(), to);
    p += to.size();
  }
  return s;
}

std::string replace_first(const std::string& s, const std::string& from, const std::string& to) {
  const size_t p = s.find(from);
  if (p == std::string::npos) return s;
  return s.substr(0, p) + to + s.substr(p + from.size());
}

// replaceBracesAndTrimSpaces (vars.go:443-448); strings.TrimSpace trims ASCII + Unicode spaces,
// ASCII suffices for the variable grammar accepted here
std::string var_name(const std::string& v) {
  std::string x = replace_all(replace_all(v, "{{", ""), "}}", "");
  const size_t b = x.find_first_not_of(" \t\n\r\v\f"), e = x.find_last_not_of(" \t\n\r\v\f");
  return b == std::string::npos ? std::string() : x.substr(b, e - b + 1);
}

// getJMESPath (vars.go:416-422) of a traversal path; false where the reference's tokens[3:]
// panics (fewer than 3 tokens)
bool jmes_path_of(const std::string& raw, std::string* out) {
  std::vector<std::string> tok;
  size_t i = 0;
  while (true) {
    const size_t j = raw.find('/', i);
    tok.push_back(raw.substr(i, j == std::string::npos ? std::string::npos : j - i));
    if (j == std::string::npos) break;
    i = j + 1;
  }
  if (tok.size() < 3) return false;
  std::string path;
  for (size_t k = 3; k < tok.size(); k++) path += (k > 3 ? "." : "") + tok[k];
  std::string b;  // regexPathDigit `\.?([\d])\.?` -> "[$1]."
  for (size_t k = 0; k < path.size();) {
    size_t d = k;
    if (path[d] == '.' && d + 1 < path.size() && isdigit((unsigned char)path[d + 1])) d++;
    if (isdigit((unsigned char)path[d])) {
      size_t e = d + 1;
      if (e < path.size() && path[e] == '.') e++;
      b += '[';
      b += path[d];
      b += "].";
      k = e;
      continue;
    }
    b += path[k++];
  }
  const size_t s0 = b.find_first_not_of('.'), s1 = b.find_last_not_of('.');
  *out = s0 == std::string::npos ? std::string() : b.substr(s0, s1 - s0 + 1);
  return true;
}

// one step of a request.object query: .field / ."quoted" / [n]
struct QStep {
  bool index;
  std::string key;
  long idx;
};

// The JMESPath subset on the device: request.object followed by field / quoted-field / index
// steps (pkg/engine/context/evaluate.go:15-50 with kyverno's go-jmespath fork: a missing map key
// is NotFoundError, a field of a non-map and an index of a non-array are null).
bool parse_query(const std::string& q, std::vector<QStep>* steps) {
  static const std::string root = "request.object";
  if (q.compare(0, root.size(), root) != 0) return false;
  size_t i = root.size();
  steps->clear();
  while (i < q.size()) {
    if (q[i] == '[') {
      const size_t e = q.find(']', i);
      if (e == std::string::npos || e == i + 1) return false;
      const std::string num = q.substr(i + 1, e - i - 1);
      for (size_t k = 0; k < num.size(); k++)
        if (!(isdigit((unsigned char)num[k]) || (k == 0 && num[k] == '-' && num.size() > 1))) return false;
      steps->push_back({true, "", atol(num.c_str())});
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
      const size_t s = i;
      while (i < q.size() && (isalnum((unsigned char)q[i]) || q[i] == '_')) i++;
      if (i == s || isdigit((unsigned char)q[s])) return false;
      key = q.substr(s, i - s);
    }
    steps->push_back({false, key, 0});
  }
  return true;
}

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

// 0: found (*node, -1 for null), 1: unknown key (*missing)
int query_doc(const std::vector<QStep>& steps, const JDoc& d, int64_t* node, std::string* missing) {
  int64_t cur = d.root;
  for (const QStep& s : steps) {
    if (cur < 0) continue;  // null: every further step is null
    const JNode& n = d.at((uint32_t)cur);
    if (s.index) {
      if (n.t != J_ARR) { cur = -1; continue; }
      long i = s.idx;
      if (i < 0) i += (long)n.count;
      cur = i >= 0 && i < (long)n.count ? (int64_t)(n.first + i) : -1;
    } else {
      if (n.t != J_MAP) { cur = -1; continue; }
      // encoding/json keeps the last of duplicate keys
      int64_t hit = -1;
      for (uint32_t c = n.first; c < n.first + n.count; c++)
        if (d.key(d.at(c)) == s.key) hit = c;
      if (hit < 0) {
        *missing = s.key;
        return 1;
      }
      cur = hit;
    }
  }
  if (cur >= 0 && d.at((uint32_t)cur).t == J_NULL) cur = -1;
  *node = cur;
  return 0;
}

// encoding/json Marshal of a string (HTMLEscape on)
void json_str(std::string& o, std::string_view s) {
  o += '"';
  for (size_t i = 0; i < s.size(); i++) {
    const unsigned char c = (unsigned char)s[i];
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
  o += '"';
}

// json.Marshal of a context value (numbers float64, map keys sorted)
void json_value(std::string& o, const JDoc& d, int64_t node) {
  if (node < 0) { o += "null"; return; }
  const JNode& n = d.at((uint32_t)node);
  switch (n.t) {
    case J_NULL: o += "null"; break;
    case J_BOOL: o += n.b ? "true" : "false"; break;
    case J_INT: o += go_json_float((double)n.i); break;
    case J_FLOAT: o += go_json_float(n.f); break;
    case J_STR: json_str(o, d.sval(n)); break;
    case J_ARR:
      o += '[';
      for (uint32_t c = n.first; c < n.first + n.count; c++) {
        if (c > n.first) o += ',';
        json_value(o, d, c);
      }
      o += ']';
      break;
    case J_MAP: {
      std::vector<uint32_t> kids;
      for (uint32_t c = n.first; c < n.first + n.count; c++) kids.push_back(c);
      std::stable_sort(kids.begin(), kids.end(), [&](uint32_t a, uint32_t b) { return d.key(d.at(a)) < d.key(d.at(b)); });
      // duplicate keys: the last one is the value encoding/json kept
      o += '{';
      bool first = true;
      for (size_t k = 0; k < kids.size(); k++) {
        if (k + 1 < kids.size() && d.key(d.at(kids[k])) == d.key(d.at(kids[k + 1]))) continue;
        if (!first) o += ',';
        first = false;
        json_str(o, d.key(d.at(kids[k])));
        o += ':';
        json_value(o, d, kids[k]);
      }
      o += '}';
      break;
    }
  }
}

}  // namespace

bool var_string(const std::string& s) { return !find_vars(s).empty(); }

bool var_string_in_scope(const std::string& s, const std::string& path) {
  std::vector<QStep> steps;
  for (std::string v : find_vars(s)) {
    if (!var_initial(v)) {
      if ((unsigned char)v[0] >= 0x80) return false;
      v = v.substr(1);
    }
    std::string q;
    if (!var_query(var_name(v), path, &q) || !parse_query(q, &steps)) return false;
  }
  return true;
}

std::string unescape_var_string(const std::string& s) {
  std::string v = s;
  for (const auto& e : find_escaped_vars(v)) v = replace_all(v, e, e.substr(1));
  return v;
}

// substituteVariablesIfAny (vars.go:319-398) on one pattern string of the traversal path `path`,
// with request.object = resource `d`. Outcome encoding (interned per batch): "S" + string,
// "F" + 8 raw bytes of a float64, "B0" / "B1", "N" (null), "E" + the error text, "C" (outside
// the device scope), "M" (a map or array: a structural pattern, outside the scope).
std::string resolve_var_string(const std::string& tmpl, const std::string& path, const JDoc& d) {
  std::string value = tmpl;
  std::vector<QStep> steps;
  auto vars = find_vars(value);
  while (!vars.empty()) {
    const std::string original = value;
    for (std::string v : vars) {
      const bool initial = var_initial(v);
      const std::string old = v;
      if (!initial) {
        // v = v[1:] (a byte): a multi-byte rune before "{{" leaves part of it in the variable,
        // which the reference then fails to parse ("failed to resolve ..."): outside the scope
        if ((unsigned char)old[0] >= 0x80) return "C";
        v = v.substr(1);
      }
      std::string q;
      if (!var_query(var_name(v), path, &q) || !parse_query(q, &steps)) return "C";
      int64_t node = -1;
      std::string missing;
      if (query_doc(steps, d, &node, &missing) == 1) return "EUnknown key \"" + missing + "\" in path";
      if (original == v) {  // the whole string: the value itself
        if (node < 0) return "N";
        const JNode& n = d.at((uint32_t)node);
        switch (n.t) {
          case J_BOOL: return n.b ? "B1" : "B0";
          case J_INT:
          case J_FLOAT: {
            const double f = n.t == J_INT ? (double)n.i : n.f;
            std::string o = "F";
            o.append((const char*)&f, 8);
            return o;
          }
          case J_STR: return "S" + std::string(d.sval(n));
          default: return "M";
        }
      }
      const std::string prefix = initial ? "" : old.substr(0, 1);
      std::string sub;
      if (node >= 0 && d.at((uint32_t)node).t == J_STR) sub = std::string(d.sval(d.at((uint32_t)node)));
      else json_value(sub, d, node);
      value = replace_first(original, prefix + v, prefix + sub);
    }
    vars = find_vars(value);
  }
  return "S" + unescape_var_string(value);
}

PV outcome_value(const std::string& o) {
  PV p;
  switch (o.empty() ? 'C' : o[0]) {
    case 'S': p.t = J_STR; p.s = o.substr(1); break;
    case 'F': p.t = J_FLOAT; memcpy(&p.f, o.data() + 1, 8); break;
    case 'B': p.t = J_BOOL; p.b = o[1] == '1'; break;
    case 'N': p.t = J_NULL; break;
    default: p.t = J_ARR; break;  // not a leaf value (error / outside the scope): never evaluated
  }
  return p;
}

void build_dyn(const PolicySet& ps, const Batch& b, DynHost* out) {
  DynHost& h = *out;
  h = DynHost();
  const uint64_t n = b.res.size();
  const size_t K = ps.vkeys.size();
  if (!K) return;
  const std::vector<std::string>& tab = b.vout_tab;
  // batch predicate table: one predicate per distinct outcome (pred id == outcome id)
  for (size_t o = 0; o < tab.size(); o++) {
    const char t = tab[o].empty() ? 'C' : tab[o][0];
    const uint32_t id = (t == 'S' || t == 'F' || t == 'B' || t == 'N') ? compile_leaf_pred(h.tbl, outcome_value(tab[o]))
                                                                     : compile_leaf_pred(h.tbl, PV{});
    if (id != h.tbl.preds.size() - 1 || id != o) {
      // equal outcomes are interned once, so every compile appends; keep ids aligned regardless
      h.tbl.preds.push_back(h.tbl.preds[id]);
    }
  }
  if (h.tbl.preds.size() != tab.size()) throw std::runtime_error("build_dyn: predicate table misaligned");
  h.tbl.strs.append(16, '\0');
  const size_t L = ps.dleaf_vstr.size(), R = ps.dyn_rules.size();
  h.dleaf.assign(L * n, 0);
  h.dyn_st.assign(R * n, 0);
  h.dyn_msg.assign(R * n, 0);
  for (uint64_t r = 0; r < n; r++) {
    const uint32_t* out_r = b.vout.data() + r * K;
    for (size_t l = 0; l < L; l++) h.dleaf[l * n + r] = out_r[ps.vstrs[ps.dleaf_vstr[l]].key];
    for (size_t q = 0; q < R; q++) {
      const auto [first, count] = ps.dyn_rules[q];
      uint8_t st = 0;
      uint32_t msg = 0;
      bool structural = false;
      for (uint32_t v = first; v < first + count && !st; v++) {
        const uint32_t o = out_r[ps.vstrs[v].key];
        const char t = tab[o].empty() ? 'C' : tab[o][0];
        if (t == 'E') { st = ST_ERROR; msg = o; }
        else if (t == 'C') st = ST_CPU;
        else if (t == 'M') structural = true;  // the traversal goes on into the value
        else if (ps.vstrs[v].want_string && t != 'S') structural = true;
      }
      if (!st && structural) st = ST_CPU;
      h.dyn_st[q * n + r] = st;
      h.dyn_msg[q * n + r] = msg;
    }
  }
}

}  // namespace kvh
