// ORACLE — test infrastructure only (see ovalue.hpp header).
// Restatement of the engine driver around the matcher:
//   pkg/engine/validation.go:26-547   Validate / validateResource / validate /
//                                     validatePatterns / message builders
//   pkg/engine/utils.go:37-369        checkKind / checkName / checkNameSpace /
//                                     checkAnnotations / checkSelector /
//                                     doesResourceMatchConditionBlock / matchSubjects /
//                                     MatchesResourceDescription
//   pkg/engine/wildcards/wildcards.go:13-63  ReplaceInSelector
//   k8s.io/apimachinery v0.21.4 LabelSelectorAsSelector / Requirement.Matches
//   pkg/kyverno/common/common.go:703-766 ProcessValidateEngineResponse (CLI counts)
// Rules that need the reference CPU engine (context, preconditions, deny,
// foreach, {{ }} variables in pattern/anyPattern) are reported with status
// "cpu" — the same deterministic routing decision the GPU compiler makes.
#include <atomic>
#include <mutex>
#include <algorithm>
#include <cstring>
#include <map>
#include <set>
#include <stdexcept>
#include <thread>
#include <vector>

#include "matcher.hpp"

namespace orc {

// ---------------------------------------------------------------- policy model
struct LabelSelector {
  bool present = false;
  std::vector<std::pair<std::string, std::string>> matchLabels;
  struct Expr { std::string key, op; std::vector<std::string> values; };
  std::vector<Expr> matchExpressions;
};

struct Subject { std::string kind, name, ns; };

struct UserInfo {
  bool rolesP = false, clusterRolesP = false, subjectsP = false;  // non-nil slices
  std::vector<std::string> roles, clusterRoles;
  std::vector<Subject> subjects;
  bool empty() const { return !rolesP && !clusterRolesP && !subjectsP; }
};

struct ResourceDescription {
  bool kindsP = false, namesP = false, namespacesP = false, annotationsP = false;
  std::vector<std::string> kinds, names, namespaces;
  std::string name;
  std::vector<std::pair<std::string, std::string>> annotations;
  LabelSelector selector, namespaceSelector;
  bool empty() const {
    return !kindsP && !namesP && !namespacesP && !annotationsP && name.empty() && !selector.present &&
           !namespaceSelector.present;
  }
};

struct ResourceFilter {
  UserInfo userInfo;
  ResourceDescription rd;
};

struct MatchBlock {
  bool anyP = false, allP = false;
  std::vector<ResourceFilter> any, all;
  UserInfo userInfo;
  ResourceDescription rd;
};

struct Rule {
  std::string name;
  MatchBlock match, exclude;
  bool hasValidate = false;
  std::string message;
  bool patternP = false, anyPatternP = false, denyP = false, foreachP = false;
  Value pattern, anyPattern;
  bool contextNonEmpty = false, preconditionsP = false;
};

struct Policy {
  std::string name, ns, validationFailureAction;
  std::vector<Rule> rules;
};

struct RequestInfo {
  std::vector<std::string> roles, clusterRoles, groups;
  std::string username;
  bool empty() const { return roles.empty() && clusterRoles.empty() && groups.empty() && username.empty(); }
};

static std::string str_of(const Value* v) { return (v && v->t == T::Str) ? v->s : ""; }

static bool str_list(const Value* v, std::vector<std::string>* out) {
  if (!v || v->t == T::Null) return false;
  if (v->t != T::Arr) throw std::runtime_error("policy: expected list");
  for (auto* x : v->a) out->push_back(str_of(x));
  return true;
}

static bool str_map(const Value* v, std::vector<std::pair<std::string, std::string>>* out) {
  if (!v || v->t == T::Null) return false;
  if (v->t != T::Map) throw std::runtime_error("policy: expected map");
  for (auto& e : v->m) out->push_back({e.key, str_of(e.val)});
  return true;
}

static LabelSelector parse_selector(const Value* v) {
  LabelSelector s;
  if (!v || v->t == T::Null) return s;
  s.present = true;
  str_map(v->get("matchLabels"), &s.matchLabels);
  const Value* me = v->get("matchExpressions");
  if (me && me->t == T::Arr) {
    for (auto* x : me->a) {
      LabelSelector::Expr e;
      e.key = str_of(x->get("key"));
      e.op = str_of(x->get("operator"));
      str_list(x->get("values"), &e.values);
      s.matchExpressions.push_back(e);
    }
  }
  return s;
}

static UserInfo parse_userinfo(const Value* v) {
  UserInfo u;
  if (!v || v->t != T::Map) return u;
  u.rolesP = str_list(v->get("roles"), &u.roles);
  u.clusterRolesP = str_list(v->get("clusterRoles"), &u.clusterRoles);
  const Value* s = v->get("subjects");
  if (s && s->t == T::Arr) {
    u.subjectsP = true;
    for (auto* x : s->a) u.subjects.push_back({str_of(x->get("kind")), str_of(x->get("name")), str_of(x->get("namespace"))});
  }
  return u;
}

static ResourceDescription parse_rd(const Value* v) {
  ResourceDescription r;
  if (!v || v->t != T::Map) return r;
  r.kindsP = str_list(v->get("kinds"), &r.kinds);
  r.name = str_of(v->get("name"));
  r.namesP = str_list(v->get("names"), &r.names);
  r.namespacesP = str_list(v->get("namespaces"), &r.namespaces);
  r.annotationsP = str_map(v->get("annotations"), &r.annotations);
  r.selector = parse_selector(v->get("selector"));
  r.namespaceSelector = parse_selector(v->get("namespaceSelector"));
  return r;
}

static MatchBlock parse_match(const Value* v) {
  MatchBlock m;
  if (!v || v->t != T::Map) return m;
  const Value* any = v->get("any");
  if (any && any->t == T::Arr) {
    m.anyP = true;
    for (auto* x : any->a) m.any.push_back({parse_userinfo(x), parse_rd(x->get("resources"))});
  }
  const Value* all = v->get("all");
  if (all && all->t == T::Arr) {
    m.allP = true;
    for (auto* x : all->a) m.all.push_back({parse_userinfo(x), parse_rd(x->get("resources"))});
  }
  m.userInfo = parse_userinfo(v);
  m.rd = parse_rd(v->get("resources"));
  return m;
}

Policy parse_policy(const Value& pv) {
  Policy p;
  const Value* md = pv.get("metadata");
  if (md) { p.name = str_of(md->get("name")); p.ns = str_of(md->get("namespace")); }
  const Value* spec = pv.get("spec");
  if (!spec) return p;
  p.validationFailureAction = str_of(spec->get("validationFailureAction"));
  const Value* rules = spec->get("rules");
  if (!rules || rules->t != T::Arr) return p;
  for (auto* rv : rules->a) {
    Rule r;
    r.name = str_of(rv->get("name"));
    r.match = parse_match(rv->get("match"));
    r.exclude = parse_match(rv->get("exclude"));
    const Value* ctx = rv->get("context");
    r.contextNonEmpty = ctx && ctx->t == T::Arr && !ctx->a.empty();
    const Value* pre = rv->get("preconditions");
    r.preconditionsP = pre && pre->t != T::Null;
    const Value* val = rv->get("validate");
    if (val && val->t == T::Map) {
      r.message = str_of(val->get("message"));
      const Value* pat = val->get("pattern");
      if (pat && pat->t != T::Null) { r.patternP = true; r.pattern = *pat; }
      const Value* ap = val->get("anyPattern");
      if (ap && ap->t != T::Null) { r.anyPatternP = true; r.anyPattern = *ap; }
      const Value* deny = val->get("deny");
      r.denyP = deny && deny->t != T::Null;
      const Value* fe = val->get("foreach");
      r.foreachP = fe && fe->t != T::Null;
      r.hasValidate = !r.message.empty() || r.patternP || r.anyPatternP || r.denyP || r.foreachP;
    }
    p.rules.push_back(r);
  }
  return p;
}

// ---------------------------------------------------------------- resource accessors
struct Resource {
  const Value* obj;
  std::string kind, apiVersion, name, ns;
  std::vector<std::pair<std::string, std::string>> labels, annotations;
  std::string group, version;
};

static void nested_string_map(const Value* v, std::vector<std::pair<std::string, std::string>>* out) {
  out->clear();
  if (!v || v->t != T::Map) return;
  for (auto& e : v->m) {
    if (!e.val || e.val->t != T::Str) { out->clear(); return; }  // NestedStringMap error -> nil
    out->push_back({e.key, e.val->s});
  }
}

Resource make_resource(const Value& obj) {
  Resource r;
  r.obj = &obj;
  r.kind = str_of(obj.get("kind"));
  r.apiVersion = str_of(obj.get("apiVersion"));
  const Value* md = obj.get("metadata");
  if (md && md->t == T::Map) {
    r.name = str_of(md->get("name"));
    r.ns = str_of(md->get("namespace"));
    nested_string_map(md->get("labels"), &r.labels);
    nested_string_map(md->get("annotations"), &r.annotations);
  }
  // schema.ParseGroupVersion
  const std::string& gv = r.apiVersion;
  if (!gv.empty() && gv != "/") {
    size_t c = std::count(gv.begin(), gv.end(), '/');
    if (c == 0) { r.version = gv; }
    else if (c == 1) { size_t i = gv.find('/'); r.group = gv.substr(0, i); r.version = gv.substr(i + 1); }
  }
  return r;
}

// ---------------------------------------------------------------- label selectors
static bool re_qname(const std::string& n) {
  // ^([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]$
  if (n.empty()) return false;
  auto alnum = [](char c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
  if (!alnum(n[0]) || !alnum(n.back())) return false;
  for (char c : n)
    if (!(alnum(c) || c == '-' || c == '_' || c == '.')) return false;
  return true;
}

static bool re_dns1123_subdomain(const std::string& s) {
  if (s.empty() || s.size() > 253) return false;
  // labels separated by '.', each ^[a-z0-9]([-a-z0-9]*[a-z0-9])?$
  size_t i = 0;
  while (true) {
    size_t j = s.find('.', i);
    std::string lab = s.substr(i, j == std::string::npos ? std::string::npos : j - i);
    if (lab.empty()) return false;
    auto ok = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
    if (!ok(lab[0]) || !ok(lab.back())) return false;
    for (char c : lab)
      if (!(ok(c) || c == '-')) return false;
    if (j == std::string::npos) break;
    i = j + 1;
  }
  return true;
}

static bool valid_label_key(const std::string& k) {
  std::vector<std::string> parts;
  size_t i = 0;
  while (true) {
    size_t j = k.find('/', i);
    if (j == std::string::npos) { parts.push_back(k.substr(i)); break; }
    parts.push_back(k.substr(i, j - i));
    i = j + 1;
  }
  std::string name;
  if (parts.size() == 1) name = parts[0];
  else if (parts.size() == 2) {
    if (parts[0].empty() || !re_dns1123_subdomain(parts[0])) return false;
    name = parts[1];
  } else return false;
  if (name.empty() || name.size() > 63) return false;
  return re_qname(name);
}

static bool valid_label_value(const std::string& v) {
  if (v.size() > 63) return false;
  if (v.empty()) return true;
  return re_qname(v);
}

static bool has_wildcards(const std::string& s) {
  return s.find('*') != std::string::npos || s.find('?') != std::string::npos;
}

static std::string replace_wc(std::string s) {
  for (auto& c : s)
    if (c == '*' || c == '?') c = '0';
  return s;
}

// checkSelector: returns 1 match, 0 no match, -1 parse error
static int check_selector(const LabelSelector& sel, const std::vector<std::pair<std::string, std::string>>& labels_in) {
  std::vector<std::pair<std::string, std::string>> labels = labels_in;
  std::sort(labels.begin(), labels.end());
  // ReplaceInSelector (wildcards.go:13-63), canonical order
  std::vector<std::pair<std::string, std::string>> ml = sel.matchLabels;
  std::sort(ml.begin(), ml.end());
  std::map<std::string, std::string> result;
  for (auto& kv : ml) {
    const std::string &k = kv.first, &v = kv.second;
    if (has_wildcards(k) || has_wildcards(v)) {
      std::string mk = replace_wc(k), mv = replace_wc(v);
      for (auto& r : labels) {
        if (wildcard_match(k, r.first) && wildcard_match(v, r.second)) { mk = r.first; mv = r.second; break; }
      }
      result[mk] = mv;
    } else {
      result[k] = v;
    }
  }
  if (result.size() + sel.matchExpressions.size() == 0) return 1;  // Everything
  auto has = [&](const std::string& k, std::string* val) {
    for (auto& r : labels)
      if (r.first == k) { *val = r.second; return true; }
    return false;
  };
  // requirement validation happens while building the selector
  for (auto& kv : result) {
    if (!valid_label_key(kv.first) || !valid_label_value(kv.second)) return -1;
  }
  for (auto& e : sel.matchExpressions) {
    if (e.op != "In" && e.op != "NotIn" && e.op != "Exists" && e.op != "DoesNotExist") return -1;
    if (!valid_label_key(e.key)) return -1;
    if ((e.op == "In" || e.op == "NotIn") && e.values.empty()) return -1;
    if ((e.op == "Exists" || e.op == "DoesNotExist") && !e.values.empty()) return -1;
    for (auto& v : e.values)
      if (!valid_label_value(v)) return -1;
  }
  for (auto& kv : result) {
    std::string val;
    if (!has(kv.first, &val) || val != kv.second) return 0;
  }
  for (auto& e : sel.matchExpressions) {
    std::string val;
    bool h = has(e.key, &val);
    bool inset = h && std::find(e.values.begin(), e.values.end(), val) != e.values.end();
    if (e.op == "In" && !inset) return 0;
    if (e.op == "NotIn" && inset) return 0;
    if (e.op == "Exists" && !h) return 0;
    if (e.op == "DoesNotExist" && h) return 0;
  }
  return 1;
}

// ---------------------------------------------------------------- match/exclude
static std::string go_title(const std::string& s) {
  std::string out = s;
  bool prev_sep = true;
  for (auto& c : out) {
    bool letter = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
    bool alnum = letter || (c >= '0' && c <= '9') || c == '_' || (unsigned char)c >= 0x80;
    if (prev_sep && c >= 'a' && c <= 'z') c = (char)(c - 'a' + 'A');
    prev_sep = !alnum;
  }
  return out;
}

static std::vector<std::string> split_slash(const std::string& s) {
  std::vector<std::string> out;
  size_t i = 0;
  while (true) {
    size_t j = s.find('/', i);
    if (j == std::string::npos) { out.push_back(s.substr(i)); break; }
    out.push_back(s.substr(i, j - i));
    i = j + 1;
  }
  return out;
}

static bool check_kind(const std::vector<std::string>& kinds, const Resource& r) {
  for (auto& k : kinds) {
    auto sp = split_slash(k);
    if (sp.size() == 1) {
      if (r.kind == go_title(k) || k == "*") return true;
    } else if (sp.size() == 2) {
      if (r.kind == go_title(sp[1]) && r.version == sp[0]) return true;
    } else {
      if (r.group == sp[0] && r.kind == go_title(sp[2]) && (r.version == sp[1] || r.version == "*")) return true;
    }
  }
  return false;
}

static bool slice_contains(const std::vector<std::string>& slice, const std::vector<std::string>& values) {
  for (auto& v : values)
    if (std::find(slice.begin(), slice.end(), v) != slice.end()) return true;
  return false;
}

static bool match_subjects(std::vector<Subject> subjects, const RequestInfo& ai, const std::vector<std::string>& dyn) {
  const std::string sa = "system:serviceaccount:";
  std::vector<std::string> ug = ai.groups;
  ug.push_back(ai.username);
  for (auto& e : dyn) subjects.push_back({"Group", e, ""});
  for (auto& s : subjects) {
    if (s.kind == "ServiceAccount") {
      if (ai.username.size() <= sa.size()) continue;
      if (ai.username.substr(sa.size()) == s.ns + ":" + s.name) return true;
    } else if (s.kind == "User" || s.kind == "Group") {
      if (std::find(ug.begin(), ug.end(), s.name) != ug.end()) return true;
    }
  }
  return false;
}

// returns number of errors (0 == block matched)
static int does_match_block(const ResourceDescription& cb, const UserInfo& ui, const RequestInfo& ai, const Resource& r,
                            const std::vector<std::string>& dyn,
                            const std::vector<std::pair<std::string, std::string>>& nsLabels) {
  int errs = 0;
  if (!cb.kinds.empty() && !check_kind(cb.kinds, r)) errs++;
  if (!cb.name.empty() && !wildcard_match(cb.name, r.name)) errs++;
  if (!cb.names.empty()) {
    bool none = true;
    for (auto& n : cb.names)
      if (wildcard_match(n, r.name)) { none = false; break; }
    if (none) errs++;
  }
  if (!cb.namespaces.empty()) {
    std::string rns = r.kind == "Namespace" ? r.name : r.ns;
    bool any = false;
    for (auto& n : cb.namespaces)
      if (wildcard_match(n, rns)) { any = true; break; }
    if (!any) errs++;
  }
  if (!cb.annotations.empty()) {
    bool all = true;
    for (auto& kv : cb.annotations) {
      bool m = false;
      for (auto& ra : r.annotations)
        if (wildcard_match(kv.first, ra.first) && wildcard_match(kv.second, ra.second)) { m = true; break; }
      if (!m) { all = false; break; }
    }
    if (!all) errs++;
  }
  if (cb.selector.present) {
    if (check_selector(cb.selector, r.labels) != 1) errs++;
  }
  if (cb.namespaceSelector.present && r.kind != "Namespace" && !r.kind.empty()) {
    if (check_selector(cb.namespaceSelector, nsLabels) != 1) errs++;
  }
  std::vector<std::string> keys = ai.groups;
  keys.push_back(ai.username);
  int uerrs = 0, checked = 0;
  if (!ui.roles.empty() && !slice_contains(keys, dyn)) {
    checked++;
    if (!slice_contains(ui.roles, ai.roles)) uerrs++;
    else return errs;
  }
  if (!ui.clusterRoles.empty() && !slice_contains(keys, dyn)) {
    checked++;
    if (!slice_contains(ui.clusterRoles, ai.clusterRoles)) uerrs++;
    else return errs;
  }
  if (!ui.subjects.empty()) {
    checked++;
    if (!match_subjects(ui.subjects, ai, dyn)) uerrs++;
    else return errs;
  }
  if (checked != uerrs) return errs;
  return errs + uerrs;
}

static int match_helper(const ResourceFilter& f, const RequestInfo& ai, const Resource& r,
                        const std::vector<std::string>& dyn, const std::vector<std::pair<std::string, std::string>>& ns) {
  UserInfo ui = f.userInfo;
  if (ai.empty()) ui = UserInfo();
  if (!f.rd.empty() || !ui.empty()) return does_match_block(f.rd, ui, ai, r, dyn, ns);
  return 1;  // "match cannot be empty"
}

static int exclude_helper(const ResourceFilter& f, const RequestInfo& ai, const Resource& r,
                          const std::vector<std::string>& dyn, const std::vector<std::pair<std::string, std::string>>& ns) {
  if (!f.rd.empty() || !f.userInfo.empty()) {
    if (does_match_block(f.rd, f.userInfo, ai, r, dyn, ns) == 0) return 1;
  }
  return 0;
}

bool MatchesResourceDescription(const Resource& r, const Rule& rule, const RequestInfo& ai, const std::vector<std::string>& dyn,
                                const std::vector<std::pair<std::string, std::string>>& ns) {
  int reasons = 0;
  if (!rule.match.any.empty()) {
    bool one = false;
    for (auto& f : rule.match.any)
      if (match_helper(f, ai, r, dyn, ns) == 0) { one = true; break; }
    if (!one) reasons++;
  } else if (!rule.match.all.empty()) {
    for (auto& f : rule.match.all) reasons += match_helper(f, ai, r, dyn, ns);
  } else {
    ResourceFilter f{rule.match.userInfo, rule.match.rd};
    reasons += match_helper(f, ai, r, dyn, ns);
  }
  if (!rule.exclude.any.empty()) {
    for (auto& f : rule.exclude.any) reasons += exclude_helper(f, ai, r, dyn, ns);
  } else if (!rule.exclude.all.empty()) {
    bool byAll = true;
    for (auto& f : rule.exclude.all)
      if (exclude_helper(f, ai, r, dyn, ns) == 0) { byAll = false; break; }
    if (byAll) reasons++;
  } else {
    ResourceFilter f{rule.exclude.userInfo, rule.exclude.rd};
    reasons += exclude_helper(f, ai, r, dyn, ns);
  }
  return reasons == 0;
}

// ---------------------------------------------------------------- validate driver
enum Status { PASS = 0, FAIL = 1, WARN = 2, ERROR = 3, SKIP = 4, NOMATCH = 5, CPU = 6, PANIC = 7 };

struct RuleResult {
  std::string name;
  int status = NOMATCH;  // NOMATCH: absent from the EngineResponse
  std::string message;
  std::string path;      // failing path (FAIL) — "" otherwise
  std::string reason;    // CPU route reason
  bool message_panics = false;  // the reference panics building the message (validation.go:519-524)
};

static std::string with_dot(const std::string& m) {
  if (!m.empty() && m.back() == '.') return m;
  return m + ".";
}

// message substitution (buildErrorMessage, validation.go:518-524): SubstituteAll of the message
// with request.object = the resource. *panics is set where the reference panics.
static std::string build_error_message(const Rule& rule, const std::string& err, const std::string& path,
                                       const Value& resource, bool* panics) {
  if (rule.message.empty()) {
    if (!path.empty()) return "validation error: rule " + rule.name + " failed at path " + path;
    return "validation error: rule " + rule.name + " execution error: " + err;
  }
  std::string sub;
  if (!SubstituteMessage(rule.message, resource, &sub)) {
    *panics = true;
    return "";
  }
  std::string msg = with_dot(sub);
  if (!path.empty()) return "validation error: " + msg + " Rule " + rule.name + " failed at path " + path;
  return "validation error: " + msg + " Rule " + rule.name + " execution error: " + err;
}

static void validate_patterns(const Rule& rule, Value pattern, Value anyPattern, const Value& resource, RuleResult* out) {
  if (rule.patternP) {
    PatternError pe = MatchPattern(&resource, pattern);
    if (pe.set) {
      if (pe.skip) { out->status = SKIP; out->message = pe.msg; return; }
      if (pe.path.empty()) { out->status = ERROR; out->message = build_error_message(rule, pe.msg, "", resource, &out->message_panics); return; }
      out->status = FAIL;
      out->path = pe.path;
      out->message = build_error_message(rule, pe.msg, pe.path, resource, &out->message_panics);
      return;
    }
    out->status = PASS;
    out->message = "validation rule '" + rule.name + "' passed.";
    return;
  }
  if (rule.anyPatternP) {
    if (anyPattern.t != T::Arr) {
      std::string tn = anyPattern.t == T::Map ? "object" : anyPattern.t == T::Str ? "string"
                       : anyPattern.t == T::Bool ? "bool" : "number";
      out->status = ERROR;
      out->message = "failed to deserialize anyPattern, expected type array: json: cannot unmarshal " + tn +
                     " into Go value of type []interface {}";
      return;
    }
    std::vector<std::string> errs;
    for (size_t idx = 0; idx < anyPattern.a.size(); idx++) {
      PatternError pe = MatchPattern(&resource, *anyPattern.a[idx]);
      if (!pe.set) {
        out->status = PASS;
        out->message = "validation rule '" + rule.name + "' anyPattern[" + std::to_string(idx) + "] passed.";
        return;
      }
      if (pe.path.empty())
        errs.push_back("Rule " + rule.name + "[" + std::to_string(idx) + "] failed: " + pe.msg + ".");
      else
        errs.push_back("Rule " + rule.name + "[" + std::to_string(idx) + "] failed at path " + pe.path + ".");
    }
    if (!errs.empty()) {
      std::string joined;
      for (size_t k = 0; k < errs.size(); k++) { if (k) joined += " "; joined += errs[k]; }
      out->status = FAIL;
      if (rule.message.empty()) out->message = "validation error: " + joined;
      else if (rule.message.back() == '.') out->message = "validation error: " + rule.message + " " + joined;
      else out->message = "validation error: " + rule.message + ". " + joined;
      return;
    }
  }
  out->status = PASS;
  out->message = rule.message;
}

// CPU-route reason for a validate rule, or "" if the GPU path evaluates it.
std::string route_reason(const Rule& rule) {
  if (rule.foreachP) return "foreach";
  if (rule.contextNonEmpty) return "context";
  if (rule.preconditionsP) return "preconditions";
  // variables: on the device when every one is request.object<path> or @ and none is in a key
  if (rule.patternP) { if (DocHasVariable(rule.pattern) && !PatternVarsInScope(rule.pattern)) return "variables"; return ""; }
  if (rule.anyPatternP) {
    if (DocHasVariable(rule.anyPattern) && !PatternVarsInScope(rule.anyPattern)) return "variables";
    return "";
  }
  if (rule.denyP) return "deny";
  return "";
}

RuleResult evaluate_rule(const Rule& rule, const Value& resource) {
  RuleResult rr;
  rr.name = rule.name;
  std::string reason = route_reason(rule);
  if (!reason.empty()) { rr.status = CPU; rr.reason = reason; return rr; }
  if (!rule.patternP && !rule.anyPatternP) { rr.status = NOMATCH; return rr; }  // validate() returns nil
  Value pattern, anyPattern;
  std::string err;
  // SubstituteAll (validation.go:549-571, vars.go:172-179): references, then variables
  Value& doc = rule.patternP ? pattern : anyPattern;
  doc = rule.patternP ? rule.pattern : rule.anyPattern;
  const bool vars = DocHasVariable(doc);
  if (!SubstituteReferences(doc, &err, !vars)) {
    rr.status = ERROR;
    rr.message = "variable substitution failed: " + err;
    return rr;
  }
  if (vars) {
    bool structural = false;
    int r = SubstitutePatternVars(doc, resource, &err, &structural);
    if (r == 1) {
      rr.status = ERROR;
      rr.message = "variable substitution failed: " + err;
      return rr;
    }
    if (r == 2 || structural) {  // a value from the resource leaves the device scope (structural / nested variable)
      rr.status = CPU;
      rr.reason = "variables";
      return rr;
    }
  }
  try {
    validate_patterns(rule, pattern, anyPattern, resource, &rr);
  } catch (const GoPanic& p) {
    rr.status = PANIC;
    rr.message = "panic: " + p.what;
  }
  return rr;
}

struct EngineCtx {
  RequestInfo ai;
  std::vector<std::string> excludeGroupRole;
  std::map<std::string, std::vector<std::pair<std::string, std::string>>> nsLabels;
};

std::vector<RuleResult> validate_policy(const Policy& pol, const Value& resource, const EngineCtx& cx) {
  std::vector<RuleResult> out;
  Resource r = make_resource(resource);
  std::vector<std::pair<std::string, std::string>> ns;
  auto it = cx.nsLabels.find(r.ns);
  if (it != cx.nsLabels.end()) ns = it->second;
  for (const auto& rule : pol.rules) {
    RuleResult rr;
    rr.name = rule.name;
    if (!rule.hasValidate) { rr.status = NOMATCH; out.push_back(rr); continue; }
    if (!MatchesResourceDescription(r, rule, cx.ai, cx.excludeGroupRole, ns)) { rr.status = NOMATCH; out.push_back(rr); continue; }
    out.push_back(evaluate_rule(rule, resource));
  }
  return out;
}

}  // namespace orc

// ---------------------------------------------------------------- serialized entry points
#include <chrono>

#include "engine_api.hpp"

namespace orc {

static std::string js(const std::string& s) { return to_json(Value::mk_str(s)); }

static EngineCtx parse_ctx(const Value& cv) {
  EngineCtx cx;
  const Value* a = cv.get("admission");
  if (a && a->t == T::Map) {
    str_list(a->get("roles"), &cx.ai.roles);
    str_list(a->get("clusterRoles"), &cx.ai.clusterRoles);
    str_list(a->get("groups"), &cx.ai.groups);
    cx.ai.username = str_of(a->get("username"));
  }
  str_list(cv.get("excludeGroupRole"), &cx.excludeGroupRole);
  const Value* nl = cv.get("namespaceLabels");
  if (nl && nl->t == T::Map) {
    for (auto& e : nl->m) {
      std::vector<std::pair<std::string, std::string>> v;
      str_map(e.val, &v);
      cx.nsLabels[e.key] = v;
    }
  }
  return cx;
}

static const char* status_name(int s) {
  static const char* n[] = {"pass", "fail", "warn", "error", "skip", "nomatch", "cpu", "panic"};
  return n[s];
}

std::string ValidateToJSON(const Value& policy, const Value& resource, const Value& ctx) {
  Policy pol = parse_policy(policy);
  EngineCtx cx = parse_ctx(ctx);
  std::vector<RuleResult> rs = validate_policy(pol, resource, cx);
  std::string out = "{\"policy\":" + js(pol.name) + ",\"rules\":[";
  for (size_t k = 0; k < rs.size(); k++) {
    const auto& r = rs[k];
    if (k) out += ",";
    out += "{\"name\":" + js(r.name) + ",\"status\":" + js(status_name(r.status)) + ",\"message\":" + js(r.message) +
           ",\"path\":" + js(r.path) + ",\"reason\":" + js(r.reason) +
           ",\"message_panics\":" + (r.message_panics ? "true" : "false") + "}";
  }
  out += "]}";
  return out;
}

// Enumerate mode: every outcome (status, failing path) the reference can produce for each
// rule of `policy` on `resource` over the Go map iteration orders (matcher.hpp Chooser):
// depth-first over choice sequences, at most `cap` evaluations per rule.
std::string EnumerateToJSON(const Value& policy, const Value& resource, const Value& ctx, int cap) {
  Policy pol = parse_policy(policy);
  EngineCtx cx = parse_ctx(ctx);
  Resource r = make_resource(resource);
  std::vector<std::pair<std::string, std::string>> ns;
  auto it = cx.nsLabels.find(r.ns);
  if (it != cx.nsLabels.end()) ns = it->second;
  std::string out = "{\"rules\":[";
  for (size_t k = 0; k < pol.rules.size(); k++) {
    const Rule& rule = pol.rules[k];
    if (k) out += ",";
    out += "{\"name\":" + js(rule.name);
    if (!rule.hasValidate || !MatchesResourceDescription(r, rule, cx.ai, cx.excludeGroupRole, ns)) {
      out += ",\"outcomes\":[[\"nomatch\",\"\"]],\"runs\":1,\"truncated\":false}";
      continue;
    }
    std::set<std::pair<int, std::string>> seen;
    std::vector<std::vector<int>> stack{{}};
    int runs = 0;
    while (!stack.empty() && runs < cap) {
      Chooser ch;
      ch.prefix = stack.back();
      stack.pop_back();
      g_choose = &ch;
      RuleResult rr;
      try {
        rr = evaluate_rule(rule, resource);
      } catch (...) {
        g_choose = nullptr;
        throw;
      }
      g_choose = nullptr;
      runs++;
      seen.insert({rr.status, rr.status == FAIL ? rr.path : std::string()});
      for (size_t d = ch.prefix.size(); d < ch.taken.size(); d++)
        for (int c = 1; c < ch.arity[d]; c++) {
          std::vector<int> p(ch.taken.begin(), ch.taken.begin() + d);
          p.push_back(c);
          stack.push_back(std::move(p));
        }
    }
    out += ",\"outcomes\":[";
    bool first = true;
    for (const auto& o : seen) {
      if (!first) out += ",";
      first = false;
      out += "[" + js(status_name(o.first)) + "," + js(o.second) + "]";
    }
    out += "],\"runs\":" + std::to_string(runs) + ",\"truncated\":" + (stack.empty() ? "false" : "true") + "}";
  }
  out += "]}";
  return out;
}

double BatchValidate(const char* policies_json, const char* resources_json, const char* ctx_json, int nthreads,
                     unsigned char* status_out, long long* n_rules_out, long long* n_res_out) {
  Value pl = parse_json(policies_json, NumMode::Float);
  Value rl = parse_json(resources_json, NumMode::Unstructured);
  Value cv = parse_json(ctx_json && *ctx_json ? ctx_json : "{}", NumMode::Float);
  if (pl.t != T::Arr || rl.t != T::Arr) throw std::runtime_error("batch: expected lists");
  std::vector<Policy> pols;
  size_t nrules = 0;
  for (auto* p : pl.a) { pols.push_back(parse_policy(*p)); nrules += pols.back().rules.size(); }
  EngineCtx cx = parse_ctx(cv);
  size_t nres = rl.a.size();
  *n_rules_out = (long long)nrules;
  *n_res_out = (long long)nres;
  if (!status_out) return 0.0;
  if (nthreads < 1) nthreads = 1;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int w = 0; w < nthreads; w++) {
    th.emplace_back([&, w]() {
      for (size_t r = w; r < nres; r += nthreads) {
        size_t rule_base = 0;
        for (const auto& pol : pols) {
          std::vector<RuleResult> rs = validate_policy(pol, *rl.a[r], cx);
          for (size_t k = 0; k < rs.size(); k++) status_out[(rule_base + k) * nres + r] = (unsigned char)rs[k].status;
          rule_base += pol.rules.size();
        }
      }
    });
  }
  for (auto& t : th) t.join();
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(t1 - t0).count();
}

// NDJSON batch for the large parity tests: one resource per line, each thread
// parses and evaluates its own contiguous range of lines (bounded memory, parse in
// parallel). status_out [n_rules][n_res] must hold CountRules() x (lines) bytes.
size_t CountRules(const char* policies_json) {
  Value pl = parse_json(policies_json, NumMode::Float);
  if (pl.t != T::Arr) throw std::runtime_error("batch: expected a list");
  size_t n = 0;
  for (auto* p : pl.a) n += parse_policy(*p).rules.size();
  return n;
}

double BatchValidateNdjson(const char* policies_json, const char* ndjson, size_t len, const char* ctx_json,
                           int nthreads, unsigned char* status_out, size_t n_res, int preparse) {
  Value pl = parse_json(policies_json, NumMode::Float);
  Value cv = parse_json(ctx_json && *ctx_json ? ctx_json : "{}", NumMode::Float);
  if (pl.t != T::Arr) throw std::runtime_error("batch: expected a list");
  std::vector<Policy> pols;
  for (auto* p : pl.a) pols.push_back(parse_policy(*p));
  EngineCtx cx = parse_ctx(cv);
  std::vector<std::pair<size_t, size_t>> lines;
  for (size_t i = 0; i < len;) {
    size_t e = i;
    while (e < len && ndjson[e] != '\n') e++;
    if (e > i) lines.push_back({i, e - i});
    i = e + 1;
  }
  if (lines.size() != n_res) throw std::runtime_error("batch: line count differs from n_res");
  if (nthreads < 1) nthreads = 1;
  std::vector<std::thread> th;
  std::vector<std::string> errs(nthreads);
  const size_t per = (n_res + nthreads - 1) / nthreads;
  auto eval = [&](size_t r, const Value& v) {
    size_t rule_base = 0;
    for (const auto& pol : pols) {
      std::vector<RuleResult> rs = validate_policy(pol, v, cx);
      for (size_t k = 0; k < rs.size(); k++) status_out[(rule_base + k) * n_res + r] = (unsigned char)rs[k].status;
      rule_base += pol.rules.size();
    }
  };
  auto parse_line = [&](size_t r) {
    return parse_json(std::string(ndjson + lines[r].first, lines[r].second), NumMode::Unstructured);
  };
  // preparse: every thread parses its range first; the timed region is the evaluation
  // alone, from the moment all threads have parsed until the last one finishes
  std::vector<std::vector<Value>> docs(preparse ? nthreads : 0);
  std::atomic<int> parsed{0};
  std::atomic<bool> go{!preparse};
  std::chrono::steady_clock::time_point t0;
  std::mutex mu;
  for (int w = 0; w < nthreads; w++) {
    th.emplace_back([&, w]() {
      const size_t b = std::min(n_res, w * per), e = std::min(n_res, (w + 1) * per);
      try {
        if (preparse) {
          for (size_t r = b; r < e; r++) docs[w].push_back(parse_line(r));
          if (++parsed == nthreads) {
            std::lock_guard<std::mutex> g(mu);
            t0 = std::chrono::steady_clock::now();
            go = true;
          }
          while (!go) std::this_thread::yield();
          for (size_t r = b; r < e; r++) eval(r, docs[w][r - b]);
        } else {
          for (size_t r = b; r < e; r++) eval(r, parse_line(r));
        }
      } catch (const std::exception& ex) {
        errs[w] = ex.what();
        if (preparse && ++parsed == nthreads) go = true;
      }
    });
  }
  if (!preparse) t0 = std::chrono::steady_clock::now();
  for (auto& t : th) t.join();
  const auto t1 = std::chrono::steady_clock::now();
  for (auto& e : errs)
    if (!e.empty()) throw std::runtime_error(e);
  std::lock_guard<std::mutex> g(mu);
  return std::chrono::duration<double>(t1 - t0).count();
}

}  // namespace orc
