// ORACLE — test infrastructure only (see ovalue.hpp header).
// Restatement of the reference pattern matcher:
//   pkg/engine/validate/validate.go:29-194   MatchPattern / validateResourceElement /
//                                            validateMap / validateArray / validateArrayOfMaps
//   pkg/engine/validate/utils.go:10-60       hasNestedAnchors / getSortedNestedAnchorResource
//   pkg/engine/anchor/anchor.go:21-277       element handlers
//   pkg/engine/common/anchorKey.go:11-145    AnchorKey, anchor-error substring tests
//   pkg/engine/validate/pattern.go:25-318    scalar comparator
//   pkg/engine/operator/operator.go:33-67    operator parsing
//   pkg/engine/wildcards/wildcards.go:69-161 ExpandInMetadata
// Go map iteration order (random in the reference) is replaced by the
// canonical order documented in DESIGN.md §Canonical order:
//   anchor tier: condition, existence, equality, negation; each byte-lex by key
//   resource tier: [global anchors + keys with nested anchors] byte-lex, then plain keys byte-lex
//   wildcard label/annotation key: byte-lex smallest matching resource key
#include "matcher.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <vector>

namespace orc {

thread_local Chooser* g_choose = nullptr;

// ---------------------------------------------------------------- anchors
bool IsConditionAnchor(const std::string& s) {
  if (s.size() < 2) return false;
  return s[0] == '(' && s.back() == ')';
}
static bool prefixed_anchor(const std::string& s, const char* left) {
  if (s.size() < 3) return false;
  return s[0] == left[0] && s[1] == left[1] && s.back() == ')';
}
bool IsGlobalAnchor(const std::string& s) { return prefixed_anchor(s, "<("); }
bool IsNegationAnchor(const std::string& s) { return prefixed_anchor(s, "X("); }
bool IsAddingAnchor(const std::string& s) { return prefixed_anchor(s, "+("); }
bool IsEqualityAnchor(const std::string& s) { return prefixed_anchor(s, "=("); }
bool IsExistenceAnchor(const std::string& s) { return prefixed_anchor(s, "^("); }

std::string RemoveAnchor(const std::string& key, std::string* prefix) {
  if (IsConditionAnchor(key)) {
    if (prefix) *prefix = key.substr(0, 1);
    return key.substr(1, key.size() - 2);
  }
  if (IsExistenceAnchor(key) || IsAddingAnchor(key) || IsEqualityAnchor(key) || IsNegationAnchor(key) ||
      IsGlobalAnchor(key)) {
    if (prefix) *prefix = key.substr(0, 2);
    return key.substr(2, key.size() - 3);
  }
  if (prefix) *prefix = "";
  return key;
}

// Go path.Clean semantics for the Join in RemoveAnchorsFromPath
static std::string go_path_clean(const std::string& p) {
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
  if (out.empty()) return ".";
  return out;
}

static std::string go_path_join(const std::vector<std::string>& elems) {
  std::string joined;
  bool any = false;
  for (const auto& e : elems) {
    if (!any && e.empty()) continue;
    if (any) joined += "/";
    joined += e;
    any = true;
  }
  if (!any) return "";
  return go_path_clean(joined);
}

std::string RemoveAnchorsFromPath(const std::string& str) {
  std::vector<std::string> comps;
  size_t i = 0;
  while (true) {
    size_t j = str.find('/', i);
    if (j == std::string::npos) { comps.push_back(str.substr(i)); break; }
    comps.push_back(str.substr(i, j - i));
    i = j + 1;
  }
  if (!comps.empty() && comps[0].empty()) comps.erase(comps.begin());
  for (auto& c : comps) c = RemoveAnchor(c);
  std::string np = go_path_join(comps);
  if (!str.empty() && str[0] == '/') np = "/" + np;
  return np;
}

bool IsConditionalAnchorError(const std::string& msg) {
  return msg.find("conditional anchor mismatch") != std::string::npos;
}
bool IsGlobalAnchorError(const std::string& msg) { return msg.find("global anchor mismatch") != std::string::npos; }

void AnchorKey::CheckAnchorInResource(const Value& pattern, const Value& resource) {
  if (pattern.t != T::Map) return;
  for (const auto& e : pattern.m) {
    const std::string& key = e.key;
    if (IsConditionAnchor(key) || IsExistenceAnchor(key) || IsNegationAnchor(key)) {
      auto it = anchorMap.find(key);
      if (it == anchorMap.end()) anchorMap[key] = false;
      else if (it->second) continue;
      // doesAnchorsKeyHasValue: resource is a map at every call site
      std::string akey = RemoveAnchor(key);
      bool has = false;
      if (resource.t == T::Map) has = resource.has(akey);
      if (has) anchorMap[key] = true;
    }
  }
}

// ---------------------------------------------------------------- operators
std::string GetOperatorFromStringPattern(const std::string& pattern) {
  if (pattern.size() < 2) return "";
  if (pattern.compare(0, 2, ">=") == 0) return ">=";
  if (pattern.compare(0, 2, "<=") == 0) return "<=";
  if (pattern[0] == '>') return ">";
  if (pattern[0] == '<') return "<";
  if (pattern[0] == '!') return "!";
  // ^(\d+(\.\d+)?)([^-]*)!-(\d+(\.\d+)?)([^-]*)$  and  ^(\d+(\.\d+)?)([^-]*)-(\d+(\.\d+)?)([^-]*)$
  auto num_then_nodash = [&](size_t k, size_t* out) -> bool {
    size_t n = pattern.size();
    size_t s = k;
    while (k < n && pattern[k] >= '0' && pattern[k] <= '9') k++;
    if (k == s) return false;
    // (\.\d+)? is subsumed by [^-]* for matching purposes
    while (k < n && pattern[k] != '-') k++;
    *out = k;
    return true;
  };
  size_t k;
  if (num_then_nodash(0, &k)) {
    size_t n = pattern.size();
    // NotInRange: the [^-]* of the left side ends right before "!-": left run stops at '-'
    if (k < n && pattern[k] == '-' && k >= 1 && pattern[k - 1] == '!') {
      size_t r;
      if (num_then_nodash(k + 1, &r) && r == n) return "!-";
    }
    if (k < n && pattern[k] == '-') {
      size_t r;
      if (num_then_nodash(k + 1, &r) && r == n) return "-";
    }
  }
  return "";
}

void getNumberAndStringPartsFromPattern(const std::string& pattern, std::string* number, std::string* str) {
  // ^(\d*(\.\d+)?)(.*)   (leftmost-first; \d ASCII)
  size_t n = pattern.size(), k = 0;
  while (k < n && pattern[k] >= '0' && pattern[k] <= '9') k++;
  size_t numend = k;
  if (k < n && pattern[k] == '.') {
    size_t j = k + 1;
    while (j < n && pattern[j] >= '0' && pattern[j] <= '9') j++;
    if (j > k + 1) numend = j;
  }
  *number = pattern.substr(0, numend);
  *str = pattern.substr(numend);
}

// ---------------------------------------------------------------- comparator
static bool is_nilv(const Value* v) { return !v || v->t == T::Null; }

bool validateValueWithNilPattern(const Value* value) {
  if (is_nilv(value)) return true;
  switch (value->t) {
    case T::Float: return value->f == 0.0;
    case T::Int: return value->i == 0;
    case T::Str: return value->s.empty();
    case T::Bool: return !value->b;
    default: return false;
  }
}

static int64_t go_f2i(double p) {
  // amd64 CVTTSD2SI: out-of-range -> INT64_MIN
  if (!(p > -9223372036854775808.0 && p < 9223372036854775808.0)) return INT64_MIN;
  return (int64_t)p;
}

bool validateValueWithFloatPattern(const Value* value, double pattern) {
  if (is_nilv(value)) return false;
  switch (value->t) {
    case T::Int:
      if (pattern == std::trunc(pattern)) return go_f2i(pattern) == value->i;
      return false;
    case T::Float: return value->f == pattern;
    case T::Str: {
      double d;
      if (!go_parse_float(value->s, &d)) return false;
      return d == pattern;
    }
    default: return false;
  }
}

bool validateString(const Value* value, const std::string& pattern, const std::string& op) {
  if (op == "!" || op == "") {
    std::string sv;
    if (is_nilv(value)) return false;
    switch (value->t) {
      case T::Float: sv = go_format_E(value->f); break;
      case T::Int: sv = std::to_string(value->i); break;
      case T::Str: sv = value->s; break;
      case T::Bool: sv = value->b ? "true" : "false"; break;
      default: return false;
    }
    bool r = wildcard_match(pattern, sv);
    if (op == "!") return !r;
    return r;
  }
  return false;
}

// convertNumberToString: pkg/engine/validate/common.go:9-28
static bool convertNumberToString(const Value* value, std::string* out) {
  if (is_nilv(value)) { *out = "0"; return true; }
  switch (value->t) {
    case T::Str: *out = value->s; return true;
    case T::Float: *out = go_format_f6(value->f); return true;
    case T::Int: *out = std::to_string(value->i); return true;
    default: return false;
  }
}

bool validateNumberWithStr(const Value* value, const std::string& pattern, const std::string& op) {
  std::string tv;
  if (!convertNumberToString(value, &tv)) return false;
  Quantity pq;
  if (parse_quantity(pattern, &pq)) {
    Quantity vq;
    if (!parse_quantity(tv, &vq)) return false;
    int r = quantity_cmp(vq, pq);
    if (op == "") return r == 0;
    if (op == "!") return r != 0;
    if (op == ">") return r == 1;
    if (op == "<") return r == -1;
    if (op == ">=") return r >= 0;
    if (op == "<=") return r <= 0;
    return false;
  }
  return wildcard_match(pattern, tv);
}

static std::string trim_chars(const std::string& s, const char* set) {
  size_t b = 0, e = s.size();
  while (b < e && strchr(set, s[b])) b++;
  while (e > b && strchr(set, s[e - 1])) e--;
  return s.substr(b, e - b);
}

static std::vector<std::string> split(const std::string& s, const std::string& sep) {
  std::vector<std::string> out;
  size_t i = 0;
  while (true) {
    size_t j = s.find(sep, i);
    if (j == std::string::npos) { out.push_back(s.substr(i)); break; }
    out.push_back(s.substr(i, j - i));
    i = j + sep.size();
  }
  return out;
}

bool validateValueWithStringPattern(const Value* value, const std::string& pattern_in) {
  std::string pattern = pattern_in;
  std::string op = GetOperatorFromStringPattern(pattern);
  if (op == "-") {
    auto ep = split(pattern, "-");
    if (!validateValueWithStringPattern(value, ">=" + ep[0])) return false;
    pattern = "<=" + ep[1];
    op = "<=";
  }
  if (op == "!-") {
    auto ep = split(pattern, "!-");
    if (validateValueWithStringPattern(value, "<" + ep[0])) return true;
    pattern = ">" + ep[1];
    op = ">";
  }
  pattern = pattern.substr(op.size());
  pattern = trim_chars(pattern, " \t\n\v\f\r");  // strings.TrimSpace (ASCII subset)
  std::string number, str;
  getNumberAndStringPartsFromPattern(pattern, &number, &str);
  if (number.empty()) return validateString(value, str, op);
  return validateNumberWithStr(value, pattern, op);
}

static bool checkForAndConditionsAndValidate(const Value* value, const std::string& pattern) {
  for (auto& c : split(pattern, "&")) {
    std::string cond = trim_chars(c, " ");
    if (!validateValueWithStringPattern(value, cond)) return false;
  }
  return true;
}

static bool validateValueWithStringPatterns(const Value* value, const std::string& pattern) {
  for (auto& c : split(pattern, "|")) {
    std::string cond = trim_chars(c, " ");
    if (checkForAndConditionsAndValidate(value, cond)) return true;
  }
  return false;
}

bool ValidateValueWithPattern(const Value* value, const Value& pattern) {
  switch (pattern.t) {
    case T::Bool:
      if (is_nilv(value) || value->t != T::Bool) return false;
      return pattern.b == value->b;
    case T::Int: {
      // validateValueWithIntPattern (only reachable from Go-typed test inputs)
      int64_t p = pattern.i;
      if (is_nilv(value)) return false;
      switch (value->t) {
        case T::Int: return value->i == p;
        case T::Float:
          if (value->f == std::trunc(value->f)) return go_f2i(value->f) == p;
          return false;
        case T::Str: {
          int64_t v;
          if (!go_parse_int(value->s, &v)) return false;
          return v == p;
        }
        default: return false;
      }
    }
    case T::Float: return validateValueWithFloatPattern(value, pattern.f);
    case T::Str: return validateValueWithStringPatterns(value, pattern.s);
    case T::Null: return validateValueWithNilPattern(value);
    case T::Map: return !is_nilv(value) && value->t == T::Map;
    case T::Arr: return false;
  }
  return false;
}

// ---------------------------------------------------------------- wildcards
static bool hasWildcards(const std::string& s) {
  return s.find('*') != std::string::npos || s.find('?') != std::string::npos;
}

// getPatternValue: first key (canonical: byte-lex smallest) whose anchor-free form == tag
static const Value::Entry* getPatternValue(const std::string& tag, const Value& m) {
  const Value::Entry* best = nullptr;
  for (const auto& e : m.m) {
    if (RemoveAnchor(e.key) == tag) {
      if (!best || e.order < best->order) best = &e;
    }
  }
  return best;
}

// getValueAsStringMap: returns false if (key, nil); panics on wrong types
static bool getValueAsStringMap(const std::string& key, const Value* data, std::string* pkey,
                                std::vector<std::pair<std::string, std::string>>* out) {
  if (is_nilv(data)) return false;
  if (data->t != T::Map) throw GoPanic{"interface conversion: interface {} is not map[string]interface {}"};
  const Value::Entry* e = getPatternValue(key, *data);
  if (!e || is_nilv(e->val)) return false;
  if (e->val->t != T::Map) throw GoPanic{"interface conversion: labels value is not map[string]interface {}"};
  *pkey = e->key;
  out->clear();
  for (const auto& x : e->val->m) {
    if (is_nilv(x.val) || x.val->t != T::Str) throw GoPanic{"interface conversion: interface {} is not string"};
    out->push_back({x.key, x.val->s});
  }
  return true;
}

static void expandWildcardsInTag(const std::string& tag, Value& patternMetadata, const Value* resourceMetadata) {
  std::string patternKey, rk;
  std::vector<std::pair<std::string, std::string>> pdata, rdata;
  if (!getValueAsStringMap(tag, &patternMetadata, &patternKey, &pdata)) return;
  if (!getValueAsStringMap(tag, resourceMetadata, &rk, &rdata)) return;
  // canonical order of resource keys for expandWildcards: byte-lex
  std::sort(rdata.begin(), rdata.end());
  std::sort(pdata.begin(), pdata.end());
  Value results = Value::mk_map();
  for (const auto& kv : pdata) {
    const std::string& k = kv.first;
    if (hasWildcards(k)) {
      std::string prefix;
      std::string af = RemoveAnchor(k, &prefix);
      std::string matchK = af;
      if (g_choose) {  // enumerate mode: the first match in any map order
        std::vector<std::string> hits;
        for (const auto& r : rdata)
          if (wildcard_match(af, r.first)) hits.push_back(r.first);
        if (!hits.empty()) matchK = hits[g_choose->choose((int)hits.size())];
      } else {
        for (const auto& r : rdata) {
          if (wildcard_match(af, r.first)) { matchK = r.first; break; }
        }
      }
      if (!prefix.empty()) matchK = prefix + matchK + ")";
      results.set(matchK, Value::mk_str(kv.second), k);
    } else {
      results.set(k, Value::mk_str(kv.second), k);
    }
  }
  patternMetadata.set(patternKey, results, patternKey);
}

void ExpandInMetadata(Value& patternMap, const Value& resourceMap) {
  const Value::Entry* pe = getPatternValue("metadata", patternMap);
  if (!pe || is_nilv(pe->val)) return;
  const Value* resourceMetadata = resourceMap.get("metadata");
  if (is_nilv(resourceMetadata)) return;
  Value* metadata = patternMap.get_mut(pe->key);
  if (metadata->t != T::Map) throw GoPanic{"interface conversion: metadata is not map[string]interface {}"};
  expandWildcardsInTag("labels", *metadata, resourceMetadata);
  expandWildcardsInTag("annotations", *metadata, resourceMetadata);
}

// ---------------------------------------------------------------- walk
static PathErr validateResourceElement(const Value* res, Value& pat, const std::string& path, AnchorKey& ac);

static bool hasNestedAnchors(const Value& p) {
  if (p.t == T::Map) {
    for (const auto& e : p.m) {
      const std::string& k = e.key;
      if (IsConditionAnchor(k) || IsExistenceAnchor(k) || IsEqualityAnchor(k) || IsNegationAnchor(k) ||
          IsGlobalAnchor(k))
        return true;
    }
    for (const auto& e : p.m)
      if (hasNestedAnchors(*e.val)) return true;
    return false;
  }
  if (p.t == T::Arr) {
    for (const auto* x : p.a)
      if (hasNestedAnchors(*x)) return true;
  }
  return false;
}

static PathErr ok() { return PathErr{"", Err::none()}; }
static PathErr fail(const std::string& path, const std::string& msg) { return PathErr{path, Err::mk(msg)}; }

// pkg/engine/anchor/anchor.go:229-262
static PathErr validateExistenceListResource(const Value& resourceList, Value& patternMap, const std::string& path,
                                             AnchorKey& ac) {
  for (size_t i = 0; i < resourceList.a.size(); i++) {
    std::string cur = path + std::to_string(i) + "/";
    PathErr r = validateResourceElement(resourceList.a[i], patternMap, cur, ac);
    if (!r.err.set) return ok();
  }
  return fail(path, "existence anchor validation failed at path " + path);
}

static PathErr handle(const std::string& key, Value& pat, const std::string& path, const Value& resMap,
                      AnchorKey& ac) {
  if (IsConditionAnchor(key) || IsGlobalAnchor(key)) {
    bool global = !IsConditionAnchor(key);
    std::string ak = RemoveAnchor(key);
    std::string cur = path + ak + "/";
    const Value* v = resMap.get(ak);
    if (v) {
      PathErr r = validateResourceElement(v, pat, cur, ac);
      if (r.err.set) {
        std::string m = std::string(global ? "global anchor mismatch: " : "conditional anchor mismatch: ") + r.err.msg;
        return fail(r.path, m);
      }
      return ok();
    }
    return ok();
  }
  if (IsExistenceAnchor(key)) {
    std::string ak = RemoveAnchor(key);
    std::string cur = path + ak + "/";
    const Value* v = resMap.get(ak);
    if (v) {
      if (v->t == T::Arr) {
        if (pat.t != T::Arr)
          return fail(cur, "invalid pattern type " + go_type_name(&pat) +
                               ": Pattern has to be of list to compare against resource");
        PathErr last = ok();
        for (auto* pm : pat.a) {
          if (pm->t != T::Map)
            return fail(cur, "invalid pattern type " + go_type_name(&pat) +
                                 ": Pattern has to be of type map to compare against items in resource");
          last = validateExistenceListResource(*v, *pm, cur, ac);
          if (last.err.set) return last;
        }
        return last;
      }
      return fail(cur, "invalid resource type " + go_type_name(v) +
                           ": Existence ^ () anchor can be used only on list/array type resource");
    }
    return ok();
  }
  if (IsEqualityAnchor(key)) {
    std::string ak = RemoveAnchor(key);
    std::string cur = path + ak + "/";
    const Value* v = resMap.get(ak);
    if (v) {
      PathErr r = validateResourceElement(v, pat, cur, ac);
      if (r.err.set) return r;
    }
    return ok();
  }
  if (IsNegationAnchor(key)) {
    std::string ak = RemoveAnchor(key);
    std::string cur = path + ak + "/";
    if (resMap.has(ak)) return fail(cur, cur + "/" + ak + " is not allowed");
    return ok();
  }
  // DefaultHandler
  std::string cur = path + key + "/";
  const Value* v = resMap.get(key);
  if (pat.t == T::Str && pat.s == "*") {
    if (!is_nilv(v)) return ok();
    return fail(path, path + "/" + key + " not found");
  }
  PathErr r = validateResourceElement(v, pat, cur, ac);
  if (r.err.set) return r;
  return ok();
}

static int anchor_rank(const std::string& k) {
  if (IsConditionAnchor(k)) return 0;
  if (IsExistenceAnchor(k)) return 1;
  if (IsEqualityAnchor(k)) return 2;
  return 3;  // negation
}

static PathErr validateMap(const Value& resMap, Value& patternMap, const std::string& path, AnchorKey& ac) {
  ExpandInMetadata(patternMap, resMap);
  std::vector<Value::Entry*> anchors, resources;
  for (auto& e : patternMap.m) {
    const std::string& k = e.key;
    if (IsConditionAnchor(k) || IsExistenceAnchor(k) || IsEqualityAnchor(k) || IsNegationAnchor(k))
      anchors.push_back(&e);
    else
      resources.push_back(&e);
  }
  std::sort(anchors.begin(), anchors.end(), [](Value::Entry* a, Value::Entry* b) {
    int ra = anchor_rank(a->key), rb = anchor_rank(b->key);
    if (ra != rb) return ra < rb;
    return a->order < b->order;
  });
  auto front = [](Value::Entry* e) { return IsGlobalAnchor(e->key) || hasNestedAnchors(*e->val); };
  std::sort(resources.begin(), resources.end(), [&](Value::Entry* a, Value::Entry* b) {
    bool fa = front(a), fb = front(b);
    if (fa != fb) return fa;
    return a->order < b->order;
  });
  // Entries may not be reallocated during handling: handlers only mutate
  // nested maps (ExpandInMetadata replaces the metadata child's children).
  if (g_choose) {  // enumerate mode: any order within each Go map iteration
    auto run = [&](std::vector<Value::Entry*> left) -> PathErr {
      while (!left.empty()) {
        const int c = g_choose->choose((int)left.size());
        Value::Entry* e = left[c];
        left.erase(left.begin() + c);
        PathErr r = handle(e->key, *e->val, path, resMap, ac);
        if (r.err.set) return r;
      }
      return ok();
    };
    std::vector<Value::Entry*> fr, bk;
    for (auto* e : resources) (front(e) ? fr : bk).push_back(e);
    PathErr r = run(anchors);
    if (r.err.set) return r;
    r = run(fr);
    if (r.err.set) return r;
    return run(bk);
  }
  for (auto* e : anchors) {
    PathErr r = handle(e->key, *e->val, path, resMap, ac);
    if (r.err.set) return r;
  }
  for (auto* e : resources) {
    PathErr r = handle(e->key, *e->val, path, resMap, ac);
    if (r.err.set) return r;
  }
  return ok();
}

static bool is_scalar_pattern(const Value& p) {
  return p.t == T::Str || p.t == T::Float || p.t == T::Int || p.t == T::Bool || p.t == T::Null;
}

static PathErr validateArray(const Value& resArr, Value& patArr, const std::string& path, AnchorKey& ac) {
  if (patArr.a.empty()) return fail(path, "pattern Array empty");
  Value& p0 = *patArr.a[0];
  if (p0.t == T::Map) {
    for (size_t i = 0; i < resArr.a.size(); i++) {
      std::string cur = path + std::to_string(i) + "/";
      PathErr r = validateResourceElement(resArr.a[i], p0, cur, ac);
      if (r.err.set) {
        if (IsConditionalAnchorError(r.err.msg)) continue;
        return r;
      }
    }
    return ok();
  }
  if (is_scalar_pattern(p0)) {
    PathErr r = validateResourceElement(&resArr, p0, path, ac);
    if (r.err.set) return r;
    return ok();
  }
  if (resArr.a.size() >= patArr.a.size()) {
    for (size_t i = 0; i < patArr.a.size(); i++) {
      std::string cur = path + std::to_string(i) + "/";
      PathErr r = validateResourceElement(resArr.a[i], *patArr.a[i], cur, ac);
      if (r.err.set) {
        if (IsConditionalAnchorError(r.err.msg)) continue;
        return r;
      }
    }
    return ok();
  }
  return fail("", "validate Array failed, array length mismatch, resource Array len is " +
                      std::to_string(resArr.a.size()) + " and pattern Array len is " +
                      std::to_string(patArr.a.size()));
}

static PathErr validateResourceElement(const Value* res, Value& pat, const std::string& path, AnchorKey& ac) {
  if (pat.t == T::Map) {
    if (is_nilv(res) || res->t != T::Map)
      return fail(path, "pattern and resource have different structures. Path: " + path + ". Expected " +
                            go_type_name(&pat) + ", found " + go_type_name(res));
    ac.CheckAnchorInResource(pat, *res);
    return validateMap(*res, pat, path, ac);
  }
  if (pat.t == T::Arr) {
    if (is_nilv(res) || res->t != T::Arr)
      return fail(path, "validation rule Failed at path " + path +
                            ", resource does not satisfy the expected overlay pattern");
    return validateArray(*res, pat, path, ac);
  }
  // scalar pattern
  if (!is_nilv(res) && res->t == T::Arr) {
    for (const auto* e : res->a) {
      if (!ValidateValueWithPattern(e, pat))
        return fail(path, "resource value '" + go_format_v(res) + "' does not match '" + go_format_v(&pat) +
                              "' at path " + path);
    }
    return ok();
  }
  if (!ValidateValueWithPattern(res, pat))
    return fail(path, "resource value '" + go_format_v(res) + "' does not match '" + go_format_v(&pat) +
                          "' at path " + path);
  return ok();
}

PatternError MatchPattern(const Value* resource, Value& pattern) {
  AnchorKey ac;
  PathErr r = validateResourceElement(resource, pattern, "/", ac);
  PatternError pe;
  if (r.err.set) {
    pe.set = true;
    pe.msg = r.err.msg;
    if (IsConditionalAnchorError(r.err.msg) || IsGlobalAnchorError(r.err.msg)) {
      pe.path = "";
      pe.skip = true;
      return pe;
    }
    if (ac.IsAnchorError()) {
      pe.path = "";
      return pe;
    }
    pe.path = r.path;
  }
  return pe;
}

}  // namespace orc

#include "engine_api.hpp"

namespace orc {
bool ValidateElementEntry(int entry, const Value& resource, Value& pattern, std::string* path, std::string* msg) {
  AnchorKey ac;
  PathErr r;
  if (entry == 2) {
    if (resource.t != T::Map || pattern.t != T::Map) throw std::runtime_error("validateMap needs maps");
    r = validateMap(resource, pattern, "/", ac);
  } else {
    r = validateResourceElement(&resource, pattern, "/", ac);
  }
  *path = r.path;
  *msg = r.err.msg;
  return r.err.set;
}
}  // namespace orc
