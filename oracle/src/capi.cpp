// ORACLE — test infrastructure only (see ovalue.hpp header).
// C entry points for tests/ (ctypes) and bench.py's cpu_baseline leg.
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <thread>
#include <vector>

#include "matcher.hpp"

#include "engine_api.hpp"

using namespace orc;

namespace {

char* dup(const std::string& s) {
  char* p = (char*)malloc(s.size() + 1);
  memcpy(p, s.data(), s.size());
  p[s.size()] = 0;
  return p;
}

std::string jstr(const std::string& s) {
  Value v = Value::mk_str(s);
  return to_json(v);
}

NumMode mode_of(int m) { return m ? NumMode::Unstructured : NumMode::Float; }

thread_local std::string g_err;

}  // namespace

extern "C" {

void orc_free(char* p) { free(p); }
const char* orc_last_error() { return g_err.c_str(); }

int orc_glob(const char* pattern, const char* name) { return wildcard_match(pattern, name) ? 1 : 0; }

// returns 1 and writes canonical text, or 0 if not a quantity
int orc_quantity(const char* s, char** out) {
  Quantity q;
  if (!parse_quantity(s, &q)) return 0;
  *out = dup(quantity_debug(q));
  return 1;
}

int orc_quantity_cmp(const char* a, const char* b) {
  Quantity qa, qb;
  if (!parse_quantity(a, &qa) || !parse_quantity(b, &qb)) return -2;
  return quantity_cmp(qa, qb);
}

char* orc_operator(const char* pattern) { return dup(GetOperatorFromStringPattern(pattern)); }

// anchor/common predicates by name; returns -1 for an unknown name
int orc_anchor_pred(const char* fn, const char* key) {
  std::string f = fn, k = key;
  if (f == "IsConditionAnchor") return IsConditionAnchor(k);
  if (f == "IsGlobalAnchor") return IsGlobalAnchor(k);
  if (f == "IsNegationAnchor") return IsNegationAnchor(k);
  if (f == "IsAddingAnchor") return IsAddingAnchor(k);
  if (f == "IsEqualityAnchor") return IsEqualityAnchor(k);
  if (f == "IsExistenceAnchor") return IsExistenceAnchor(k);
  return -1;
}

char* orc_remove_anchors_from_path(const char* p) { return dup(RemoveAnchorsFromPath(p)); }

char* orc_number_parts(const char* pattern) {
  std::string n, s;
  getNumberAndStringPartsFromPattern(pattern, &n, &s);
  return dup("[" + jstr(n) + "," + jstr(s) + "]");
}

char* orc_format(const char* what, double v) {
  std::string w = what;
  if (w == "E") return dup(go_format_E(v));
  if (w == "f") return dup(go_format_f6(v));
  return dup(go_format_g(v));
}

// kind: 0 ValidateValueWithPattern, 1 validateValueWithStringPattern (pattern is a
// raw string), 2 validateNumberWithStr (op), 3 validateString (op),
// 4 validateValueWithNilPattern, 5 validateValueWithFloatPattern
int orc_compare(int kind, const char* value_json, int value_mode, const char* pattern_json, int pattern_mode,
                const char* op) {
  try {
    Value v = parse_json(value_json, mode_of(value_mode));
    switch (kind) {
      case 0: {
        Value p = parse_json(pattern_json, mode_of(pattern_mode));
        return ValidateValueWithPattern(&v, p) ? 1 : 0;
      }
      case 1: return validateValueWithStringPattern(&v, pattern_json) ? 1 : 0;
      case 2: return validateNumberWithStr(&v, pattern_json, op) ? 1 : 0;
      case 3: return validateString(&v, pattern_json, op) ? 1 : 0;
      case 4: return validateValueWithNilPattern(&v) ? 1 : 0;
      case 5: {
        Value p = parse_json(pattern_json, NumMode::Float);
        return validateValueWithFloatPattern(&v, p.f) ? 1 : 0;
      }
    }
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
  return -1;
}

// ExpandInMetadata (pkg/engine/wildcards/wildcards.go:69-161) of a pattern / resource pair:
// the pattern after replaceWildcardsInMapKeys, as JSON ({"panic": msg} when the reference panics)
char* orc_expand_in_metadata(const char* pattern_json, const char* resource_json) {
  try {
    Value p = parse_json(pattern_json, NumMode::Float);
    Value r = parse_json(resource_json, NumMode::Unstructured);
    try {
      ExpandInMetadata(p, r);
    } catch (const GoPanic& e) {
      return dup("{\"panic\":" + jstr(e.what) + "}");
    }
    return dup(to_json(p));
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
}

// MatchPattern(resource, pattern) -> {"set":b,"msg":s,"path":s,"skip":b}
// entry: 0 MatchPattern, 1 validateResourceElement("/"), 2 validateMap("/")
char* orc_match_pattern(int entry, const char* resource_json, int res_mode, const char* pattern_json, int do_subst) {
  try {
    Value r = parse_json(resource_json, mode_of(res_mode));
    Value p = parse_json(pattern_json, NumMode::Float);
    if (do_subst) {
      std::string err;
      if (!SubstituteReferences(p, &err)) return dup("{\"subst_error\":" + jstr(err) + "}");
    }
    std::string out;
    try {
      if (entry == 0) {
        PatternError pe = MatchPattern(&r, p);
        out = std::string("{\"set\":") + (pe.set ? "true" : "false") + ",\"msg\":" + jstr(pe.msg) +
              ",\"path\":" + jstr(pe.path) + ",\"skip\":" + (pe.skip ? "true" : "false") + "}";
      } else {
        std::string path, msg;
        bool set = ValidateElementEntry(entry, r, p, &path, &msg);
        out = std::string("{\"set\":") + (set ? "true" : "false") + ",\"msg\":" + jstr(msg) + ",\"path\":" +
              jstr(path) + "}";
      }
    } catch (const GoPanic& gp) {
      out = "{\"panic\":" + jstr(gp.what) + "}";
    }
    return dup(out);
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
}

// Substitute $() references in a pattern document; returns the JSON or error
char* orc_substitute(const char* pattern_json) {
  try {
    Value p = parse_json(pattern_json, NumMode::Float);
    std::string err;
    if (!SubstituteReferences(p, &err)) return dup("{\"error\":" + jstr(err) + "}");
    return dup("{\"doc\":" + to_json(p) + "}");
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
}

// SubstituteAll of a validate.pattern document with request.object = resource (references,
// then variables): {"doc": ...} | {"error": ...} | {"scope": false} (outside the device scope)
char* orc_substitute_vars(const char* pattern_json, const char* resource_json) {
  try {
    Value p = parse_json(pattern_json, NumMode::Float);
    Value rv = parse_json(resource_json, NumMode::Unstructured);
    std::string err;
    if (!PatternVarsInScope(p)) return dup("{\"scope\":false}");
    if (!SubstituteReferences(p, &err, !DocHasVariable(p))) return dup("{\"error\":" + jstr(err) + "}");
    int r = SubstitutePatternVars(p, rv, &err);
    if (r == 1) return dup("{\"error\":" + jstr(err) + "}");
    if (r == 2) return dup("{\"scope\":false}");
    return dup("{\"doc\":" + to_json(p) + "}");
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
}

// buildErrorMessage's SubstituteAll of a validate message against request.object = resource
// (validation.go:518-524). Returns nullptr where the reference panics.
char* orc_substitute_message(const char* msg, const char* resource_json) {
  try {
    Value rv = parse_json(resource_json, NumMode::Unstructured);
    std::string out;
    if (!SubstituteMessage(msg, rv, &out)) {
      g_err = "reference panics";
      return nullptr;
    }
    return dup(out);
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
}

// engine.Validate for one policy x one resource.
// ctx_json: {"admission": {"roles":[],"clusterRoles":[],"groups":[],"username":""},
//            "excludeGroupRole": [], "namespaceLabels": {"ns": {"k":"v"}}}
char* orc_validate(const char* policy_json, const char* resource_json, const char* ctx_json) {
  try {
    Value pv = parse_json(policy_json, NumMode::Float);
    Value rv = parse_json(resource_json, NumMode::Unstructured);
    Value cv = parse_json(ctx_json && *ctx_json ? ctx_json : "{}", NumMode::Float);
    return dup(ValidateToJSON(pv, rv, cv));
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
}

// Enumerate mode: {"rules": [{"name", "outcomes": [[status, path]...], "runs", "truncated"}]}
char* orc_enumerate(const char* policy_json, const char* resource_json, const char* ctx_json, int cap) {
  try {
    Value pv = parse_json(policy_json, NumMode::Float);
    Value rv = parse_json(resource_json, NumMode::Unstructured);
    Value cv = parse_json(ctx_json && *ctx_json ? ctx_json : "{}", NumMode::Float);
    return dup(EnumerateToJSON(pv, rv, cv, cap));
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
}

// Batch: policies_json = JSON list of policies; resources = JSON list of
// resources. Writes status[n_res * n_rules_total] (rule-major:
// status[rule * n_res + res]) and returns elapsed evaluation seconds
// (parse excluded). nthreads workers split the resources.
double orc_validate_batch(const char* policies_json, const char* resources_json, const char* ctx_json, int nthreads,
                          unsigned char* status_out, long long* n_rules_out, long long* n_res_out) {
  try {
    return BatchValidate(policies_json, resources_json, ctx_json, nthreads, status_out, n_rules_out, n_res_out);
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1.0;
  }
}

long long orc_count_rules(const char* policies_json) {
  try {
    return (long long)CountRules(policies_json);
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

double orc_validate_ndjson(const char* policies_json, const char* ndjson, size_t len, const char* ctx_json, int nthreads,
                           unsigned char* status_out, size_t n_res, int preparse) {
  try {
    return BatchValidateNdjson(policies_json, ndjson, len, ctx_json, nthreads, status_out, n_res, preparse);
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1.0;
  }
}

}  // extern "C"
