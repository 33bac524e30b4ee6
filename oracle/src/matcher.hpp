// ORACLE — test infrastructure only (see ovalue.hpp header).
#pragma once
#include <map>
#include <string>
#include <vector>

#include "ovalue.hpp"

namespace orc {

// Thrown where the reference would panic (Go type assertions in
// pkg/engine/wildcards/wildcards.go:85,129,132).
struct GoPanic {
  std::string what;
};

// pkg/engine/common/anchorKey.go:81-145
struct AnchorKey {
  std::map<std::string, bool> anchorMap;
  bool IsAnchorError() const {
    for (auto& kv : anchorMap)
      if (!kv.second) return true;
    return false;
  }
  void CheckAnchorInResource(const Value& pattern, const Value& resource);
};

struct Err {
  bool set = false;
  std::string msg;
  static Err none() { return Err(); }
  static Err mk(const std::string& m) { Err e; e.set = true; e.msg = m; return e; }
};

struct PathErr {
  std::string path;
  Err err;
};

// pkg/engine/validate/validate.go:13-50
struct PatternError {
  bool set = false;
  std::string msg;
  std::string path;
  bool skip = false;
};

PatternError MatchPattern(const Value* resource, Value& pattern);  // pattern may be mutated (ExpandInMetadata)

// pkg/engine/validate/pattern.go:25-318
bool ValidateValueWithPattern(const Value* value, const Value& pattern);
bool validateValueWithStringPattern(const Value* value, const std::string& pattern);
bool validateNumberWithStr(const Value* value, const std::string& pattern, const std::string& op);
bool validateString(const Value* value, const std::string& pattern, const std::string& op);
bool validateValueWithNilPattern(const Value* value);
bool validateValueWithFloatPattern(const Value* value, double pattern);
// pkg/engine/operator/operator.go:33-67
std::string GetOperatorFromStringPattern(const std::string& pattern);
void getNumberAndStringPartsFromPattern(const std::string& pattern, std::string* number, std::string* str);

// pkg/engine/anchor/common/common.go
bool IsConditionAnchor(const std::string& s);
bool IsGlobalAnchor(const std::string& s);
bool IsNegationAnchor(const std::string& s);
bool IsAddingAnchor(const std::string& s);
bool IsEqualityAnchor(const std::string& s);
bool IsExistenceAnchor(const std::string& s);
std::string RemoveAnchor(const std::string& key, std::string* prefix = nullptr);
std::string RemoveAnchorsFromPath(const std::string& s);
bool IsConditionalAnchorError(const std::string& msg);
bool IsGlobalAnchorError(const std::string& msg);

// pkg/engine/wildcards/wildcards.go
void ExpandInMetadata(Value& patternMap, const Value& resourceMap);

// $() references: pkg/engine/variables/vars.go:253-309,450-554
// Returns false with *err set on failure (message as the reference formats it).
bool SubstituteReferences(Value& document, std::string* err, bool unescape = true);
// validate.pattern variables (subst.cpp "pattern variables"): QueryObject returns 0 found
// (*out, nullptr for null), 1 unknown key (*missing), 2 outside the device scope;
// SubstitutePatternVars 0 ok, 1 error (*err = the reference's message), 2 outside scope;
// *structural: some whole-string variable resolved to a map / array (a structural pattern)
int QueryObject(const std::string& q, const Value& resource, const Value** out, std::string* missing);
bool PatternVarsInScope(const Value& doc);
int SubstitutePatternVars(Value& doc, const Value& resource, std::string* err, bool* structural = nullptr);
bool SubstituteMessage(const std::string& msg, const Value& resource, std::string* out);
// True if the string contains an unescaped {{...}} (RegexVariables, vars.go:20)
bool HasVariable(const std::string& s);
bool DocHasVariable(const Value& v);

// Enumerate mode: where the reference iterates a Go map (random order)
// — the anchors and the non-anchor keys of validateMap (validate.go:110-135, with
// getSortedNestedAnchorResource's front / back lists, validate/utils.go:37-51) and the
// resource label keys of expandWildcards (wildcards.go:38-49) — the oracle asks g_choose
// (thread-local, null = canonical order) which element comes next; the enumerator replays
// every sequence of choices to collect the set of outcomes.
struct Chooser {
  std::vector<int> prefix;   // choices to replay
  std::vector<int> taken;    // choices made this run
  std::vector<int> arity;    // number of options at each choice
  int choose(int n) {
    if (n <= 1) return 0;
    const size_t k = taken.size();
    const int c = k < prefix.size() ? prefix[k] : 0;
    taken.push_back(c);
    arity.push_back(n);
    return c;
  }
};
extern thread_local Chooser* g_choose;

}  // namespace orc
