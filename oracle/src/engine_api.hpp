// ORACLE — test infrastructure only (see ovalue.hpp header).
#pragma once
#include <string>

#include "ovalue.hpp"

namespace orc {
// validateResourceElement / validateMap entry for matcher fixtures (entry 1 / 2)
bool ValidateElementEntry(int entry, const Value& resource, Value& pattern, std::string* path, std::string* msg);
// engine.Validate of one policy on one resource, serialized as JSON
std::string ValidateToJSON(const Value& policy, const Value& resource, const Value& ctx);
// every outcome over the reference's Go map iteration orders (matcher.hpp Chooser), per rule
std::string EnumerateToJSON(const Value& policy, const Value& resource, const Value& ctx, int cap);
double BatchValidate(const char* policies_json, const char* resources_json, const char* ctx_json, int nthreads,
                     unsigned char* status_out, long long* n_rules_out, long long* n_res_out);
size_t CountRules(const char* policies_json);
double BatchValidateNdjson(const char* policies_json, const char* ndjson, size_t len, const char* ctx_json,
                           int nthreads, unsigned char* status_out, size_t n_res, int preparse);
}  // namespace orc
