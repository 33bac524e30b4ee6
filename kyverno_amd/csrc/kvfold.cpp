// Launch-time host folding shared by the device runtime (kvapi.cpp) and the
// host-side debugging harness of the generated kernels (tools/kvemu):
//  * batch-constant user-info criteria of match/exclude blocks
//    (pkg/engine/utils.go:183-229, :340-342) folded into per-filter flags;
//  * the key string table of a batch (static dictionary, then batch keys).
#include <algorithm>
#include <cstring>

#include "kvinternal.hpp"

namespace kvh {

using namespace kv;

namespace {

struct AdmissionCtx {
  std::vector<std::string> roles, clusterRoles, groups, dyn;
  std::string username;
  bool empty() const { return roles.empty() && clusterRoles.empty() && groups.empty() && username.empty(); }
};

// ctx_json: {"admission": {"roles":[], "clusterRoles":[], "groups":[], "username":""}, "excludeGroupRole": []}
AdmissionCtx parse_ctx(const char* ctx_json) {
  AdmissionCtx c;
  if (!ctx_json || !*ctx_json) return c;
  JDoc d;
  parse_json(ctx_json, strlen(ctx_json), NUM_FLOAT, &d);
  auto list = [&](int64_t n, std::vector<std::string>* out) {
    if (n < 0 || d.at((uint32_t)n).t != J_ARR) return;
    const JNode& a = d.at((uint32_t)n);
    for (uint32_t k = a.first; k < a.first + a.count; k++)
      if (d.at(k).t == J_STR) out->push_back(std::string(d.sval(d.at(k))));
  };
  int64_t a = d.get(d.root, "admission");
  if (a >= 0 && d.at((uint32_t)a).t == J_MAP) {
    list(d.get((uint32_t)a, "roles"), &c.roles);
    list(d.get((uint32_t)a, "clusterRoles"), &c.clusterRoles);
    list(d.get((uint32_t)a, "groups"), &c.groups);
    int64_t u = d.get((uint32_t)a, "username");
    if (u >= 0 && d.at((uint32_t)u).t == J_STR) c.username = std::string(d.sval(d.at((uint32_t)u)));
  }
  list(d.get(d.root, "excludeGroupRole"), &c.dyn);
  return c;
}

bool slice_contains(const std::vector<std::string>& s, const std::vector<std::string>& v) {
  for (auto& x : v)
    if (std::find(s.begin(), s.end(), x) != s.end()) return true;
  return false;
}

// user-info part of doesResourceMatchConditionBlock (pkg/engine/utils.go:183-229):
// true if it appends errors (every checked criterion failed)
bool ui_fails(const UserInfoSpec& ui, const AdmissionCtx& ai) {
  std::vector<std::string> keys = ai.groups;
  keys.push_back(ai.username);
  int checked = 0, uerr = 0;
  if (!ui.roles.empty() && !slice_contains(keys, ai.dyn)) {
    checked++;
    if (!slice_contains(ui.roles, ai.roles)) uerr++;
    else return false;
  }
  if (!ui.clusterRoles.empty() && !slice_contains(keys, ai.dyn)) {
    checked++;
    if (!slice_contains(ui.clusterRoles, ai.clusterRoles)) uerr++;
    else return false;
  }
  if (!ui.subjects.empty()) {
    checked++;
    const std::string sa = "system:serviceaccount:";
    std::vector<UserInfoSpec::Subj> subs = ui.subjects;
    for (auto& e : ai.dyn) subs.push_back({"Group", e, ""});
    bool m = false;
    for (auto& s : subs) {
      if (s.kind == "ServiceAccount") {
        if (ai.username.size() <= sa.size()) continue;
        if (ai.username.substr(sa.size()) == s.ns + ":" + s.name) { m = true; break; }
      } else if (s.kind == "User" || s.kind == "Group") {
        if (std::find(keys.begin(), keys.end(), s.name) != keys.end()) { m = true; break; }
      }
    }
    if (!m) uerr++;
    else return false;
  }
  return checked == uerr && uerr > 0;
}

}  // namespace

std::vector<uint32_t> fold_filters(const PolicySet& ps, const char* ctx_json) {
  const AdmissionCtx ai = parse_ctx(ctx_json);
  std::vector<uint32_t> out(ps.filters.size());
  size_t f = 0;
  for (size_t r = 0; r < ps.rules.size(); r++) {
    const RuleHost& rh = ps.rhost[r];
    for (size_t k = 0; k < rh.filter_ui.size(); k++, f++) {
      uint32_t fl = ps.filters[f].flags & ~(MF_EMPTY | MF_UI_FAIL);
      bool rd_empty = ps.filters[f].flags & MF_EMPTY;
      UserInfoSpec ui = rh.filter_ui[k];
      if (rh.filter_is_match[k] && ai.empty()) ui = UserInfoSpec();  // utils.go:340-342
      if (rd_empty && !ui.present) fl |= MF_EMPTY;
      if (ui.present && ui_fails(ui, ai)) fl |= MF_UI_FAIL;
      out[f] = fl;
    }
  }
  return out;
}

void key_table(const PolicySet& ps, const Batch& b, std::vector<uint32_t>* off, std::vector<uint32_t>* len,
               std::string* ks) {
  off->clear();
  len->clear();
  ks->clear();
  auto addk = [&](const std::string& k) {  // 4-byte aligned (word-granular glob)
    while (ks->size() & 3) ks->push_back('\0');
    off->push_back((uint32_t)ks->size());
    len->push_back((uint32_t)k.size());
    *ks += k;
  };
  for (auto& k : ps.keys) addk(k);
  for (auto& k : b.dyn_keys) addk(k);
  ks->append(16, '\0');
}

std::vector<uint32_t> mtab_bit_filters(const PolicySet& ps) {
  const uint32_t ns_w = (ps.n_nss_bits + 31) / 32, an_w = (ps.n_ann_bits + 31) / 32;
  std::vector<uint32_t> out((size_t)(ns_w + an_w) * 32, 0xFFFFFFFFu);
  for (uint32_t f = 0; f < ps.filters.size(); f++) {
    const MFilter& F = ps.filters[f];
    if (F.flags & MF_NSS) out[F.nss_bit] = f;
    if (F.flags & MF_ANN) out[(size_t)ns_w * 32 + F.ann_bit] = f;
  }
  return out;
}

}  // namespace kvh
