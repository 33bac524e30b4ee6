// Host-side internal structures of libkvgpu (compiled policy set, ingested batch).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <new>
#include <string>
#include <type_traits>
#include <utility>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "kvcell.h"
#include "kv_layout.h"
#include "kvjson.hpp"

namespace kvh {

// Mutable pattern tree (copy of an apiextensions.JSON value: numbers are float64)
struct PV {
  uint8_t t = J_NULL;
  bool b = false;
  double f = 0;
  std::string s;
  std::vector<std::string> mk;  // map keys
  std::vector<std::string> mo;  // canonical order keys (== mk unless renamed)
  std::vector<PV> mv;           // map values
  std::vector<PV> a;            // array elements
  int32_t vstr = -1;            // J_STR holding {{ }} variables: its VarStr (PolicySet::vstrs)
  int find(const std::string& k) const {
    for (size_t i = 0; i < mk.size(); i++)
      if (mk[i] == k) return (int)i;
    return -1;
  }
};
PV to_pv(const JDoc& d, uint32_t node);

// Path template of a pattern node, for rendering failing paths on the host.
enum SegKind : uint8_t { SEG_ROOT = 0, SEG_KEY = 1, SEG_LOOP = 2, SEG_CONST_INDEX = 3, SEG_RESOLVED = 4 };
struct PNodeInfo {
  uint32_t parent;   // 0xFFFFFFFF for root
  uint8_t seg;       // SegKind
  uint32_t level;    // SEG_LOOP: loop level; SEG_CONST_INDEX: index
  std::string key;   // SEG_KEY text; SEG_RESOLVED: literal fallback (anchor-free pattern key)
  // Error-message operands of the pattern value at this node (kv_result_error_message):
  uint8_t wrap = 0;      // 1: condition-anchor key, 2: global-anchor key (anchor.go:72-95 wraps errors below)
  std::string pat_t;     // Go %T of the pattern value ("map[string]interface {}", "[]interface {}", ...)
  std::string pat_v;     // Go %v of the compared scalar (the value, or element 0 of a scalar list)
  uint32_t pat_len = 0;  // pattern array length (validate.go:172)
  int32_t dleaf = -1;    // a dynamic leaf (pattern variables) compares here: pat_v is per resource
};

// A pattern string holding {{ }} variables (kvvars.cpp): `text` after $() references, `path`
// its traversal path in the pattern document (getJMESPath of {{@}}), `key` the distinct
// (text, path) resolved once per resource at ingest.
struct VarStr {
  uint32_t rule = 0;
  std::string text, path;
  uint32_t key = 0;
  bool want_string = false;  // under metadata.labels / annotations (ExpandInMetadata needs a string)
};

// Projection trie over resource key paths referenced by any compiled pattern
// or match block. Arrays are transparent: `elem` is the element trie.
struct Trie {
  struct N {
    std::unordered_map<std::string, uint32_t> kids;
    int32_t elem = -1;
    bool keep_all = false;   // keep every child (labels/annotations with wildcard keys)
    bool keep_subtree = false;
    // slot-addressed layout (finalize_slots): kid keys sorted by bytes; a
    // resource map at this trie node stores child i in slot i (NT_ABSENT if missing)
    std::vector<std::string> slot_keys;
    std::unordered_map<std::string, uint32_t> slot;
  };
  std::vector<N> nodes;
  Trie() { nodes.emplace_back(); }
  uint32_t child(uint32_t n, const std::string& k) {
    auto it = nodes[n].kids.find(k);
    if (it != nodes[n].kids.end()) return it->second;
    uint32_t id = (uint32_t)nodes.size();
    nodes.emplace_back();
    nodes[n].kids[k] = id;
    return id;
  }
  uint32_t elem(uint32_t n) {
    if (nodes[n].elem >= 0) return (uint32_t)nodes[n].elem;
    uint32_t id = (uint32_t)nodes.size();
    nodes.emplace_back();
    nodes[n].elem = (int32_t)id;
    return id;
  }
};

struct UserInfoSpec {
  bool present = false;  // any of roles/clusterRoles/subjects non-nil
  std::vector<std::string> roles, clusterRoles;
  struct Subj { std::string kind, name, ns; };
  std::vector<Subj> subjects;
};

struct SelectorHost {   // namespaceSelector, evaluated on the host per namespace (batch constant)
  std::vector<std::pair<std::string, std::string>> matchLabels;
  struct Expr { std::string key, op; std::vector<std::string> values; };
  std::vector<Expr> exprs;
};

struct RuleHost {
  uint32_t policy = 0;
  std::string name;
  std::string route_reason;  // "" for GPU
  std::string message;
  bool anypattern = false;
  uint32_t root_pnode = 0;
  std::vector<uint32_t> alt_roots;
  std::vector<UserInfoSpec> filter_ui;  // per MFilter of this rule (match then exclude)
  std::vector<bool> filter_is_match;
  std::string const_message;            // route 3
};

struct PolicySet {
  std::vector<std::string> policy_names;
  std::vector<uint32_t> policy_rule_first, policy_rule_count;
  // dictionary of keys (pattern keys, kinds, groups, versions)
  std::vector<std::string> keys;
  std::unordered_map<std::string, uint32_t> key_id;
  uint32_t intern(const std::string& k) {
    auto it = key_id.find(k);
    if (it != key_id.end()) return it->second;
    uint32_t id = (uint32_t)keys.size();
    keys.push_back(k);
    key_id.emplace(k, id);
    return id;
  }
  uint32_t lookup(std::string_view k) const {
    auto it = key_id.find(std::string(k));
    return it == key_id.end() ? kv::KEY_NONE : it->second;
  }
  std::string strs;  // program string table
  uint32_t add_str(const std::string& s) {
    uint32_t off = (uint32_t)strs.size();
    strs += s;
    return off;
  }
  std::vector<kv::Inst> prog;
  std::vector<kv::Pred> preds;
  std::vector<kv::Alt> alts;
  std::vector<kv::Conj> conjs;
  std::vector<kv::Atom> atoms;
  std::unordered_map<std::string, uint32_t> pred_cache;
  std::vector<uint32_t> kg_specs;  // wildcard label-map sibling specs (OP_KEYGLOB)
  std::vector<kv::GSeg> gsegs;     // compiled glob segments
  std::vector<kv::GWord> gwords;
  void compile_glob(kv::Atom& a, const std::string& pattern);
  std::vector<kv::RuleRec> rules;
  std::vector<RuleHost> rhost;
  std::vector<kv::MFilter> filters;
  std::vector<kv::KindSpec> kinds;
  std::vector<kv::StrRef> strrefs;
  std::vector<kv::StrPair> strpairs;
  std::vector<kv::Selector> selectors;
  std::vector<kv::SelLabel> sellabels;
  std::vector<kv::SelExpr> selexprs;
  std::vector<SelectorHost> nsselectors;  // bit i of the namespace table
  uint32_t n_nss_bits = 0, n_ann_bits = 0;  // rows of the namespace-glob / annotation match tables
  // per filter: compiled glob atoms of `name` (first, if MF_NAME) then `names` (specialized kernels)
  std::vector<std::vector<uint32_t>> filter_name_atoms;
  std::vector<PNodeInfo> pnodes;
  Trie trie;
  std::vector<std::tuple<uint32_t, uint32_t, std::string>> slot_fix;  // (pc, trie node, key)
  uint32_t max_depth = 0, max_loops = 0;
  std::string flags_info;
  // pattern variables (kvvars.cpp): strings in traversal order per rule, distinct
  // (text, path) keys, dynamic leaves (OP_VLEAF a) -> VarStr, and per dynamic rule
  // (RuleRec::dyn - 1) its VarStr range
  std::vector<VarStr> vstrs;
  std::vector<std::pair<std::string, std::string>> vkeys;
  std::vector<uint32_t> dleaf_vstr;
  std::vector<std::pair<uint32_t, uint32_t>> dyn_rules;
};

// Compiles a JSON list of (already autogen-expanded) ClusterPolicy/Policy
// objects. Throws std::runtime_error on malformed input.
void compile_policies(const char* json, size_t len, PolicySet* ps);

// Host memory of the large store arrays of an ingested batch. libkvgpu (kvapi.cpp)
// installs a pooled page-locked allocator, so the store's H2D upload is one direct
// DMA instead of a copy through a staging ring; without it (host-only builds) plain
// malloc. `take` returns nullptr to fall back; `give` returns false for a block it
// does not own.
struct HostMem {
  void* (*take)(size_t bytes) = nullptr;
  bool (*give)(void* p) = nullptr;
};
extern HostMem g_hostmem;  // kvingest.cpp

// Large pageable host arrays (the ingest's per-thread parts, its interning tables) in
// transparent huge pages: 2 MiB-aligned blocks advised MADV_HUGEPAGE (the hosts run THP in
// `madvise` mode). Each part's arrays are written once and freed by the merge; with 4 KiB pages
// their faults and unmapping cost ~40 ms of a million-Pod ingest on the GPU box (C2 2.5 -> 2.9-3.0
// M Pods/s measured with the same advice through glibc's malloc.hugetlb tunable).
void* thp_alloc(size_t bytes);
inline void thp_free(void* p) { free(p); }
template <class T>
struct ThpAlloc {
  using value_type = T;
  ThpAlloc() = default;
  template <class U>
  ThpAlloc(const ThpAlloc<U>&) {}
  T* allocate(size_t n) { return (T*)thp_alloc(n * sizeof(T)); }
  void deallocate(T* p, size_t) { thp_free(p); }
  template <class U>
  bool operator==(const ThpAlloc<U>&) const { return true; }
  template <class U>
  bool operator!=(const ThpAlloc<U>&) const { return false; }
};

// Allocator of the store arrays: `pinned` (the merged batch and its shards) takes
// blocks of >= 16 MiB from g_hostmem; the ingest's per-thread parts stay pageable (huge pages).
template <class T>
struct StoreAlloc {
  using value_type = T;
  using propagate_on_container_swap = std::true_type;
  using propagate_on_container_move_assignment = std::true_type;
  using propagate_on_container_copy_assignment = std::true_type;
  using is_always_equal = std::false_type;
  bool pinned = false;
  StoreAlloc() = default;
  explicit StoreAlloc(bool p) : pinned(p) {}
  template <class U>
  StoreAlloc(const StoreAlloc<U>& o) : pinned(o.pinned) {}
  T* allocate(size_t n) {
    const size_t bytes = n * sizeof(T);
    if (pinned && g_hostmem.take && bytes >= (16u << 20))
      if (void* p = g_hostmem.take(bytes)) return (T*)p;
    return (T*)thp_alloc(bytes);
  }
  void deallocate(T* p, size_t) {
    if (pinned && g_hostmem.give && g_hostmem.give(p)) return;
    thp_free(p);
  }
  // resize() leaves trivially constructible elements uninitialised (the merge and the
  // shard builder write every element; zero-filling 1.5 GB of cells was a serial pass)
  template <class U>
  void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) {
    ::new ((void*)p) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new ((void*)p) U(std::forward<A>(a)...);
  }
  template <class U>
  bool operator==(const StoreAlloc<U>& o) const { return pinned == o.pinned; }
  template <class U>
  bool operator!=(const StoreAlloc<U>& o) const { return pinned != o.pinned; }
};
template <class T>
using StoreVec = std::vector<T, StoreAlloc<T>>;
// the string heap: page-locked in the merged batch (one direct DMA), huge pages in the parts
using HeapStr = std::basic_string<char, std::char_traits<char>, StoreAlloc<char>>;

// Ingested batch (host mirror of the HBM store)
struct Batch {
  // Node rows in packed form: the wave-group layout (kvingest.cpp) has n_rows rows of
  // KV_LANES cells (node index = row * KV_LANES + lane); the host keeps only the non-zero
  // cells of every row in row order, in their transfer form (`tcells`, kv_layout.h: 8 bytes a
  // cell, 16 for the lanes of the row's `rwide` mask), a 64-bit lane mask per row (`rmask`) and
  // the first 8-byte unit of each row (`roff`). kv_validate uploads these and expands the rows
  // on the device (kv_expand_rows_kernel), so neither the row padding (40+ % of the cells at
  // C2) nor the Node fields that follow from the values cross PCIe.
  uint64_t n_rows = 0;
  uint64_t cells_used = 0;           // populated cells (incl. absent-slot markers)
  StoreVec<kv::Val> vals;
  StoreVec<kv::Res> res;
  StoreVec<uint64_t> tcells;
  StoreVec<uint64_t> rmask, rwide;
  StoreVec<uint32_t> roff;
  // the transfer units of (row, lane), a set rmask bit
  const uint64_t* unit(uint64_t row, uint64_t lane) const {
    const uint64_t below = (1ull << lane) - 1ull;
    return tcells.data() + roff[row] + __builtin_popcountll(rmask[row] & below) +
           __builtin_popcountll(rwide[row] & below);
  }
  // cell `idx` of the padded layout (zero Node where the row has no cell in that lane)
  kv::Node cell(uint64_t idx) const {
    const uint64_t row = idx / kv::KV_LANES, lane = idx % kv::KV_LANES;
    if (row >= n_rows || !((rmask[row] >> lane) & 1ull)) return kv::Node{0u, 0u, 0u, 0u};
    const uint64_t* u = unit(row, lane);
    if ((rwide[row] >> lane) & 1ull)
      return kv::Node{(uint32_t)u[0], (uint32_t)(u[0] >> 32), (uint32_t)u[1], (uint32_t)(u[1] >> 32)};
    return kv::cell_widen((uint32_t)u[0], (uint32_t)(u[0] >> 32), row, vals.data());
  }
  // bytes the batch's store crosses PCIe in (kv_validate's upload)
  uint64_t transfer_bytes() const;
  // f(row, unit index, wide) for every cell of rows [0, n_rows), in unit order
  template <class F>
  void each_unit(F f) const {
    uint64_t u = 0;
    for (uint64_t row = 0; row < n_rows; row++) {
      const uint64_t w = rwide[row];
      for (uint64_t m = rmask[row]; m; m &= m - 1) {
        const bool wide = (w >> __builtin_ctzll(m)) & 1ull;
        f(row, u, wide);
        u += wide ? 2 : 1;
      }
    }
  }
  uint64_t n_cells() const { return n_rows * kv::KV_LANES; }
  // store order: resource i of the store (its wave group, its status column) is resource
  // order[i] of the caller's input; empty = the input order. Ingest groups resources of one
  // kind into common wave groups (kvingest.cpp), the result accessors map indices back.
  std::vector<uint32_t> order;
  // match tuples (Res::tup): a store index of each tuple's first resource
  std::vector<uint32_t> tup_rep;
  // kind entities (factored match, DevBatch::tup_kent): distinct (kind, group, version, kind
  // flags) of the tuples; the entity of each tuple and a resource of each entity
  std::vector<uint32_t> tup_kent, kent_rep;
  // the arrays that cross PCIe in page-locked memory when g_hostmem provides it
  void pin_store() {
    vals = StoreVec<kv::Val>(StoreAlloc<kv::Val>(true));
    res = StoreVec<kv::Res>(StoreAlloc<kv::Res>(true));
    tcells = StoreVec<uint64_t>(StoreAlloc<uint64_t>(true));
    rmask = StoreVec<uint64_t>(StoreAlloc<uint64_t>(true));
    rwide = StoreVec<uint64_t>(StoreAlloc<uint64_t>(true));
    roff = StoreVec<uint32_t>(StoreAlloc<uint32_t>(true));
    strs = HeapStr(StoreAlloc<char>(true));
  }
  std::vector<kv::KV> kvs;
  HeapStr strs;                      // string heap
  std::vector<std::string> dyn_keys; // key ids >= ps.keys.size()
  std::vector<std::string> namespaces;
  std::vector<kv::StrRef> nsms;      // distinct checkNameSpace strings (Res::nsm)
  std::vector<kv::KVSet> lsets;      // distinct label lists (Res::lset)
  std::vector<kv::KVSet> asets;      // distinct annotation lists (Res::aset)
  std::vector<std::string> nsm_keys, lset_keys, aset_keys;  // interning keys (ingest only)
  std::vector<std::vector<std::pair<std::string, std::string>>> ns_labels;
  std::vector<uint32_t> ns_bits;     // [n_ns][ceil(n_nssel/32)]
  uint32_t ns_words = 1;
  uint64_t bytes_referenced = 0;     // algorithmic bytes of the projected store
  // pattern variables: outcome id per (resource, PolicySet::vkeys entry), resource-major,
  // and the distinct outcomes (kvvars.cpp resolve_var_string encoding)
  std::vector<uint32_t> vout;
  std::vector<std::string> vout_tab;
  std::unordered_map<std::string, uint32_t> vout_id;  // (ingest only)
};

// Per-batch tables of the pattern variables (kvvars.cpp build_dyn): the predicate of every
// distinct outcome (pred id == outcome id), the outcome of each dynamic leaf
// [dleaf][res], and the status substitution decides per [dyn rule][res] (0 / ST_ERROR /
// ST_CPU) with the ERROR's outcome id (its message) in dyn_msg.
struct DynHost {
  PolicySet tbl;
  std::vector<uint32_t> dleaf;
  std::vector<uint8_t> dyn_st;
  std::vector<uint32_t> dyn_msg;
};
void build_dyn(const PolicySet& ps, const Batch& b, DynHost* out);
bool var_string(const std::string& s);
bool var_string_in_scope(const std::string& s, const std::string& path);
std::string unescape_var_string(const std::string& s);
std::string resolve_var_string(const std::string& tmpl, const std::string& path, const JDoc& d);
PV outcome_value(const std::string& o);
uint32_t compile_leaf_pred(PolicySet& tbl, const PV& value);  // kvcompile.cpp
std::string pattern_go_v(const PV& p);                         // Go %v of a scalar pattern value

void ingest_resources(const PolicySet& ps, const char* json, size_t len, const char* ns_labels_json, Batch* b);
// Res::tup and Batch::tup_rep: resources whose match inputs (kind, group, version, checkNameSpace
// string, label / annotation lists, namespace, flags) are equal share a tuple id, numbered in
// store order (kvingest.cpp)
void match_tuples(Batch* b);

// Launch-time folding (kvfold.cpp): per-filter flags with the batch-constant
// user-info criteria folded in (ctx_json: AdmissionInfo / ExcludeGroupRole, or
// NULL), and the batch key string table (4-byte aligned entries).
std::vector<uint32_t> fold_filters(const PolicySet& ps, const char* ctx_json);
// DevPS::mt_bitf: the filter owning each namespace-glob bit, then each annotation bit
// (rows padded to 32 bits, 0xFFFFFFFF where no filter)
std::vector<uint32_t> mtab_bit_filters(const PolicySet& ps);
void key_table(const PolicySet& ps, const Batch& b, std::vector<uint32_t>* off, std::vector<uint32_t>* len,
               std::string* ks);

// Resource shards of a batch (kvshard.cpp): resources [lo, hi), lo a multiple of
// KV_LANES; rows rebased, values renumbered onto those the shard references.
void make_shard(const Batch& b, uint64_t lo, uint64_t hi, Batch* out);
// G contiguous ranges [k*N/G, (k+1)*N/G) of N resources, cut at 64-resource boundaries
std::vector<std::pair<uint64_t, uint64_t>> shard_ranges(uint64_t n, uint32_t g);

// Go-semantics helpers shared by compiler and ingest
bool wildcard_match_host(std::string_view pattern, std::string_view name);
bool valid_label_key(const std::string& k);
bool valid_label_value(const std::string& v);
std::string remove_anchor(const std::string& key, std::string* prefix);
bool is_condition_anchor(const std::string& s);
bool is_global_anchor(const std::string& s);
bool is_negation_anchor(const std::string& s);
bool is_equality_anchor(const std::string& s);
bool is_existence_anchor(const std::string& s);
int selector_eval_host(const SelectorHost& sel, std::vector<std::pair<std::string, std::string>> labels);

}  // namespace kvh
