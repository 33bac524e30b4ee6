// Resource shards of an ingested batch for multi-device evaluation
// (kv_validate_devices / kv_session_create_devices): resources
// [lo, hi) with lo a multiple of KV_LANES, so the wave-group layout, lanes and
// every kernel stay unchanged on the shard. The shard's node rows are rebased
// to start at 0 and its scalar cells are renumbered onto the values the shard
// references (kept in global order, so the value-predicate table of each device
// covers only its own values, still grouped by position class). The string heap,
// label / annotation lists, namespace tables and key ids stay global.
#include <algorithm>
#include <stdexcept>

#include "kvinternal.hpp"

namespace kvh {

using namespace kv;

void make_shard(const Batch& b, uint64_t lo, uint64_t hi, Batch* out) {
  if (lo % KV_LANES != 0 || lo > hi || hi > b.res.size())
    throw std::runtime_error("shard: range must start at a multiple of 64 resources");
  Batch& s = *out;
  s = Batch();
  s.pin_store();
  const uint64_t row_lo = lo < b.res.size() ? b.res[lo].root : b.n_rows;
  const uint64_t row_hi = hi < b.res.size() ? b.res[hi].root : b.n_rows;
  s.n_rows = row_hi - row_lo;
  // the shard's packed cells: rows [row_lo, row_hi), their transfer units [c_lo, c_hi)
  const uint64_t c_lo = row_lo < b.n_rows ? b.roff[row_lo] : b.tcells.size();
  const uint64_t c_hi = row_hi < b.n_rows ? b.roff[row_hi] : b.tcells.size();
  const uint64_t* src = b.tcells.data() + c_lo;
  s.rmask.assign(b.rmask.begin() + row_lo, b.rmask.begin() + row_hi);
  s.rwide.assign(b.rwide.begin() + row_lo, b.rwide.begin() + row_hi);
  s.roff.resize(s.n_rows);
  for (uint64_t r = 0; r < s.n_rows; r++) s.roff[r] = b.roff[row_lo + r] - (uint32_t)c_lo;
  // values referenced by the shard, renumbered in global order (a scalar's Val id is the hi
  // word of its first unit in both transfer forms)
  std::vector<uint32_t> vmap(b.vals.size(), 0xFFFFFFFFu);
  size_t ncell = 0;
  s.each_unit([&](uint64_t, uint64_t u, bool) {
    ncell++;
    if (node_scalar_t(node_type((uint32_t)src[u]))) vmap[src[u] >> 32] = 0;
  });
  size_t nv = 0;
  for (uint32_t m : vmap) nv += m == 0;
  s.vals.reserve(nv);
  for (size_t v = 0; v < vmap.size(); v++)
    if (vmap[v] == 0) {
      vmap[v] = (uint32_t)s.vals.size();
      s.vals.push_back(b.vals[v]);
    }
  s.tcells.assign(src, src + (c_hi - c_lo));
  uint64_t* tc = s.tcells.data();
  s.each_unit([&](uint64_t, uint64_t u, bool wide) {
    const uint32_t t = node_type((uint32_t)tc[u]);
    uint32_t a = (uint32_t)(tc[u] >> 32);
    if (node_scalar_t(t)) a = vmap[a];
    else if (wide && (t == NT_MAP || t == NT_ARR)) a -= (uint32_t)row_lo;  // (the 8-byte form is row-relative)
    tc[u] = (tc[u] & 0xFFFFFFFFull) | (uint64_t)a << 32;
  });
  s.cells_used = ncell;
  s.res.assign(b.res.begin() + lo, b.res.begin() + hi);
  for (Res& r : s.res) r.root -= (uint32_t)row_lo;
  match_tuples(&s);  // the shard's own tuples (its table holds only those)
  s.kvs = b.kvs;
  s.strs = b.strs;
  s.dyn_keys = b.dyn_keys;
  s.namespaces = b.namespaces;
  s.nsms = b.nsms;
  s.lsets = b.lsets;
  s.asets = b.asets;
  s.ns_labels = b.ns_labels;
  s.ns_bits = b.ns_bits;
  s.ns_words = b.ns_words;
  if (!b.vout.empty()) {  // pattern-variable outcomes of the shard's resources (ids stay global)
    const size_t K = b.vout.size() / b.res.size();
    s.vout.assign(b.vout.begin() + lo * K, b.vout.begin() + hi * K);
    s.vout_tab = b.vout_tab;
  }
  s.bytes_referenced = s.cells_used * sizeof(Node) + s.vals.size() * sizeof(Val) + s.res.size() * sizeof(Res) +
                       s.kvs.size() * sizeof(KV) + s.strs.size() + s.nsms.size() * sizeof(StrRef) +
                       (s.lsets.size() + s.asets.size()) * sizeof(KVSet);
}

std::vector<std::pair<uint64_t, uint64_t>> shard_ranges(uint64_t n, uint32_t g) {
  // contiguous ranges [k*N/G, (k+1)*N/G), cut at wave-group (64 resource) boundaries
  std::vector<std::pair<uint64_t, uint64_t>> out;
  const uint64_t groups = (n + KV_LANES - 1) / KV_LANES;
  for (uint32_t k = 0; k < g; k++) {
    const uint64_t a = std::min<uint64_t>(n, groups * k / g * KV_LANES);
    const uint64_t e = std::min<uint64_t>(n, groups * (k + 1) / g * KV_LANES);
    out.push_back({a, e});
  }
  return out;
}

}  // namespace kvh
