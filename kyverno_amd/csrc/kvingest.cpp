// Resource ingest: JSON (unstructured typing) -> projected, string-interned
// node store laid out for HBM (kv_layout.h). Only key paths referenced by the
// compiled policy set are kept (projection trie); match/exclude inputs go to the
// per-resource header. Scalar values are deduplicated into Val records whose
// Go-semantics string/number/quantity forms are precomputed once here:
//   validateString form       pkg/engine/validate/pattern.go:222-260
//   validateNumberWithStr form pkg/engine/validate/pattern.go:264-289, common.go:9-28
//   float pattern compare      pkg/engine/validate/pattern.go:96-127
//   nil pattern compare        pkg/engine/validate/pattern.go:129-150
// Resource identity for match/exclude follows unstructured accessors
// (GetKind/GetName/GetNamespace/GetLabels/GetAnnotations, GroupVersionKind).
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <unordered_map>

#include "kvinternal.hpp"

namespace kvh {

using namespace kv;

namespace {

struct Ingest {
  const PolicySet& ps;
  Batch& b;
  std::unordered_map<std::string, uint32_t> str_off;   // dedup of string heap
  std::unordered_map<std::string, uint32_t> val_id;    // dedup of scalars
  std::unordered_map<std::string, uint32_t> dyn_key;   // batch-local key ids
  std::unordered_map<std::string, uint32_t> ns_index;
  uint32_t nstatic;

  Ingest(const PolicySet& p, Batch& bb) : ps(p), b(bb), nstatic((uint32_t)p.keys.size()) {
    // offset 0 holds "0": convertNumberToString(nil) for the device glob (kvkernel.hip atom_eval)
    str("0");
  }

  uint32_t str(std::string_view s) {
    std::string k(s);
    auto it = str_off.find(k);
    if (it != str_off.end()) return it->second;
    // 4-byte aligned: the device glob compares whole words (kvkernel.hip seg_at)
    while (b.strs.size() & 3) b.strs.push_back('\0');
    uint32_t off = (uint32_t)b.strs.size();
    b.strs.append(s.data(), s.size());
    str_off.emplace(std::move(k), off);
    return off;
  }

  uint32_t key_of(std::string_view k) {
    uint32_t id = ps.lookup(k);
    if (id != KEY_NONE) return id;
    std::string ks(k);
    auto it = dyn_key.find(ks);
    if (it != dyn_key.end()) return it->second;
    uint32_t nid = nstatic + (uint32_t)b.dyn_keys.size();
    b.dyn_keys.push_back(ks);
    dyn_key.emplace(ks, nid);
    return nid;
  }

  uint32_t val(const JDoc& d, const JNode& n) {
    std::string k;
    switch (n.t) {
      case J_BOOL: k = n.b ? "b1" : "b0"; break;
      case J_INT: k = "i" + std::to_string(n.i); break;
      case J_FLOAT: { k = "f"; k.append((const char*)&n.f, 8); break; }
      default: k = "s"; k += d.sval(n); break;
    }
    auto it = val_id.find(k);
    if (it != val_id.end()) return it->second;
    Val v{};
    std::string e, num;
    bool nvalid = true;
    switch (n.t) {
      case J_BOOL:
        v.type = NT_BOOL;
        e = n.b ? "true" : "false";
        nvalid = false;
        v.flags |= n.b ? VF_BOOLV : VF_NILLIKE;
        break;
      case J_INT:
        v.type = NT_INT;
        v.i = n.i;
        e = std::to_string(n.i);
        num = e;
        if (n.i == 0) v.flags |= VF_NILLIKE;
        break;
      case J_FLOAT:
        v.type = NT_FLOAT;
        v.f = n.f;
        e = go_format_E(n.f);
        num = go_format_f6(n.f);
        if (n.f == 0.0) v.flags |= VF_NILLIKE;
        break;
      default: {
        v.type = NT_STR;
        std::string_view sv = d.sval(n);
        e = std::string(sv);
        num = e;
        double f;
        if (go_parse_float(sv, &f)) { v.flags |= VF_PF_OK; v.f = f; }
        if (sv.empty()) v.flags |= VF_NILLIKE;
        break;
      }
    }
    v.e_off = str(e);
    v.e_len = (uint32_t)e.size();
    if (utf8_ascii(e)) v.flags |= VF_ASCII_E;
    if (nvalid) {
      v.flags |= VF_N_VALID;
      v.n_off = str(num);
      v.n_len = (uint32_t)num.size();
      if (utf8_ascii(num)) v.flags |= VF_ASCII_N;
      QCanon q = parse_quantity(num);
      if (q.valid) {
        v.flags |= VF_Q_VALID;
        if (q.neg) v.flags |= VF_Q_NEG;
        if (q.zero) v.flags |= VF_Q_ZERO;
        v.q_exp = q.exp;
        v.q_hi = q.hi;
        v.q_lo = q.lo;
      }
    }
    uint32_t id = (uint32_t)b.vals.size();
    b.vals.push_back(v);
    val_id.emplace(std::move(k), id);
    return id;
  }

  // Fill node `slot` from JSON node jn projected through trie node t (-1: leaf only)
  void fill(const JDoc& d, uint32_t jn, int32_t t, uint32_t slot, uint32_t key) {
    const JNode& n = d.at(jn);
    Node out{key, NT_NULL, 0, 0};
    switch (n.t) {
      case J_NULL: out.type = NT_NULL; break;
      case J_BOOL: out.type = NT_BOOL; out.a = val(d, n); out.b = n.b ? 1 : 0; break;
      case J_INT: out.type = NT_INT; out.a = val(d, n); break;
      case J_FLOAT: out.type = NT_FLOAT; out.a = val(d, n); break;
      case J_STR: out.type = NT_STR; out.a = val(d, n); break;
      case J_MAP: {
        out.type = NT_MAP;
        if (t >= 0) {
          const Trie::N& tn = ps.trie.nodes[t];
          std::vector<std::pair<std::string_view, uint32_t>> kept;  // key, json child
          std::vector<int32_t> ktrie;
          for (uint32_t c = n.first; c < n.first + n.count; c++) {
            std::string_view k = d.key(d.at(c));
            auto it = tn.kids.find(std::string(k));
            if (it != tn.kids.end()) { kept.push_back({k, c}); ktrie.push_back((int32_t)it->second); }
            else if (tn.keep_all) { kept.push_back({k, c}); ktrie.push_back(-1); }
          }
          std::vector<size_t> ord(kept.size());
          for (size_t i = 0; i < ord.size(); i++) ord[i] = i;
          std::sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return kept[x].first < kept[y].first; });
          uint32_t first = (uint32_t)b.nodes.size();
          b.nodes.resize(b.nodes.size() + kept.size());
          out.a = first;
          out.b = (uint32_t)kept.size();
          for (size_t i = 0; i < ord.size(); i++) {
            size_t x = ord[i];
            fill(d, kept[x].second, ktrie[x], first + (uint32_t)i, key_of(kept[x].first));
          }
        }
        break;
      }
      case J_ARR: {
        out.type = NT_ARR;
        int32_t et = t >= 0 ? ps.trie.nodes[t].elem : -1;
        uint32_t first = (uint32_t)b.nodes.size();
        b.nodes.resize(b.nodes.size() + n.count);
        out.a = first;
        out.b = n.count;
        for (uint32_t i = 0; i < n.count; i++) fill(d, n.first + i, et, first + i, KEY_NONE);
        break;
      }
    }
    b.nodes[slot] = out;
  }

  static bool is_str_map(const JDoc& d, const JNode& m) {
    if (m.t != J_MAP) return false;
    for (uint32_t c = m.first; c < m.first + m.count; c++)
      if (d.at(c).t != J_STR) return false;
    return true;
  }

  // ExpandInMetadata panics on non-map metadata / labels, non-string label values
  bool bad_meta(const JDoc& d) {
    for (const JNode& m : d.nodes) {
      if (m.t != J_MAP) continue;
      for (uint32_t c = m.first; c < m.first + m.count; c++) {
        const JNode& ch = d.at(c);
        if (d.key(ch) != "metadata" || ch.t == J_NULL) continue;
        if (ch.t != J_MAP) return true;
        for (uint32_t g = ch.first; g < ch.first + ch.count; g++) {
          const JNode& t = d.at(g);
          std::string_view k = d.key(t);
          if ((k == "labels" || k == "annotations") && t.t != J_NULL && !is_str_map(d, t)) return true;
        }
      }
    }
    return false;
  }

  void kvs(const JDoc& d, int64_t mapnode, uint32_t* first, uint32_t* count, bool labels) {
    *first = (uint32_t)b.kvs.size();
    *count = 0;
    if (mapnode < 0) return;
    const JNode& m = d.at((uint32_t)mapnode);
    if (!is_str_map(d, m)) return;  // NestedStringMap error -> nil map
    std::vector<std::pair<std::string_view, std::string_view>> pairs;
    for (uint32_t c = m.first; c < m.first + m.count; c++) pairs.push_back({d.key(d.at(c)), d.sval(d.at(c))});
    std::sort(pairs.begin(), pairs.end());
    for (auto& p : pairs) {
      KV kv{};
      kv.k_off = str(p.first);
      kv.k_len = (uint32_t)p.first.size();
      kv.v_off = str(p.second);
      kv.v_len = (uint32_t)p.second.size();
      if (labels) {
        if (valid_label_key(std::string(p.first))) kv.k_len |= KV_VALID;
        if (valid_label_value(std::string(p.second))) kv.v_len |= KV_VALID;
      }
      b.kvs.push_back(kv);
    }
    *count = (uint32_t)pairs.size();
  }

  void add(const JDoc& d) {
    const JNode& root = d.at(d.root);
    Res r{};
    if (root.t != J_MAP) throw std::runtime_error("ingest: resource is not a JSON object");
    auto gs = [&](uint32_t m, const char* k) -> std::string_view {
      int64_t c = d.get(m, k);
      if (c < 0 || d.at((uint32_t)c).t != J_STR) return std::string_view();
      return d.sval(d.at((uint32_t)c));
    };
    std::string_view kind = gs(d.root, "kind"), apiv = gs(d.root, "apiVersion");
    int64_t md = d.get(d.root, "metadata");
    std::string_view name, ns;
    int64_t labels = -1, ann = -1;
    if (md >= 0 && d.at((uint32_t)md).t == J_MAP) {
      name = gs((uint32_t)md, "name");
      ns = gs((uint32_t)md, "namespace");
      labels = d.get((uint32_t)md, "labels");
      ann = d.get((uint32_t)md, "annotations");
    }
    r.kind = ps.lookup(kind);
    std::string_view grp, ver;
    if (!apiv.empty() && apiv != "/") {
      size_t c = std::count(apiv.begin(), apiv.end(), '/');
      if (c == 0) ver = apiv;
      else if (c == 1) { size_t i = apiv.find('/'); grp = apiv.substr(0, i); ver = apiv.substr(i + 1); }
    }
    r.group = ps.lookup(grp);
    r.version = ps.lookup(ver);
    r.name_off = str(name);
    r.name_len = (uint32_t)name.size();
    bool isns = kind == "Namespace";
    std::string_view nsm = isns ? name : ns;
    r.ns_off = str(nsm);
    r.ns_len = (uint32_t)nsm.size();
    if (isns) r.flags |= RF_KIND_NAMESPACE;
    if (kind.empty()) r.flags |= RF_KIND_EMPTY;
    kvs(d, labels, &r.labels_first, &r.labels_count, true);
    kvs(d, ann, &r.annot_first, &r.annot_count, false);
    std::string nss(ns);
    auto it = ns_index.find(nss);
    if (it == ns_index.end()) {
      it = ns_index.emplace(nss, (uint32_t)b.namespaces.size()).first;
      b.namespaces.push_back(nss);
    }
    r.ns_index = it->second;
    if (bad_meta(d)) r.flags |= RF_BAD_META;
    if (d.strs.find("conditional anchor mismatch") != std::string::npos ||
        d.strs.find("global anchor mismatch") != std::string::npos)
      r.flags |= RF_MAGIC;
    uint32_t slot = (uint32_t)b.nodes.size();
    b.nodes.emplace_back();
    r.root = slot;
    fill(d, d.root, 0, slot, KEY_NONE);
    b.res.push_back(r);
  }
};

}  // namespace

void ingest_resources(const PolicySet& ps, const char* json, size_t len, const char* ns_labels_json, Batch* b) {
  Ingest in(ps, *b);
  parse_json_stream(json, len, NUM_UNSTRUCTURED, [&](const JDoc& d) { in.add(d); });
  // namespace labels (CLI --values-file namespaceSelector map / cluster namespaces)
  b->ns_labels.assign(b->namespaces.size(), {});
  if (ns_labels_json && *ns_labels_json) {
    JDoc d;
    parse_json(ns_labels_json, strlen(ns_labels_json), NUM_FLOAT, &d);
    const JNode& r = d.at(d.root);
    if (r.t == J_MAP) {
      for (uint32_t c = r.first; c < r.first + r.count; c++) {
        std::string nsn(d.key(d.at(c)));
        auto it = in.ns_index.find(nsn);
        if (it == in.ns_index.end()) continue;
        const JNode& m = d.at(c);
        if (m.t != J_MAP) continue;
        for (uint32_t g = m.first; g < m.first + m.count; g++)
          if (d.at(g).t == J_STR) b->ns_labels[it->second].push_back({std::string(d.key(d.at(g))), std::string(d.sval(d.at(g)))});
      }
    }
  }
  // namespaceSelector outcome per (namespace, selector): batch constant
  uint32_t nsel = (uint32_t)ps.nsselectors.size();
  b->ns_words = std::max<uint32_t>(1, (nsel + 31) / 32);
  b->ns_bits.assign((size_t)b->namespaces.size() * b->ns_words, 0);
  for (size_t n = 0; n < b->namespaces.size(); n++)
    for (uint32_t s = 0; s < nsel; s++)
      if (selector_eval_host(ps.nsselectors[s], b->ns_labels[n]) == 1) b->ns_bits[n * b->ns_words + s / 32] |= 1u << (s % 32);
  // word-granular readers may touch up to 8 bytes past the last string
  b->strs.append(16, '\0');
  b->bytes_referenced = b->nodes.size() * sizeof(Node) + b->vals.size() * sizeof(Val) + b->res.size() * sizeof(Res) +
                        b->kvs.size() * sizeof(KV) + b->strs.size();
}

}  // namespace kvh
