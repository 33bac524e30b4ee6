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
#include <atomic>

#include <emmintrin.h>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <thread>
#include <sys/mman.h>
#include <unordered_map>

#include "kvinternal.hpp"

namespace kvh {

HostMem g_hostmem;

using namespace kv;

namespace {

struct Ingest {
  const PolicySet& ps;
  Batch& b;
  // Interning tables (open addressing, linear probing, keyed by a 64-bit hash of the bytes;
  // a hit is confirmed against the bytes already stored in the heap / the value record, so
  // no key string is built or kept per lookup)
  struct Probe {
    struct Slot {
      uint64_t h;    // 0 = empty
      uint32_t id;   // entry id
      uint32_t aux;  // entry length (string heap) or 0
    };
    std::vector<Slot, ThpAlloc<Slot>> t;  // one cache line holds 4 slots: a miss costs one line
    size_t n = 0;
    void init(size_t cap) {
      size_t c = 64;
      while (c < cap * 2) c <<= 1;
      t.assign(c, Slot{0, 0, 0});
      n = 0;
    }
    // id of the entry with hash hv that eq(slot) confirms, -1 when absent
    template <class Eq>
    int64_t find(uint64_t hv, Eq eq) const {
      const size_t m = t.size() - 1;
      for (size_t i = hv & m;; i = (i + 1) & m) {
        if (t[i].h == 0) return -1;
        if (t[i].h == hv && eq(t[i])) return t[i].id;
      }
    }
    void insert(uint64_t hv, uint32_t v, uint32_t aux = 0) {
      if ((n + 1) * 2 > t.size()) grow();
      const size_t m = t.size() - 1;
      size_t i = hv & m;
      while (t[i].h != 0) i = (i + 1) & m;
      t[i] = Slot{hv, v, aux};
      n++;
    }
    void grow() {
      std::vector<Slot, ThpAlloc<Slot>> o;
      o.swap(t);
      t.assign(o.size() * 2, Slot{0, 0, 0});
      n = 0;
      for (const Slot& x : o)
        if (x.h) insert(x.h, x.id, x.aux);
    }
  };
  static uint64_t hash_bytes(const void* p, size_t len, uint64_t seed) {
    if (len <= 16) {  // (most keys and values: two multiplies instead of the word loop)
      uint64_t w0 = 0, w1 = 0;
      if (len) memcpy(&w0, p, len < 8 ? len : 8);  // (an empty view may carry a null pointer)
      if (len > 8) memcpy(&w1, (const uint8_t*)p + 8, len - 8);
      uint64_t h = (w0 * 0x9E3779B97F4A7C15ull) ^ (w1 * 0xC2B2AE3D27D4EB4Full) ^ ((len + 1) * 0x165667B19E3779F9ull) ^
                   (seed * 0x27D4EB2F165667C5ull);
      h ^= h >> 32;
      h *= 0xD6E8FEB86659FD93ull;
      h ^= h >> 29;
      return h ? h : 1;
    }
    const uint8_t* s = (const uint8_t*)p;  // FNV-1a 64 over 8-byte words, then a final mix
    uint64_t h = 1469598103934665603ull ^ seed ^ (len * 0x9E3779B97F4A7C15ull);
    size_t i = 0;
    for (; i + 8 <= len; i += 8) {
      uint64_t w;
      memcpy(&w, s + i, 8);
      h = (h ^ w) * 1099511628211ull;
      h ^= h >> 29;
    }
    for (; i < len; i++) h = (h ^ s[i]) * 1099511628211ull;
    h ^= h >> 32;
    h *= 0xD6E8FEB86659FD93ull;
    h ^= h >> 32;
    return h ? h : 1;
  }
  Probe str_off;  // string heap offsets (id = offset, aux = length; confirmed against the heap)
  // scalars: a slot carries what a node needs (id, e_off, e_len | NC_* flags, position
  // classes so far) and the value's first 8 bytes, so a hit is confirmed and answered from
  // the slot alone (strings longer than 8 bytes compare their tail in the heap)
  struct VSlot {
    uint64_t h;     // 0 = empty
    uint64_t key8;  // INT / FLOAT bits, BOOL, or a string's first 8 bytes (zero padded)
    uint32_t id, e_off, c, cls, type;
  };
  std::vector<VSlot, ThpAlloc<VSlot>> vtab;
  size_t vn = 0;
  Probe dict;     // the policy set's key dictionary (id = static key id)
  Probe dyn_key;  // batch-local key ids (id = index into b.dyn_keys)
  Probe ns_probe, nsm_probe, lset_probe, aset_probe;  // namespaces, match inputs (confirmed by key)
  uint32_t nstatic;
  std::vector<std::vector<uint32_t>> slot_ids;  // per trie node: key ids of its slots
  std::vector<Probe> slot_tab;                  // per trie node: slot of a key (built on first use)

  bool meta_rules = false;  // some rule reads labels / annotations through ExpandInMetadata (RR_META_*)
  Ingest(const PolicySet& p, Batch& bb) : ps(p), b(bb), nstatic((uint32_t)p.keys.size()), slot_ids(p.trie.nodes.size()),
                                          slot_tab(p.trie.nodes.size()) {
    for (const RuleRec& rr : p.rules) meta_rules |= meta_bad_flags(rr.flags) != 0u;
    str_off.init(1 << 14);
    vtab.assign(1 << 15, VSlot{});
    dict.init(p.keys.size());
    for (uint32_t i = 0; i < (uint32_t)p.keys.size(); i++) dict.insert(hash_bytes(p.keys[i].data(), p.keys[i].size(), 'K'), i);
    dyn_key.init(64);
    ns_probe.init(1024);
    nsm_probe.init(1024);
    lset_probe.init(1024);
    aset_probe.init(1024);
    // offset 0 holds "0": convertNumberToString(nil) for the device glob (kvkernel.hip atom_eval)
    str("0");
  }

  uint32_t str(std::string_view s) {
    const uint64_t hv = hash_bytes(s.data(), s.size(), 0x5354u);
    const int64_t e = str_off.find(hv, [&](const Probe::Slot& x) {
      return x.aux == s.size() && memcmp(b.strs.data() + x.id, s.data(), s.size()) == 0;
    });
    if (e >= 0) return (uint32_t)e;
    // 4-byte aligned: the device glob compares whole words (kvkernel.hip seg_at)
    while (b.strs.size() & 3) b.strs.push_back('\0');
    uint32_t off = (uint32_t)b.strs.size();
    b.strs.append(s.data(), s.size());
    str_off.insert(hv, off, (uint32_t)s.size());
    return off;
  }

  // static key id of k (KEY_NONE when the policy set does not know it)
  uint32_t lookup(std::string_view k) const {
    const int64_t id = dict.find(hash_bytes(k.data(), k.size(), 'K'), [&](const Probe::Slot& x) { return ps.keys[x.id] == k; });
    return id >= 0 ? (uint32_t)id : KEY_NONE;
  }

  uint32_t key_of(std::string_view k) {
    uint32_t id = lookup(k);
    if (id != KEY_NONE) return id;
    const uint64_t hv = hash_bytes(k.data(), k.size(), 'D');
    const int64_t hit = dyn_key.find(hv, [&](const Probe::Slot& x) { return b.dyn_keys[x.id] == k; });
    if (hit >= 0) return nstatic + (uint32_t)hit;
    uint32_t nid = nstatic + (uint32_t)b.dyn_keys.size();
    if (nid >= KEY_NONE28) throw std::runtime_error("ingest: too many distinct keys in one batch");
    dyn_key.insert(hv, (uint32_t)b.dyn_keys.size());
    b.dyn_keys.emplace_back(k);
    return nid;
  }

  // id of `k` among `keys` (interned through `pr`), appending it when new
  static uint32_t intern(Probe& pr, std::vector<std::string>& keys, std::string_view k, bool* fresh) {
    const uint64_t hv = hash_bytes(k.data(), k.size(), 'I');
    const int64_t hit = pr.find(hv, [&](const Probe::Slot& x) { return keys[x.id] == k; });
    *fresh = hit < 0;
    if (hit >= 0) return (uint32_t)hit;
    const uint32_t id = (uint32_t)keys.size();
    keys.emplace_back(k);
    pr.insert(hv, id);
    return id;
  }

  // new Val for scalar n (sv: its bytes when a string)
  uint32_t val_new(const JNode& n, std::string_view sv) {
    Val v{};
    // e: the validateString form; num: the number-with-string form (same bytes except for
    // floats, where they are FormatFloat 'E' and %f)
    std::string_view e, num;
    std::string fe, fnum;
    char ibuf[24];
    bool nvalid = true;
    switch (n.t) {
      case J_BOOL:
        v.type = NT_BOOL;
        e = n.b ? "true" : "false";
        nvalid = false;
        v.flags |= n.b ? VF_BOOLV : VF_NILLIKE;
        break;
      case J_INT: {
        v.type = NT_INT;
        v.i = n.i;
        const int len = snprintf(ibuf, sizeof ibuf, "%lld", (long long)n.i);
        e = num = std::string_view(ibuf, (size_t)len);
        if (n.i == 0) v.flags |= VF_NILLIKE;
        break;
      }
      case J_FLOAT:
        v.type = NT_FLOAT;
        v.f = n.f;
        fe = go_format_E(n.f);
        fnum = go_format_f6(n.f);
        e = fe;
        num = fnum;
        if (n.f == 0.0) v.flags |= VF_NILLIKE;
        break;
      default: {
        v.type = NT_STR;
        e = num = sv;
        double f;
        if (go_parse_float(sv, &f)) { v.flags |= VF_PF_OK; v.f = f; }
        if (sv.empty()) v.flags |= VF_NILLIKE;
        break;
      }
    }
    v.e_off = str(e);
    v.e_len = (uint32_t)e.size();
    const bool e_ascii = utf8_ascii(e);
    if (e_ascii) v.flags |= VF_ASCII_E;
    if (nvalid) {
      v.flags |= VF_N_VALID;
      const bool same = num.data() == e.data();
      v.n_off = same ? v.e_off : str(num);
      v.n_len = (uint32_t)num.size();
      if (same ? e_ascii : utf8_ascii(num)) v.flags |= VF_ASCII_N;
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
    return id;
  }

  void vgrow() {
    std::vector<VSlot, ThpAlloc<VSlot>> o(vtab.size() * 2, VSlot{});
    o.swap(vtab);
    const size_t m = vtab.size() - 1;
    for (const VSlot& x : o)
      if (x.h) {
        size_t i = x.h & m;
        while (vtab[i].h) i = (i + 1) & m;
        vtab[i] = x;
      }
  }

  // ---------------------------------------------------------------- wave-group layout
  // Resources are laid out in groups of KV_LANES (one wavefront): the group's
  // nodes form rows of KV_LANES cells, cell (row, lane) = node of resource
  // 64*g + lane. Rows follow the union shape of the group's projected trees
  // (slot-addressed maps share a fixed slot block; arrays get max-length element
  // blocks; keep-all maps max-count blocks), so one logical position has the
  // same row in every lane and the device's uniform-pc walk reads whole rows
  // (coalesced) instead of 64 scattered nodes. Node index = row * 64 + lane.
  struct Shape {
    int32_t t = -1;            // projection-trie node (-1: leaf-only)
    uint32_t row = 0;          // row within the group
    bool has_map = false, has_arr = false, keep_all = false;
    uint32_t map_row = 0, arr_row = 0;
    // map block (slot-addressed: one per slot key; keep-all: max count) and array block (max
    // length): the first nk / ne entries; the vectors are pools kept across groups
    uint32_t nk = 0, ne = 0;
    std::vector<Shape> kids;
    std::vector<Shape> elems;
    void reset(int32_t trie) {
      t = trie;
      row = map_row = arr_row = 0;
      has_map = has_arr = keep_all = false;
      nk = ne = 0;
    }
  };
  Shape shape_root;  // the current group's shape (reused)
  // slot of each map child at a slot-addressed trie node, found by unite and reused by put:
  // per lane, indexed by the child's node index in its document
  std::vector<int32_t> jslot[KV_LANES];
  std::vector<uint32_t> kids_sorted;  // (reused)

  // slot of key k in slot-addressed trie node t (a hash table of its slot keys, built on
  // first use; no string built per lookup), -1 when the key is not projected
  int32_t slot_of(int32_t t, std::string_view k) {
    const Trie::N& tn = ps.trie.nodes[t];
    Probe& tab = slot_tab[t];
    if (tab.t.empty()) {
      tab.init(tn.slot_keys.size());
      for (uint32_t i = 0; i < (uint32_t)tn.slot_keys.size(); i++)
        tab.insert(hash_bytes(tn.slot_keys[i].data(), tn.slot_keys[i].size(), 'S'), i);
    }
    return (int32_t)tab.find(hash_bytes(k.data(), k.size(), 'S'),
                             [&](const Probe::Slot& x) { return tn.slot_keys[x.id] == k; });
  }

  // slot of the key at child position `pos` of a slot-addressed map at trie node t, remembered
  // per (node, position): documents of one kind list their keys in the same order, so most
  // lookups are one compare against the previous document's key instead of a hash and probe
  struct PosSlot {
    std::string key;
    int32_t slot = -2;  // -2: empty
  };
  std::vector<std::vector<PosSlot>> pos_cache;
  int32_t slot_at(int32_t t, uint32_t pos, std::string_view k) {
    if (pos >= 64u) return slot_of(t, k);
    if (pos_cache.size() <= (size_t)t) pos_cache.resize(ps.trie.nodes.size());
    std::vector<PosSlot>& pc = pos_cache[t];
    if (pc.size() <= pos) pc.resize(pos + 1);
    PosSlot& e = pc[pos];
    if (e.slot != -2 && e.key == k) return e.slot;
    e.key.assign(k.data(), k.size());
    e.slot = slot_of(t, k);
    return e.slot;
  }

  // sorted-children buffers of the keep-all maps being walked, one per nesting depth (a
  // deque: growing it keeps the outer frames' references valid)
  std::deque<std::vector<uint32_t>> ch_pool;
  size_t ch_depth = 0;
  std::vector<uint32_t>& child_buf() {
    if (ch_pool.size() <= ch_depth) ch_pool.emplace_back();
    return ch_pool[ch_depth++];
  }

  void sorted_children(const JDoc& d, const JNode& n, std::vector<uint32_t>* out) {
    out->clear();
    for (uint32_t c = n.first; c < n.first + n.count; c++) out->push_back(c);
    std::sort(out->begin(), out->end(), [&](uint32_t x, uint32_t y) { return d.key(d.at(x)) < d.key(d.at(y)); });
  }

  void unite(Shape& s, const JDoc& d, uint32_t jn, std::vector<int32_t>& js) {
    const JNode& n = d.at(jn);
    if (n.t == J_MAP) {
      if (s.t < 0) return;
      const Trie::N& tn = ps.trie.nodes[s.t];
      if (!s.has_map) {
        s.has_map = true;
        s.keep_all = tn.keep_all;
        if (!tn.keep_all) {
          const uint32_t K = (uint32_t)tn.slot_keys.size();
          if (s.kids.size() < K) s.kids.resize(K);
          for (uint32_t i = 0; i < K; i++) s.kids[i].reset((int32_t)tn.kids.at(tn.slot_keys[i]));
          s.nk = K;
        }
      }
      if (tn.keep_all) {
        if (s.nk < n.count) {  // children leaf-only (t = -1)
          if (s.kids.size() < n.count) s.kids.resize(n.count);
          for (uint32_t i = s.nk; i < n.count; i++) s.kids[i].reset(-1);
          s.nk = n.count;
        }
        std::vector<uint32_t>& ch = child_buf();
        sorted_children(d, n, &ch);
        for (size_t i = 0; i < ch.size(); i++) unite(s.kids[i], d, ch[i], js);
        ch_depth--;
      } else {
        for (uint32_t c = n.first; c < n.first + n.count; c++) {
          const int32_t si = slot_at(s.t, c - n.first, d.key(d.at(c)));
          js[c] = si;
          if (si >= 0) unite(s.kids[si], d, c, js);
        }
      }
    } else if (n.t == J_ARR) {
      s.has_arr = true;
      const int32_t et = s.t >= 0 ? ps.trie.nodes[s.t].elem : -1;
      if (s.ne < n.count) {
        if (s.elems.size() < n.count) s.elems.resize(n.count);
        for (uint32_t j = s.ne; j < n.count; j++) s.elems[j].reset(et);
        s.ne = n.count;
      }
      for (uint32_t j = 0; j < n.count; j++) unite(s.elems[j], d, n.first + j, js);
    }
  }

  void assign(Shape& s, uint32_t* next) {
    if (s.has_map) {
      s.map_row = *next;
      *next += s.nk;
      for (uint32_t i = 0; i < s.nk; i++) s.kids[i].row = s.map_row + i;
    }
    if (s.has_arr) {
      s.arr_row = *next;
      *next += s.ne;
      for (uint32_t j = 0; j < s.ne; j++) s.elems[j].row = s.arr_row + j;
    }
    for (uint32_t i = 0; i < s.nk; i++) assign(s.kids[i], next);
    for (uint32_t j = 0; j < s.ne; j++) assign(s.elems[j], next);
  }

  Node scalar(const JDoc& d, const JNode& n, uint32_t type, uint32_t key, int32_t pos) {
    uint64_t k8 = 0, hv;
    std::string_view sv;
    switch (n.t) {
      case J_BOOL: k8 = n.b ? 1 : 0; hv = hash_bytes(&k8, 8, 'b'); break;
      case J_INT: memcpy(&k8, &n.i, 8); hv = hash_bytes(&k8, 8, 'i'); break;
      case J_FLOAT: memcpy(&k8, &n.f, 8); hv = hash_bytes(&k8, 8, 'f'); break;
      default:
        sv = d.sval(n);
        memcpy(&k8, sv.data(), std::min<size_t>(8, sv.size()));
        hv = hash_bytes(sv.data(), sv.size(), 's');
        break;
    }
    const uint32_t bit = kv_tcls(pos);
    const size_t m = vtab.size() - 1;
    size_t i = hv & m;
    for (;; i = (i + 1) & m) {
      VSlot& x = vtab[i];
      if (x.h == 0) break;
      if (x.h != hv || x.key8 != k8 || x.type != type) continue;
      if (type == NT_STR && ((x.c & NC_LEN_MASK) != sv.size() ||
                             (sv.size() > 8 && memcmp(b.strs.data() + x.e_off + 8, sv.data() + 8, sv.size() - 8) != 0)))
        continue;
      if (!(x.cls & bit)) {
        x.cls |= bit;
        b.vals[x.id].cls |= bit;
      }
      return Node{(key & KEY_NONE28) << 4 | type, x.id, x.e_off, x.c};
    }
    const uint32_t vid = val_new(n, sv);
    Val& v = b.vals[vid];
    v.cls |= bit;
    if (v.e_len > NC_LEN_MASK) throw std::runtime_error("ingest: string value too long");
    uint32_t c = v.e_len;
    if (v.flags & VF_ASCII_E) c |= NC_ASCII_E;
    if (v.flags & VF_BOOLV) c |= NC_BOOLV;
    if (v.flags & VF_NILLIKE) c |= NC_NILLIKE;
    vtab[i] = VSlot{hv, k8, vid, v.e_off, c, v.cls, type};
    if (++vn * 2 > vtab.size()) vgrow();
    return Node{(key & KEY_NONE28) << 4 | type, vid, v.e_off, c};
  }

  uint64_t base_row = 0;  // first row of the current group
  const bool check_cells = getenv("KVGPU_CHECK_CELLS") != nullptr;
  // the current group's padded rows (reused, cache-resident); packed into b.tcells at its end
  std::vector<Node> gcells;
  std::vector<uint64_t> gmask;  // lanes written per row of the group
  void set_cell(uint32_t row, uint32_t lane, const Node& v) {
    gcells[(size_t)row * KV_LANES + lane] = v;
    gmask[row] |= 1ull << lane;
  }

  // Write lane's value at shape position s (key = key id in the parent map)
  // pos: position class id of this value (kv_pos_*; Val::cls)
  void put(const Shape& s, const JDoc& d, uint32_t jn, uint32_t lane, uint32_t key, int32_t pos) {
    const std::vector<int32_t>& js = jslot[lane];
    const JNode& n = d.at(jn);
    Node out{(key & KEY_NONE28) << 4 | NT_NULL, 0, 0, 0};
    switch (n.t) {
      case J_NULL: break;
      case J_BOOL: out = scalar(d, n, NT_BOOL, key, pos); break;
      case J_INT: out = scalar(d, n, NT_INT, key, pos); break;
      case J_FLOAT: out = scalar(d, n, NT_FLOAT, key, pos); break;
      case J_STR: out = scalar(d, n, NT_STR, key, pos); break;
      case J_MAP: {
        out.kt = (key & KEY_NONE28) << 4 | NT_MAP;
        if (s.t < 0) break;
        const Trie::N& tn = ps.trie.nodes[s.t];
        out.a = (uint32_t)(base_row + s.map_row);
        if (tn.keep_all) {
          out.b = n.count;
          std::vector<uint32_t>& ch = child_buf();
          sorted_children(d, n, &ch);
          for (size_t i = 0; i < ch.size(); i++) put(s.kids[i], d, ch[i], lane, key_of(d.key(d.at(ch[i]))), -1);
          ch_depth--;
        } else {
          const uint32_t K = (uint32_t)tn.slot_keys.size();
          out.b = K;
          auto& ids = slot_ids[s.t];
          for (uint32_t i = (uint32_t)ids.size(); i < K; i++) ids.push_back(key_of(tn.slot_keys[i]));
          for (uint32_t i = 0; i < K; i++) set_cell(s.map_row + i, lane, Node{(ids[i] & KEY_NONE28) << 4 | NT_ABSENT, 0, 0, 0});
          for (uint32_t c = n.first; c < n.first + n.count; c++) {
            const int32_t si = js[c];
            if (si >= 0) put(s.kids[si], d, c, lane, ids[si], s.kids[si].t);
          }
        }
        break;
      }
      case J_ARR: {
        out.kt = (key & KEY_NONE28) << 4 | NT_ARR;
        out.a = (uint32_t)(base_row + s.arr_row);
        out.b = n.count;
        for (uint32_t j = 0; j < n.count; j++) put(s.elems[j], d, n.first + j, lane, KEY_NONE, kv_pos_elem(pos, s.t));
        break;
      }
    }
    set_cell(s.row, lane, out);
  }

  std::vector<JDoc> group;
  uint32_t group_n = 0;
  size_t expected_res = 0;  // resources this Ingest will take (0: unknown)

  void flush_group() {
    if (group_n == 0) return;
    Shape& root = shape_root;
    root.reset(0);
    for (uint32_t l = 0; l < group_n; l++) {
      if (jslot[l].size() < group[l].nodes.size()) jslot[l].resize(group[l].nodes.size());
      unite(root, group[l], group[l].root, jslot[l]);
    }
    uint32_t rows = 1;
    root.row = 0;
    assign(root, &rows);
    base_row = b.n_rows;
    b.n_rows += rows;
    if (b.n_rows * KV_LANES >= 0xFFFFFFF0ull) throw std::runtime_error("ingest: batch too large for 32-bit node indices");
    if (gcells.size() < (size_t)rows * KV_LANES) gcells.resize((size_t)rows * KV_LANES);
    gmask.assign(rows, 0);
    for (uint32_t l = 0; l < group_n; l++) {
      put(root, group[l], group[l].root, l, KEY_NONE, 0);
      b.res[b.res.size() - group_n + l].root = (uint32_t)base_row;
    }
    // capacity for the rest of the part from the cells per group so far (+1/8), instead of
    // the vector's doubling (each doubling copies every cell written so far)
    const size_t want = b.tcells.size() + gcells.size();
    if (want > b.tcells.capacity()) {
      size_t cap = want;
      if (expected_res > b.res.size())
        cap = std::max(cap, (size_t)((double)want / (double)b.res.size() * (double)expected_res * 1.125));
      b.tcells.reserve(std::max(cap, b.tcells.capacity() * 2));
      if (expected_res > b.res.size()) {  // values, strings and headers grow in proportion
        const double f = (double)expected_res / (double)b.res.size() * 1.125;
        if (b.vals.capacity() < (size_t)(b.vals.size() * f)) b.vals.reserve((size_t)(b.vals.size() * f));
        if (b.strs.capacity() < (size_t)(b.strs.size() * f)) b.strs.reserve((size_t)(b.strs.size() * f));
        if (b.res.capacity() < expected_res) b.res.reserve(expected_res);
      }
      b.rmask.reserve(std::max<size_t>(b.rmask.capacity() * 2, cap / KV_LANES + rows));
      b.rwide.reserve(std::max<size_t>(b.rwide.capacity() * 2, cap / KV_LANES + rows));
      b.roff.reserve(std::max<size_t>(b.roff.capacity() * 2, cap / KV_LANES + rows));
    }
    // packed rows: the non-zero cells of each row in their transfer form (kv_layout.h), its
    // lane mask, wide-lane mask and first 8-byte unit
    size_t pc = b.tcells.size(), nw = 0;
    for (uint32_t row = 0; row < rows; row++) nw += (size_t)__builtin_popcountll(gmask[row]);
    b.tcells.resize(pc + 2 * nw);
    const size_t r0 = b.rmask.size();
    b.rmask.resize(r0 + rows);
    b.rwide.resize(r0 + rows);
    b.roff.resize(r0 + rows);
    uint64_t* out = b.tcells.data();
    uint64_t used = 0;
    for (uint32_t row = 0; row < rows; row++) {
      const Node* c = &gcells[(size_t)row * KV_LANES];
      uint64_t m = 0, wm = 0;
      b.roff[r0 + row] = (uint32_t)pc;
      for (uint64_t w = gmask[row]; w; w &= w - 1) {
        const uint32_t l = (uint32_t)__builtin_ctzll(w);
        if (c[l].kt | c[l].a | c[l].b | c[l].c) {
          m |= 1ull << l;
          used++;
          uint32_t hi;
          if (cell_narrow(c[l], base_row + row, b.vals.data(), &hi)) {
            if (check_cells) {  // KVGPU_CHECK_CELLS: the 8-byte form rebuilds the Node exactly
              const Node r = cell_widen(c[l].kt, hi, base_row + row, b.vals.data());
              if (memcmp(&r, &c[l], sizeof(Node)) != 0) throw std::runtime_error("ingest: transfer cell does not round-trip");
            }
            out[pc++] = (uint64_t)c[l].kt | (uint64_t)hi << 32;
          } else {
            wm |= 1ull << l;
            memcpy(&out[pc], &c[l], sizeof(Node));
            pc += 2;
          }
        }
      }
      b.rmask[r0 + row] = m;
      b.rwide[r0 + row] = wm;
    }
    b.tcells.resize(pc);
    if (b.tcells.size() >= 0xFFFFFFF0ull) throw std::runtime_error("ingest: batch too large for 32-bit cell offsets");
    b.cells_used += used;
    group_n = 0;
  }

  static bool is_str_map(const JDoc& d, const JNode& m) {
    if (m.t != J_MAP) return false;
    for (uint32_t c = m.first; c < m.first + m.count; c++)
      if (d.at(c).t != J_STR) return false;
    return true;
  }

  // ExpandInMetadata panics on non-map metadata / labels, non-string label values
  // (wildcards.go:69-139, per tag the pattern reads): RF_BAD_LABELS / RF_BAD_ANN. Any
  // `metadata` key at any depth counts (the pattern's expansion sites may be nested).
  uint32_t bad_meta(const JDoc& d) {
    uint32_t f = 0;
    for (const JNode& m : d.nodes) {
      if (m.t != J_MAP) continue;
      for (uint32_t c = m.first; c < m.first + m.count; c++) {
        const JNode& ch = d.at(c);
        if (d.key(ch) != "metadata" || ch.t == J_NULL) continue;
        if (ch.t != J_MAP) return RF_BAD_LABELS | RF_BAD_ANN;
        for (uint32_t g = ch.first; g < ch.first + ch.count; g++) {
          const JNode& t = d.at(g);
          std::string_view k = d.key(t);
          if ((k == "labels" || k == "annotations") && t.t != J_NULL && !is_str_map(d, t))
            f |= k == "labels" ? RF_BAD_LABELS : RF_BAD_ANN;
        }
      }
    }
    return f;
  }

  // Interned label / annotation list of a resource: identical lists (same pairs, same
  // validity bits) share one KVSet, so the match tables evaluate a selector or an
  // annotation filter once per distinct list.
  std::vector<std::pair<std::string_view, std::string_view>> pairs;  // (reused)
  std::string kbuf;                                                  // (reused)
  uint32_t kvset(const JDoc& d, int64_t mapnode, bool labels) {
    pairs.clear();
    if (mapnode >= 0) {
      const JNode& m = d.at((uint32_t)mapnode);
      if (is_str_map(d, m))  // else NestedStringMap error -> nil map
        for (uint32_t c = m.first; c < m.first + m.count; c++) pairs.push_back({d.key(d.at(c)), d.sval(d.at(c))});
    }
    std::sort(pairs.begin(), pairs.end());
    std::string& key = kbuf;
    key.clear();
    for (auto& p : pairs) {
      key.append(p.first.data(), p.first.size());
      key.push_back('\0');
      key.append(p.second.data(), p.second.size());
      key.push_back('\0');
    }
    auto& sets = labels ? b.lsets : b.asets;
    bool fresh = false;
    const uint32_t id = intern(labels ? lset_probe : aset_probe, labels ? b.lset_keys : b.aset_keys, key, &fresh);
    if (!fresh) return id;
    KVSet set{(uint32_t)b.kvs.size(), (uint32_t)pairs.size()};
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
    sets.push_back(set);
    return id;
  }

  uint32_t nsm(std::string_view s) {
    bool fresh = false;
    const uint32_t id = intern(nsm_probe, b.nsm_keys, s, &fresh);
    if (fresh) b.nsms.push_back(StrRef{str(s), (uint32_t)s.size()});
    return id;
  }

  void add(const JDoc& d) {  // per-resource header (match/exclude inputs)
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
    r.kind = lookup(kind);
    std::string_view grp, ver;
    if (!apiv.empty() && apiv != "/") {
      size_t c = std::count(apiv.begin(), apiv.end(), '/');
      if (c == 0) ver = apiv;
      else if (c == 1) { size_t i = apiv.find('/'); grp = apiv.substr(0, i); ver = apiv.substr(i + 1); }
    }
    r.group = lookup(grp);
    r.version = lookup(ver);
    r.name_off = str(name);
    r.name_len = (uint32_t)name.size();
    if (utf8_ascii(name)) r.flags |= RF_NAME_ASCII;
    bool isns = kind == "Namespace";
    r.nsm = nsm(isns ? name : ns);
    if (isns) r.flags |= RF_KIND_NAMESPACE;
    if (kind.empty()) r.flags |= RF_KIND_EMPTY;
    r.lset = kvset(d, labels, true);
    r.aset = kvset(d, ann, false);
    bool fresh = false;
    r.ns_index = intern(ns_probe, b.namespaces, ns, &fresh);
    if (meta_rules)  // (the flags only route rules whose ExpandInMetadata sites read labels / annotations)
      if (const uint32_t bm = bad_meta(d)) r.flags |= RF_BAD_META | bm;
    // the anchor-mismatch error substrings (common/anchorKey.go:12-19): both end in
    // "anchor mismatch", so one search finds any candidate
    if (memmem(d.strs.data(), d.strs.size(), "anchor mismatch", 15) &&
        (d.strs.find("conditional anchor mismatch") != std::string::npos ||
         d.strs.find("global anchor mismatch") != std::string::npos))
      r.flags |= RF_MAGIC;
    b.res.push_back(r);  // root row assigned by flush_group
    // pattern variables: every distinct (string, path) resolved on this resource (kvvars.cpp)
    for (const auto& vk : ps.vkeys) {
      std::string o = resolve_var_string(vk.first, vk.second, d);
      auto it = b.vout_id.find(o);
      if (it == b.vout_id.end()) {
        it = b.vout_id.emplace(o, (uint32_t)b.vout_tab.size()).first;
        b.vout_tab.push_back(std::move(o));
      }
      b.vout.push_back(it->second);
    }
  }

  void take(JDoc& d) {
    if (group.size() < KV_LANES) group.resize(KV_LANES);
    add(d);
    std::swap(group[group_n++], d);
    if (group_n == KV_LANES) flush_group();
  }
};

}  // namespace

void* thp_alloc(size_t bytes) {
  constexpr size_t kHuge = 2u << 20;
  void* p = nullptr;
  if (bytes >= kHuge) {
    const size_t sz = (bytes + kHuge - 1) & ~(kHuge - 1);
    p = aligned_alloc(kHuge, sz);
    if (p) (void)madvise(p, sz, MADV_HUGEPAGE);
  } else {
    p = malloc(bytes ? bytes : 1);
  }
  if (!p) throw std::bad_alloc();
  return p;
}

namespace {

unsigned ingest_threads() {
  if (const char* e = getenv("KVGPU_INGEST_THREADS")) return (unsigned)std::max(1, atoi(e));
  return std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

// Start offsets of the top-level values of a JSON value stream (NDJSON, one or
// more values per line). The stream is cut at newlines followed by '{' and each
// piece is scanned in parallel (string / escape / depth tracking); a cut that
// fell inside a value (pretty-printed input) shows up as a piece not ending at
// depth 0, and the caller then ingests serially.
bool scan_values(const char* p, size_t n, unsigned T, std::vector<size_t>* starts) {
  std::vector<size_t> cut{0};
  for (unsigned k = 1; k < T; k++) {
    size_t x = std::max(cut.back() + 1, n / T * k);
    while (x < n && !(p[x - 1] == '\n' && p[x] == '{')) x++;
    if (x >= n) break;
    cut.push_back(x);
  }
  cut.push_back(n);
  const size_t P = cut.size() - 1;
  std::vector<std::vector<size_t>> part(P);
  std::vector<char> ok(P, 0);
  std::vector<std::thread> th;
  for (size_t k = 0; k < P; k++)
    th.emplace_back([&, k]() {
      // byte classes: 0 plain, 1 quote, 2 backslash, 3 open, 4 close
      static const auto cls = []() {
        std::array<uint8_t, 256> t{};
        t['"'] = 1; t['\\'] = 2; t['{'] = 3; t['['] = 3; t['}'] = 4; t[']'] = 4;
        return t;
      }();
      int depth = 0;
      const uint8_t* q = (const uint8_t*)p;
      size_t i = cut[k];
      const size_t e = cut[k + 1];
      while (i < e) {
        const uint8_t c = cls[q[i]];
        if (c == 0) { i++; continue; }
        if (c == 1) {  // string: skip to the closing quote
          if (depth == 0) return;  // top-level scalar: not a resource stream
          i++;
          while (i < e) {
            const uint8_t d = cls[q[i]];
            if (d == 1) break;
            i += d == 2 ? 2 : 1;
          }
          if (i >= e) return;  // unterminated string in this piece
          i++;
          continue;
        }
        if (c == 3) {
          if (depth == 0) part[k].push_back(i);
          depth++;
        } else if (c == 4) {
          if (--depth < 0) return;
        }
        i++;
      }
      ok[k] = depth == 0;
    });
  for (auto& t : th) t.join();
  for (size_t k = 0; k < P; k++)
    if (!ok[k]) return false;
  for (auto& v : part) starts->insert(starts->end(), v.begin(), v.end());
  return true;
}

// Start offsets of the documents of NDJSON input, one object per line (the usual form of
// a resource dump): a memchr per line over parallel pieces, no byte-by-byte scan. The parse
// threads check that each document ends its line; any other form (pretty-printed objects,
// several values on a line) fails that check and goes through scan_values.
struct NotLines {};

bool split_lines(const char* p, size_t n, unsigned T, std::vector<size_t>* starts) {
  std::vector<size_t> cut{0};
  for (unsigned k = 1; k < T; k++) {
    const size_t x = std::max(cut.back(), n / T * k);
    const char* nl = x < n ? (const char*)memchr(p + x, '\n', n - x) : nullptr;
    if (!nl) break;
    cut.push_back((size_t)(nl - p) + 1);
  }
  cut.push_back(n);
  const size_t P = cut.size() - 1;
  std::vector<std::vector<size_t>> part(P);
  std::vector<char> ok(P, 1);
  std::vector<std::thread> th;
  for (size_t k = 0; k < P; k++)
    th.emplace_back([&, k]() {
      for (size_t q = cut[k], e = cut[k + 1]; q < e;) {
        while (q < e && (p[q] == ' ' || p[q] == '\t' || p[q] == '\r' || p[q] == '\n')) q++;
        if (q >= e) break;
        if (p[q] != '{') {
          ok[k] = 0;
          return;
        }
        part[k].push_back(q);
        const char* nl = (const char*)memchr(p + q, '\n', e - q);
        q = nl ? (size_t)(nl - p) + 1 : e;
      }
    });
  for (auto& t : th) t.join();
  for (size_t k = 0; k < P; k++)
    if (!ok[k]) return false;
  for (auto& v : part) starts->insert(starts->end(), v.begin(), v.end());
  return true;
}

// Concatenate per-thread batches (each a whole number of 64-resource wave
// groups, in input order): heaps, values, KV pairs and rows are appended with
// their offsets rebased; batch-local key ids and namespace indices are remapped
// onto tables built in thread order (= the serial first-seen order).
// Val order: the value-predicate table kernel (kvj_ptab) runs one lane per Val and
// one grid row per 16 leaf predicates, each row gated by the position classes of
// the value (Val.cls). Numbering the Vals grouped by (cls, type) makes its waves
// class-homogeneous: a wave whose values no predicate of the row applies to
// exits after one load, and the rest run the same predicate code without
// divergence. Buckets are ordered by key and stable inside (ingest order).
// class, type, then length bucket of the e-form bytes (16-byte steps up to 64, <= 128,
// longer): kvj_ptab keeps values of <= 64 / <= 128 bytes in registers, so a wave of one
// bucket runs one path, and its byte masks cover only the words its bucket occupies
inline uint64_t val_order_key(const Val& v) {
  const uint32_t lb = v.e_len <= 64u ? (v.e_len + 15u) / 16u : v.e_len <= 128u ? 5u : 6u;
  return (uint64_t)v.cls << 16 | (uint64_t)v.type << 8 | lb;
}

using KeyCount = std::unordered_map<uint64_t, uint32_t>;

// per-bucket first new id for each of `hists` (parts in order), buckets by ascending key
std::vector<KeyCount> val_order_cursors(const std::vector<KeyCount>& hists) {
  std::vector<uint64_t> keys;
  KeyCount total;
  for (const KeyCount& h : hists)
    for (const auto& kv : h)
      if (total.emplace(kv.first, 0).second) keys.push_back(kv.first);
  std::sort(keys.begin(), keys.end());
  std::vector<KeyCount> cur(hists.size());
  uint32_t next = 0;
  for (uint64_t key : keys)
    for (size_t k = 0; k < hists.size(); k++) {
      auto it = hists[k].find(key);
      if (it == hists[k].end()) continue;
      cur[k][key] = next;
      next += it->second;
    }
  return cur;
}

KeyCount val_hist(const StoreVec<Val>& vals) {
  KeyCount h;
  for (const Val& v : vals) h[val_order_key(v)]++;
  return h;
}

// serial ingest: renumber the Vals in place and remap the scalar cells
void order_vals(Batch& b) {
  std::vector<KeyCount> cur = val_order_cursors({val_hist(b.vals)});
  std::vector<uint32_t> perm(b.vals.size());
  StoreVec<Val> out(b.vals.size(), Val{}, b.vals.get_allocator());
  for (size_t i = 0; i < b.vals.size(); i++) {
    perm[i] = cur[0][val_order_key(b.vals[i])]++;
    out[perm[i]] = b.vals[i];
  }
  b.vals.swap(out);
  // a scalar's Val id is the hi word of its first unit in both transfer forms
  uint64_t* tc = b.tcells.data();
  b.each_unit([&](uint64_t, uint64_t u, bool) {
    if (node_scalar_t(node_type((uint32_t)tc[u]))) tc[u] = (tc[u] & 0xFFFFFFFFull) | (uint64_t)perm[tc[u] >> 32] << 32;
  });
}

void merge_batches(std::vector<Batch>& parts, Batch& b, uint32_t nstatic) {
  const size_t P = parts.size();
  std::unordered_map<std::string, uint32_t> dyn, nsi, gnsm, glset, gaset;
  std::vector<std::vector<uint32_t>> dmap(P), nmap(P), nsmmap(P), lmap(P), amap(P);
  std::vector<uint64_t> hb(P), vb(P), kb(P), rb(P), resb(P);
  uint64_t H = 0, V = 0, K = 0, R = 0, RS = 0;
  for (size_t k = 0; k < P; k++) {  // offsets and id remaps (serial, small)
    Batch& q = parts[k];
    H = (H + 3) & ~3ull;
    hb[k] = H; vb[k] = V; kb[k] = K; rb[k] = R; resb[k] = RS;
    H += q.strs.size(); V += q.vals.size(); K += q.kvs.size(); R += q.n_rows; RS += q.res.size();
    for (const std::string& s : q.dyn_keys) {
      auto it = dyn.find(s);
      if (it == dyn.end()) {
        it = dyn.emplace(s, nstatic + (uint32_t)b.dyn_keys.size()).first;
        b.dyn_keys.push_back(s);
      }
      dmap[k].push_back(it->second);
    }
    for (const std::string& s : q.namespaces) {
      auto it = nsi.find(s);
      if (it == nsi.end()) {
        it = nsi.emplace(s, (uint32_t)b.namespaces.size()).first;
        b.namespaces.push_back(s);
      }
      nmap[k].push_back(it->second);
    }
    // interned match inputs: first occurrence (in part order) is kept, offsets rebased
    for (size_t i = 0; i < q.nsm_keys.size(); i++) {
      auto it = gnsm.find(q.nsm_keys[i]);
      if (it == gnsm.end()) {
        it = gnsm.emplace(q.nsm_keys[i], (uint32_t)b.nsms.size()).first;
        b.nsms.push_back(StrRef{q.nsms[i].off + (uint32_t)hb[k], q.nsms[i].len});
      }
      nsmmap[k].push_back(it->second);
    }
    for (size_t i = 0; i < q.lset_keys.size(); i++) {
      auto it = glset.find(q.lset_keys[i]);
      if (it == glset.end()) {
        it = glset.emplace(q.lset_keys[i], (uint32_t)b.lsets.size()).first;
        b.lsets.push_back(KVSet{q.lsets[i].first + (uint32_t)kb[k], q.lsets[i].count});
      }
      lmap[k].push_back(it->second);
    }
    for (size_t i = 0; i < q.aset_keys.size(); i++) {
      auto it = gaset.find(q.aset_keys[i]);
      if (it == gaset.end()) {
        it = gaset.emplace(q.aset_keys[i], (uint32_t)b.asets.size()).first;
        b.asets.push_back(KVSet{q.asets[i].first + (uint32_t)kb[k], q.asets[i].count});
      }
      amap[k].push_back(it->second);
    }
    b.cells_used += q.cells_used;
  }
  // pattern-variable outcomes: re-interned globally, rows concatenated in resource order
  {
    std::unordered_map<std::string, uint32_t> gid;
    for (size_t k = 0; k < P; k++) {
      Batch& q = parts[k];
      std::vector<uint32_t> m(q.vout_tab.size());
      for (size_t i = 0; i < q.vout_tab.size(); i++) {
        auto it = gid.find(q.vout_tab[i]);
        if (it == gid.end()) {
          it = gid.emplace(q.vout_tab[i], (uint32_t)b.vout_tab.size()).first;
          b.vout_tab.push_back(q.vout_tab[i]);
        }
        m[i] = it->second;
      }
      for (uint32_t x : q.vout) b.vout.push_back(m[x]);
      std::vector<uint32_t>().swap(q.vout);
    }
  }
  if (H >= 0xFFFFFFF0ull) throw std::runtime_error("ingest: string heap exceeds 4 GiB");
  if (R * KV_LANES >= 0xFFFFFFF0ull) throw std::runtime_error("ingest: batch too large for 32-bit node indices");
  b.pin_store();
  std::vector<uint64_t> pcb(P + 1, 0);  // transfer-unit base of each part (its non-zero cells)
  for (size_t k = 0; k < P; k++) pcb[k + 1] = pcb[k] + parts[k].tcells.size();
  if (pcb[P] >= 0xFFFFFFF0ull) throw std::runtime_error("ingest: batch too large for 32-bit cell offsets");
  b.tcells.resize(pcb[P]);
  b.rmask.resize(R);
  b.rwide.resize(R);
  b.roff.resize(R);
  b.strs.reserve(H + 16);  // + the word-reader pad appended after the merge (no 2nd copy)
  b.strs.assign(H, '\0');
  b.vals.resize(V);
  b.kvs.resize(K);
  b.res.resize(RS);
  b.n_rows = R;
  std::vector<KeyCount> hists(P);
  std::vector<std::thread> th;
  for (size_t k = 0; k < P; k++) th.emplace_back([&, k]() { hists[k] = val_hist(parts[k].vals); });
  for (auto& t : th) t.join();
  th.clear();
  std::vector<KeyCount> cur = val_order_cursors(hists);
  for (size_t k = 0; k < P; k++)
    th.emplace_back([&, k]() {  // each part fills its own disjoint ranges (Vals: its share of every bucket)
      Batch& q = parts[k];
      const uint32_t h = (uint32_t)hb[k], k0 = (uint32_t)kb[k], r0 = (uint32_t)rb[k];
      memcpy(&b.strs[h], q.strs.data(), q.strs.size());
      std::vector<uint32_t> perm(q.vals.size());
      for (size_t i = 0; i < q.vals.size(); i++) {
        Val v = q.vals[i];
        v.e_off += h;
        if (v.flags & VF_N_VALID) v.n_off += h;
        perm[i] = cur[k][val_order_key(v)]++;
        b.vals[perm[i]] = v;
      }
      for (size_t i = 0; i < q.kvs.size(); i++) {
        KV x = q.kvs[i];
        x.k_off += h;
        x.v_off += h;
        b.kvs[kb[k] + i] = x;
      }
      // packed cells with key ids, values and (16-byte cells') rows and string offsets rebased:
      // each cell keeps its form (the 8-byte forms are rebase-invariant), so row masks and
      // offsets carry over, offset by the part's base
      uint64_t* out = &b.tcells[pcb[k]];
      const uint64_t* in = q.tcells.data();
      q.each_unit([&](uint64_t, uint64_t u, bool wide) {
        uint64_t x = in[u];
        const uint32_t t = node_type((uint32_t)x);
        uint32_t key = node_key((uint32_t)x);
        if (key >= nstatic && key != KEY_NONE28) key = dmap[k][key - nstatic];
        uint32_t a = (uint32_t)(x >> 32);
        if (node_scalar_t(t)) a = perm[a];
        else if (wide && (t == NT_MAP || t == NT_ARR)) a += r0;
        out[u] = (uint64_t)(key << 4 | t) | (uint64_t)a << 32;
        if (wide) out[u + 1] = node_scalar_t(t) ? in[u + 1] + h : in[u + 1];  // (b += h: the low word, no carry)
      });
      memcpy(&b.rmask[r0], q.rmask.data(), q.n_rows * sizeof(uint64_t));
      memcpy(&b.rwide[r0], q.rwide.data(), q.n_rows * sizeof(uint64_t));
      for (uint64_t row = 0; row < q.n_rows; row++) b.roff[r0 + row] = q.roff[row] + (uint32_t)pcb[k];
      for (size_t i = 0; i < q.res.size(); i++) {
        Res r = q.res[i];
        r.root += r0;
        r.name_off += h;
        r.nsm = nsmmap[k][r.nsm];
        r.lset = lmap[k][r.lset];
        r.aset = amap[k][r.aset];
        r.ns_index = nmap[k][r.ns_index];
        b.res[resb[k] + i] = r;
      }
      // the part's arrays are released here, in parallel (freed serially by the parts'
      // destructors they cost ~70 ms per million Pods on the GPU box: page unmapping)
      StoreVec<uint64_t>().swap(q.tcells);
      decltype(q.vals)().swap(q.vals);
      decltype(q.res)().swap(q.res);
      decltype(q.rmask)().swap(q.rmask);
      decltype(q.rwide)().swap(q.rwide);
      decltype(q.roff)().swap(q.roff);
      decltype(q.kvs)().swap(q.kvs);
      HeapStr().swap(q.strs);
    });
  for (auto& t : th) t.join();
}

}  // namespace

// The string value of the first `"<key>":` in a resource's JSON text (no escapes; empty when
// absent): the store-order key. A miss only changes which resources share a wave group.
std::string_view raw_string_of(const char* p, size_t n, const char* key, size_t kl) {
  const char* e = p + n;
  for (const char* q = p; q < e;) {
    const char* k = (const char*)memmem(q, (size_t)(e - q), key, kl);
    if (!k) return {};
    const char* v = k + kl;
    while (v < e && (*v == ' ' || *v == '\t' || *v == '\n' || *v == '\r')) v++;
    if (v < e && *v == ':') {
      v++;
      while (v < e && (*v == ' ' || *v == '\t' || *v == '\n' || *v == '\r')) v++;
      if (v >= e || *v != '"') return {};
      const char* a = ++v;
      while (v < e && *v != '"' && *v != '\\') v++;
      return std::string_view(a, (size_t)(v - a));
    }
    q = k + kl;
  }
  return {};
}

// The store-order weight of a resource from its JSON text, one pass over its quotes: the
// "image" keys (its containers) above a "volumes" key above the "securityContext", "resources"
// and "ports" keys (the containers' optional parts), so like resources sort together
uint32_t shape_weight(const char* p, size_t n) {
  uint32_t img = 0, vol = 0, sc = 0, rs = 0, po = 0;
  const char* e = p + n;
  auto key = [&](const char* q) {  // q: the byte after a quote
    auto is = [&](const char* k, size_t kl) { return (size_t)(e - q) >= kl && memcmp(q, k, kl) == 0; };
    switch (*q) {
      case 'i': img += is("image\"", 6); break;
      case 'v': vol |= is("volumes\"", 8); break;
      case 's': sc += is("securityContext\"", 16); break;
      case 'r': rs += is("resources\"", 10); break;
      case 'p': po += is("ports\"", 6); break;
      default: break;
    }
  };
  const __m128i qq = _mm_set1_epi8('"');  // quotes 16 bytes at a time (SSE2)
  const char* q = p;
  for (; q + 16 <= e; q += 16) {
    unsigned m = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i*)q), qq));
    while (m) {
      const unsigned b = (unsigned)__builtin_ctz(m);
      m &= m - 1;
      if (q + b + 1 < e) key(q + b + 1);
    }
  }
  for (; q < e; q++)
    if (*q == '"' && q + 1 < e) key(q + 1);
  return std::min(img, 255u) << 24 | vol << 23 | std::min(sc, 15u) << 16 | std::min(rs, 15u) << 12 | std::min(po, 15u) << 8;
}

// Store order from per-resource (kind, namespace) keys: kinds in order of first appearance,
// inside a kind its namespaces in order of first appearance, input order inside a (kind,
// namespace) run (stable counting sort, per-thread key tables merged in thread order); empty
// when every resource has the same key. Resources of one kind share wave groups, so a rule that
// matches other kinds only is skipped by whole waves (its match fails uniformly) instead of
// running its pattern walk for the few lanes of a mixed wave (C5: 6.1 -> 4.3 ms per pass); and
// resources of one namespace share waves and workgroups, so the rule kernels count per-scope
// PolicyReport results for a whole wave at once (kv_end_flush) and neighbouring resources share
// match tuples.
// Inside a (kind, namespace) run the resources are ordered by descending weight (`weight`,
// shape_weight: the "image" keys of each document, i.e. its containers, init and ephemeral
// containers, then a "volumes" key, then the containers' optional parts), input order among
// equals. A fused loop over an array
// runs as many iterations as the wave's largest array: waves of like resources run fewer of them
// (C2: most waves held a 4-container Pod, ran 4 iterations for 1.75 containers per Pod on average),
// and iteration i runs on a prefix of the lanes, so the active cells of the element rows of the path
// columns share cache lines (round 6: sorting inside each wave group alone took C2 0.517 -> 0.483,
// C4 0.844 -> 0.786, C5 2.57 -> 2.445 ms per pass).
std::vector<uint32_t> store_order(const std::vector<std::string_view>& kinds, const std::vector<std::string_view>& nss,
                                  const std::vector<uint32_t>* weight, unsigned T) {
  struct KeyHash {
    size_t operator()(const std::pair<std::string_view, std::string_view>& k) const {
      return std::hash<std::string_view>()(k.first) * 1000003u ^ std::hash<std::string_view>()(k.second);
    }
  };
  using Map = std::unordered_map<std::pair<std::string_view, std::string_view>, uint32_t, KeyHash>;
  const size_t n = kinds.size();
  const size_t C = std::max<size_t>(1, std::min<size_t>(T, n / 4096 + 1));
  const size_t per = (n + C - 1) / C;
  std::vector<Map> local(C);
  std::vector<std::vector<std::pair<std::string_view, std::string_view>>> lkeys(C);
  std::vector<uint32_t> key(n);
  auto run = [&](auto&& f) {
    std::vector<std::thread> th;
    for (size_t c = 1; c < C; c++) th.emplace_back(f, c);
    f((size_t)0);
    for (auto& t : th) t.join();
  };
  run([&](size_t c) {
    for (size_t i = c * per; i < std::min(n, (c + 1) * per); i++) {
      const auto k = std::make_pair(kinds[i], nss[i]);
      auto it = local[c].find(k);
      if (it == local[c].end()) {
        it = local[c].emplace(k, (uint32_t)lkeys[c].size()).first;
        lkeys[c].push_back(k);
      }
      key[i] = it->second;
    }
  });
  // global key ids in first-appearance order; kinds and namespaces ranked by first appearance
  Map gid;
  std::unordered_map<std::string_view, uint32_t> kid, nid;
  std::vector<std::pair<uint64_t, uint32_t>> rank;  // (kind rank << 32 | namespace rank, key id)
  std::vector<std::vector<uint32_t>> remap(C);
  for (size_t c = 0; c < C; c++)
    for (const auto& k : lkeys[c]) {
      auto it = gid.find(k);
      if (it == gid.end()) {
        it = gid.emplace(k, (uint32_t)gid.size()).first;
        const uint64_t kr = kid.emplace(k.first, (uint32_t)kid.size()).first->second;
        const uint64_t nr = nid.emplace(k.second, (uint32_t)nid.size()).first->second;
        rank.push_back({kr << 32 | nr, it->second});
      }
      remap[c].push_back(it->second);
    }
  if (gid.size() < 2 && !weight) return {};
  std::sort(rank.begin(), rank.end());
  std::vector<uint32_t> slot(gid.size());  // key id -> position of its run
  for (size_t q = 0; q < rank.size(); q++) slot[rank[q].second] = (uint32_t)q;
  // counting sort: per-thread run sizes, run offsets per thread, parallel scatter
  const size_t K = gid.size();
  std::vector<std::vector<uint32_t>> cnt(C, std::vector<uint32_t>(K, 0));
  run([&](size_t c) {
    for (size_t i = c * per; i < std::min(n, (c + 1) * per); i++) {
      key[i] = slot[remap[c][key[i]]];
      cnt[c][key[i]]++;
    }
  });
  uint32_t at = 0;
  for (size_t k = 0; k < K; k++)
    for (size_t c = 0; c < C; c++) {
      const uint32_t x = cnt[c][k];
      cnt[c][k] = at;
      at += x;
    }
  std::vector<uint32_t> order(n);
  run([&](size_t c) {
    for (size_t i = c * per; i < std::min(n, (c + 1) * per); i++) order[cnt[c][key[i]]++] = (uint32_t)i;
  });
  if (weight && weight->size() == n) {  // descending weight inside each (kind, namespace) run
    std::vector<std::pair<size_t, size_t>> runs;
    for (size_t a = 0; a < n;) {
      size_t b = a + 1;
      while (b < n && key[order[b]] == key[order[a]]) b++;
      runs.push_back({a, b});
      a = b;
    }
    std::atomic<size_t> next{0};
    std::atomic<bool> moved{false};
    auto by_weight = [&](uint32_t x, uint32_t y) { return (*weight)[x] > (*weight)[y]; };
    run([&](size_t) {
      for (size_t q; (q = next++) < runs.size();) {
        auto a = order.begin() + runs[q].first, b = order.begin() + runs[q].second;
        if (std::is_sorted(a, b, by_weight)) continue;
        std::stable_sort(a, b, by_weight);
        moved = true;
      }
    });
    if (!moved && gid.size() < 2) return {};
  }
  return order;
}

// The match inputs of a resource: every Res field the match code reads (kvfac.h, the generated
// g_blk_* filters: kind, group, version, nsm, lset, aset, ns_index, flags; name-dependent rules
// are evaluated per resource behind bit 1). A new match input in Res must join the key; the
// assert trips when Res changes shape.
static_assert(sizeof(Res) == 64, "Res changed: check that tuple_key still covers every match input");
static void tuple_key(const Res& r, uint32_t* k) {
  k[0] = r.kind; k[1] = r.group; k[2] = r.version; k[3] = r.nsm;
  k[4] = r.lset; k[5] = r.aset; k[6] = r.ns_index; k[7] = r.flags;
}

void match_tuples(Batch* b) {
  // open addressing over 64-bit hashes of the match inputs, confirmed field by field against
  // the tuple's first resource; tables sized by the tuples found (grown at half load), so a
  // few thousand tuples over a million resources stay cache-resident
  auto key = tuple_key;
  auto hash = [](const uint32_t* k) {
    uint64_t h = 1469598103934665603ull;
    for (int j = 0; j < 8; j++) h = (h ^ k[j]) * 1099511628211ull, h ^= h >> 29;
    return h ? h : 1;
  };
  struct Tab {
    size_t cap = 4096;
    std::vector<uint64_t> hs = std::vector<uint64_t>(4096, 0);
    std::vector<uint32_t> ids = std::vector<uint32_t>(4096, 0);
    std::vector<uint32_t> rep;  // first resource of each tuple, in first-occurrence order
    void grow() {
      std::vector<uint64_t> oh(cap * 2, 0);
      std::vector<uint32_t> oi(cap * 2, 0);
      oh.swap(hs);
      oi.swap(ids);
      cap *= 2;
      for (size_t j = 0; j < oh.size(); j++)
        if (oh[j]) {
          size_t at = oh[j] & (cap - 1);
          while (hs[at]) at = (at + 1) & (cap - 1);
          hs[at] = oh[j];
          ids[at] = oi[j];
        }
    }
    // id of resource i's tuple (k, hash h), added when new
    uint32_t id(const Batch* b, uint32_t i, const uint32_t* k, uint64_t h) {
      size_t at = h & (cap - 1);
      for (;; at = (at + 1) & (cap - 1)) {
        if (hs[at] == 0) {
          hs[at] = h;
          ids[at] = (uint32_t)rep.size();
          rep.push_back(i);
          const uint32_t r = ids[at];
          if (rep.size() * 2 > cap) grow();
          return r;
        }
        if (hs[at] == h) {
          uint32_t q[8];
          tuple_key(b->res[rep[ids[at]]], q);
          if (memcmp(k, q, 8 * sizeof(uint32_t)) == 0) return ids[at];
        }
      }
    }
  };
  // chunks numbered locally in parallel, then their tuple lists merged in chunk order (so
  // ids stay in first-occurrence order over the whole batch) and the ids remapped
  const size_t n = b->res.size();
  const size_t C = std::max<size_t>(1, std::min<size_t>({(size_t)ingest_threads(), (size_t)16, n / 256}));
  const size_t per = (n + C - 1) / std::max<size_t>(C, 1);
  std::vector<Tab> tabs(C);
  auto run = [&](auto&& f) {
    std::vector<std::thread> th;
    for (size_t c = 1; c < C; c++) th.emplace_back(f, c);
    f((size_t)0);
    for (auto& t : th) t.join();
  };
  run([&](size_t c) {
    for (size_t i = c * per; i < std::min(n, (c + 1) * per); i++) {
      uint32_t k[8];
      key(b->res[i], k);
      b->res[i].tup = tabs[c].id(b, (uint32_t)i, k, hash(k));
    }
  });
  Tab g;
  std::vector<std::vector<uint32_t>> remap(C);
  for (size_t c = 0; c < C; c++)
    for (uint32_t r : tabs[c].rep) {
      uint32_t k[8];
      key(b->res[r], k);
      remap[c].push_back(g.id(b, r, k, hash(k)));
    }
  run([&](size_t c) {
    for (size_t i = c * per; i < std::min(n, (c + 1) * per); i++) b->res[i].tup = remap[c][b->res[i].tup];
  });
  b->tup_rep = std::move(g.rep);
  // kind entities of the tuples (few: kinds x versions), found through the last hit first
  // (tuples of one kind are numbered together in the kind-grouped store order)
  b->tup_kent.resize(b->tup_rep.size());
  b->kent_rep.clear();
  auto kkey = [&](const Res& r) {
    return std::array<uint32_t, 4>{r.kind, r.group, r.version, r.flags & (RF_KIND_NAMESPACE | RF_KIND_EMPTY)};
  };
  std::vector<std::array<uint32_t, 4>> kents;
  uint32_t last = 0;
  for (size_t t = 0; t < b->tup_rep.size(); t++) {
    const auto k = kkey(b->res[b->tup_rep[t]]);
    if (kents.empty() || kents[last] != k) {
      last = 0;
      while (last < kents.size() && kents[last] != k) last++;
      if (last == kents.size()) {
        kents.push_back(k);
        b->kent_rep.push_back(b->tup_rep[t]);
      }
    }
    b->tup_kent[t] = last;
  }
}

void ingest_resources(const PolicySet& ps, const char* json, size_t len, const char* ns_labels_json, Batch* b) {
  const unsigned T = ingest_threads();
  size_t first = 0;
  while (first < len && (json[first] == ' ' || json[first] == '\t' || json[first] == '\n' || json[first] == '\r')) first++;
  std::vector<size_t> starts;
  bool parallel = false;
  std::unordered_map<std::string, uint32_t> ns_index;
  const auto t0 = std::chrono::steady_clock::now();
  auto ms = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
  const bool verbose = getenv("KVGPU_VERBOSE") != nullptr;
  // NDJSON first (documents = lines); when a document does not end its line, the values are
  // found again by the full scan
  bool lines = T > 1 && len >= (1u << 20) && first < len && json[first] == '{' && split_lines(json, len, T, &starts);
  // The merged store's page-locked blocks are taken from the pool while the documents are parsed:
  // a thread takes blocks of the estimated sizes (resource headers: exact; packed node cells: about
  // the input's bytes; values: an eighth of them) and hands them back, so the merge finds them in
  // the pool instead of page-locking fresh memory then (the first batch of a process: ~200 ms
  // per million Pods on the GPU box). A block is used when it is 1-2x the size asked for.
  struct Join {
    std::thread t;
    ~Join() {
      if (t.joinable()) t.join();
    }
  } prewarm;
  if (g_hostmem.take && g_hostmem.give && starts.size() >= 65536) {
    const size_t est[3] = {starts.size() * sizeof(Res), len, len / 8};
    prewarm.t = std::thread([est]() {
      for (size_t e : est)
        if (e >= (16u << 20))
          if (void* p = g_hostmem.take(e)) g_hostmem.give(p);
    });
  }
  for (int attempt = 0; attempt < 2 && !parallel; attempt++) {
    if (attempt == 1 || !lines) {
      starts.clear();
      lines = false;
      b->order.clear();
      if (!(T > 1 && len >= (1u << 20) && first < len && json[first] == '{' && scan_values(json, len, T, &starts))) break;
    }
    if (verbose) fprintf(stderr, "[kvgpu] ingest: %s %.1f ms (%zu values)\n", lines ? "lines" : "scan", ms(), starts.size());
    // whole wave groups per thread, so lane = resource index % 64 holds in the merged batch
    const size_t nres = starts.size(), groups = (nres + KV_LANES - 1) / KV_LANES;
    const size_t per = (groups + T - 1) / T * KV_LANES;
    const size_t P = (nres + per - 1) / per;
    {  // store order: resources grouped by kind, then namespace
      std::vector<std::string_view> kinds(nres), nss(nres);
      std::vector<uint32_t> weight(nres);
      std::vector<std::thread> kt;
      for (size_t k = 0; k < P; k++)
        kt.emplace_back([&, k]() {
          for (size_t i = k * per; i < std::min(nres, (k + 1) * per); i++) {
            const size_t end = i + 1 < nres ? starts[i + 1] : len;
            kinds[i] = raw_string_of(json + starts[i], end - starts[i], "\"kind\"", 6);
            nss[i] = raw_string_of(json + starts[i], end - starts[i], "\"namespace\"", 11);
            weight[i] = shape_weight(json + starts[i], end - starts[i]);
          }
        });
      for (auto& t : kt) t.join();
      b->order = store_order(kinds, nss, &weight, T);
    }
    if (verbose) fprintf(stderr, "[kvgpu] ingest: store order %.1f ms\n", ms());
    const std::vector<uint32_t>& order = b->order;
    std::vector<Batch> parts(P);
    std::vector<std::string> errs(P);
    std::vector<double> tparse(P, 0.0), ttake(P, 0.0);
    std::vector<std::thread> th;
    for (size_t k = 0; k < P; k++)
      th.emplace_back([&, k]() {
        try {
          Ingest in(ps, parts[k]);
          JDoc doc;
          const size_t e = std::min(nres, (k + 1) * per);
          in.expected_res = e > k * per ? e - k * per : 0;
          for (size_t q = k * per; q < e; q++) {
            const size_t i = order.empty() ? q : order[q];
            const size_t end = i + 1 < nres ? starts[i + 1] : len;
            doc.nodes.clear();
            doc.strs.clear();
            const auto tp0 = std::chrono::steady_clock::now();
            const size_t used = parse_one(json + starts[i], end - starts[i], NUM_UNSTRUCTURED, &doc);
            const auto tp1 = std::chrono::steady_clock::now();
            tparse[k] += std::chrono::duration<double, std::milli>(tp1 - tp0).count();
            if (lines)  // the document must end its line
              for (size_t x = starts[i] + used; x < end; x++)
                if (json[x] != ' ' && json[x] != '\t' && json[x] != '\r' && json[x] != '\n') throw NotLines();
            in.take(doc);
            ttake[k] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp1).count();
          }
          const auto tf0 = std::chrono::steady_clock::now();
          in.flush_group();
          ttake[k] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tf0).count();
        } catch (const NotLines&) {
          errs[k] = "\x01";
        } catch (const std::exception& ex) {
          errs[k] = lines ? "\x01" : ex.what();  // (a line-split document may be a fragment)
        }
      });
    for (auto& t : th) t.join();
    bool relines = false;
    for (auto& e : errs) relines |= e == "\x01";
    if (relines) continue;  // not one document per line: scan
    for (auto& e : errs)
      if (!e.empty()) throw std::runtime_error(e);
    if (verbose) {
      double tp = 0, tt = 0;
      for (size_t k = 0; k < P; k++) tp += tparse[k], tt += ttake[k];
      fprintf(stderr, "[kvgpu] ingest: %zu threads %.1f ms (per thread: parse %.1f ms, take %.1f ms)\n", P, ms(), tp / P, tt / P);
    }
    if (prewarm.t.joinable()) prewarm.t.join();
    merge_batches(parts, *b, (uint32_t)ps.keys.size());
    {  // what the parts still hold is freed in parallel too (serially ~70-80 ms per million
       // Pods on the GPU box, after the merge threads have released the store arrays)
      std::vector<std::thread> ft;
      for (size_t k = 0; k < P; k++) ft.emplace_back([&parts, k]() { Batch dead(std::move(parts[k])); });
      for (auto& t : ft) t.join();
    }
    if (verbose)
      fprintf(stderr, "[kvgpu] ingest: merge %.1f ms (%zu vals, %llu rows, %zu string bytes, %zu/%zu/%zu nsm/label/annotation sets)\n",
              ms(), b->vals.size(), (unsigned long long)b->n_rows, b->strs.size(), b->nsms.size(), b->lsets.size(),
              b->asets.size());
    for (size_t i = 0; i < b->namespaces.size(); i++) ns_index.emplace(b->namespaces[i], (uint32_t)i);
    parallel = true;
  }
  if (verbose) fprintf(stderr, "[kvgpu] ingest: parts released %.1f ms\n", ms());
  if (!parallel) {
    Ingest in(ps, *b);
    if (len <= (64u << 20)) {  // small inputs: documents held, taken in store order
      std::vector<JDoc> docs;
      parse_json_stream(json, len, NUM_UNSTRUCTURED, [&](JDoc& d) { docs.push_back(std::move(d)); });
      std::vector<std::string_view> kinds(docs.size()), nss(docs.size());
      for (size_t i = 0; i < docs.size(); i++) {
        const JDoc& d = docs[i];
        const int64_t c = d.at(d.root).t == J_MAP ? d.get(d.root, "kind") : -1;
        if (c >= 0 && d.at((uint32_t)c).t == J_STR) kinds[i] = d.sval(d.at((uint32_t)c));
        const int64_t m = d.at(d.root).t == J_MAP ? d.get(d.root, "metadata") : -1;
        const int64_t ns = m >= 0 && d.at((uint32_t)m).t == J_MAP ? d.get((uint32_t)m, "namespace") : -1;
        if (ns >= 0 && d.at((uint32_t)ns).t == J_STR) nss[i] = d.sval(d.at((uint32_t)ns));
      }
      b->order = store_order(kinds, nss, nullptr, 1);
      for (size_t q = 0; q < docs.size(); q++) in.take(docs[b->order.empty() ? q : b->order[q]]);
    } else {
      parse_json_stream(json, len, NUM_UNSTRUCTURED, [&](JDoc& d) { in.take(d); });
    }
    in.flush_group();
    for (size_t i = 0; i < b->namespaces.size(); i++) ns_index.emplace(b->namespaces[i], (uint32_t)i);
    order_vals(*b);
  }
  // namespace labels (CLI --values-file namespaceSelector map / cluster namespaces)
  b->ns_labels.assign(b->namespaces.size(), {});
  if (ns_labels_json && *ns_labels_json) {
    JDoc d;
    parse_json(ns_labels_json, strlen(ns_labels_json), NUM_FLOAT, &d);
    const JNode& r = d.at(d.root);
    if (r.t == J_MAP) {
      for (uint32_t c = r.first; c < r.first + r.count; c++) {
        std::string nsn(d.key(d.at(c)));
        auto it = ns_index.find(nsn);
        if (it == ns_index.end()) continue;
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
  if (verbose) fprintf(stderr, "[kvgpu] ingest: namespace selectors %.1f ms\n", ms());
  // word-granular readers may touch up to 8 bytes past the last string
  b->strs.append(16, '\0');
  if (verbose) fprintf(stderr, "[kvgpu] ingest: namespaces %.1f ms\n", ms());
  match_tuples(b);
  if (verbose) fprintf(stderr, "[kvgpu] ingest: match tuples %.1f ms (%zu)\n", ms(), b->tup_rep.size());
  // interning keys are only needed while ingesting
  std::unordered_map<std::string, uint32_t>().swap(b->vout_id);
  std::vector<std::string>().swap(b->nsm_keys);
  std::vector<std::string>().swap(b->lset_keys);
  std::vector<std::string>().swap(b->aset_keys);
  // algorithmic bytes: populated cells only (row padding of the wave-group layout excluded)
  b->bytes_referenced = b->cells_used * sizeof(Node) + b->vals.size() * sizeof(Val) + b->res.size() * sizeof(Res) +
                        b->kvs.size() * sizeof(KV) + b->strs.size() + b->nsms.size() * sizeof(StrRef) +
                        (b->lsets.size() + b->asets.size()) * sizeof(KVSet);
  if (verbose)
    fprintf(stderr,
            "[kvgpu] ingest: transfer bytes: tcells %zu rmask+rwide %zu roff %zu vals %zu res %zu kvs %zu strs %zu "
            "(cells used %zu, rows %zu)\n",
            b->tcells.size() * 8, b->rmask.size() * 16, b->roff.size() * 4, b->vals.size() * sizeof(Val),
            b->res.size() * sizeof(Res), b->kvs.size() * sizeof(KV), b->strs.size(), (size_t)b->cells_used,
            (size_t)b->n_rows);
}

uint64_t Batch::transfer_bytes() const {
  return tcells.size() * 8 + (rmask.size() + rwide.size()) * 8 + roff.size() * 4 + vals.size() * sizeof(Val) +
         res.size() * sizeof(Res) + kvs.size() * sizeof(KV) + strs.size() + ns_bits.size() * 4 +
         nsms.size() * sizeof(StrRef) + (lsets.size() + asets.size()) * sizeof(KVSet) +
         (tup_rep.size() + tup_kent.size() + kent_rep.size()) * 4;
}

}  // namespace kvh
