// Specialized kernels for a compiled policy set (see kvjit.hpp).
//
// Every GPU-routed rule's bytecode program (kvcompile.cpp) is re-emitted as a
// device function whose statements are the interpreter's op semantics
// (kvkernel.hip) with the operands folded in: key slots, predicate constants,
// glob segment words and quantity operands become immediates, the cursor stack
// becomes registers c0..cN, and the interpreter's parked-lane wake-up pcs
// (skip / catch targets) become gotos that each lane takes on its own (the
// hardware exec mask runs the divergence). Rule functions are inlined into
// chunk kernels, so lookups shared by several rules (root -> spec ->
// containers ...) are loaded once per chunk (the node store is __restrict__).
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <dlfcn.h>
#include <sched.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/wait.h>

#include <cerrno>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <sstream>
#include <stdexcept>
#include <thread>
#include <unordered_map>

#include "kvjit.hpp"
#include "kvdevtypes.h"

extern char** environ;

namespace kvh {

using namespace kv;

namespace {

const char* kPrelude =
#include "kvjit_prelude.inc"
    ;

std::string hex32(uint32_t v) {
  char b[16];
  snprintf(b, sizeof b, "0x%08xu", v);
  return b;
}
std::string u32(uint32_t v) { return std::to_string(v) + "u"; }
std::string u64(uint64_t v) { return std::to_string(v) + "ull"; }
std::string i64(int64_t v) {
  if (v == INT64_MIN) return "(-9223372036854775807ll - 1)";
  return std::to_string(v) + "ll";
}
std::string f64(double v) {
  uint64_t b;
  memcpy(&b, &v, 8);
  return "__longlong_as_double(" + i64((int64_t)b) + ")";
}

// rule groups of at least this many members write their records at the resource's slot of the
// record row; the other rules append theirs to the wave's segment (kvdevfn.h kv_gfin). Round 4
// (gpurun_out/ab3, ms per pass / GB written): from 16 members C2 0.720 / 0.47 (its 20- and
// 21-member image-glob groups go to slots), C3 8.22 / 9.7; from 22 C2 0.701 / 0.40, C3 8.24 /
// 9.4; never C2 0.699 / 0.40, C3 9.13 / 7.5.
constexpr uint32_t kGslotMembers = 22u;
uint32_t gslot_members() { return kGslotMembers; }

struct Gen {
  const PolicySet& ps;
  std::ostringstream o;
  std::set<uint32_t> preds_done, atoms_done;
  // value-predicate memo: a leaf predicate on a scalar is a pure function of the
  // (deduplicated) Val it reads, so each one is evaluated once per distinct value
  // of the batch (kvj_ptab) and the rule kernels test one bit of the table
  std::vector<uint32_t> mpreds;  // memo slot -> pred
  std::map<uint32_t, uint32_t> pslot;  // pred -> memo slot
  // Leaves on a hoisted scalar read their table word(s) through a load hoisted with the
  // cursor (issued with the other lookups of the region instead of one dependent load
  // per rule). Hoisted lookups are branch-free (a failed guard reads cell 0 and discards
  // it) and are placed at the top of their chunk / fused-loop body, so the loads of one
  // tree level issue together instead of one dependent wait per lookup.
  explicit Gen(const PolicySet& p) : ps(p), rec_slot(p.rules.size(), 0) {
    fams.emplace_back();
    col_of(0, "R");  // column 0 of family 0: the root
  }

  // ---------------------------------------------------------------- path columns
  // Hoisted lookups (below) read the node at their static path from a column of the batch
  // (kvdevtypes.h, built per batch by kvcol.h) instead of walking the node rows from the root
  // or the loop element: one independent coalesced load per lookup instead of a chain of
  // dependent ones. Family 0 holds root paths; family f > 0 the paths relative to the elements
  // of one array path (a column of family 0). Columns are numbered in order of first use; the
  // column count of each family is a macro (KVC_J<f>) defined at the head of every kernel
  // program once the whole image is generated.
  // Site records of rule groups (kvdevtypes.h GSiteDesc): per group of 2+ members its descriptor
  // (n, gpre, moff, 0) in gs_desc and its members' (rule, pattern-node shift) in gs_mem, numbered
  // in generation order over the image; k_gs0 / k_gsn: the first group and the groups of the kernel
  // being generated (round 5, with the unwritten NOMATCH segments: C3 writes 9.4 -> 2.9 GB per pass).
  std::vector<uint32_t> gs_desc, gs_mem;
  uint32_t gs_members = 0, k_gs0 = 0, k_gsn = 0;
  struct Fam {
    std::string arr;                          // family array expr (family 0: "")
    std::map<std::string, uint32_t> idx;      // relative expr -> column
    std::vector<std::vector<uint32_t>> steps; // per column: its path steps
  };
  std::vector<Fam> fams;
  std::map<std::string, uint32_t> fam_of;  // family array expr -> family
  static constexpr uint32_t kNoCol = 0xFFFFFFFFu;
  // steps of a symbolic path: "/s<slot>" (slot-addressed map) or "/k<key>" (keep-all map
  // scan) after the root token ("R", or "E<tag>" of a loop element, or nothing)
  static bool expr_steps(const std::string& ex, std::vector<uint32_t>* out) {
    out->clear();
    size_t at = ex.find('/');
    while (at != std::string::npos) {
      const size_t nx = ex.find('/', at + 1);
      const std::string tok = ex.substr(at + 1, nx == std::string::npos ? std::string::npos : nx - at - 1);
      if (tok.size() < 2 || (tok[0] != 's' && tok[0] != 'k')) return false;
      const unsigned long v = strtoul(tok.c_str() + 1, nullptr, 10);
      if (v >= KV_COL_SCAN) return false;
      out->push_back((uint32_t)v | (tok[0] == 'k' ? KV_COL_SCAN : 0u));
      at = nx;
    }
    return out->size() <= KV_COL_MAXD;
  }
  uint32_t col_of(uint32_t f, const std::string& rel) {
    Fam& F = fams.at(f);
    auto it = F.idx.find(rel);
    if (it != F.idx.end()) return it->second;
    std::vector<uint32_t> st;
    if (!expr_steps(rel, &st)) return kNoCol;
    const uint32_t j = (uint32_t)F.steps.size();
    F.idx.emplace(rel, j);
    F.steps.push_back(st);
    return j;
  }
  // family of the elements of array expr `arr` (a root path); its column 0 is the element itself
  uint32_t family(const std::string& arr) {
    auto it = fam_of.find(arr);
    if (it != fam_of.end()) return it->second;
    if (col_of(0, arr) == kNoCol) return kNoCol;
    const uint32_t f = (uint32_t)fams.size();
    fams.emplace_back();
    fams.back().arr = arr;
    col_of(f, "");
    fam_of.emplace(arr, f);
    return f;
  }
  // the plan (JitImage::cols / fam_*) and the macro block of the kernel programs
  void col_plan(JitImage* out, std::string* defs) const {
    out->cols.clear();
    out->fam_arr.clear();
    out->fam_ncols.clear();
    std::ostringstream d;
    for (uint32_t f = 0; f < fams.size(); f++) {
      const Fam& F = fams[f];
      out->fam_arr.push_back(f ? fams[0].idx.at(F.arr) : 0u);  // (family 0 columns come first)
      out->fam_ncols.push_back((uint32_t)F.steps.size());
      d << "#define KVC_J" << f << " " << F.steps.size() << "u\n";
      for (uint32_t j = 0; j < F.steps.size(); j++) {
        ColDesc c{};
        c.fam = f;
        c.j = j;
        c.nsteps = (uint32_t)F.steps[j].size();
        for (uint32_t s = 0; s < c.nsteps; s++) c.steps[s] = F.steps[j][s];
        out->cols.push_back(c);
      }
    }
    for (uint32_t f = 1; f < fams.size(); f++) out->cols.at(out->fam_arr[f]).arr_fam = f;
    *defs = d.str();
  }

  // leaf predicate `pi` on node expression `n` (arrays: every element): one bit of the
  // value-predicate table
  std::string leaf_test(uint32_t pi, const std::string& n) {
    const uint32_t slot = slot_for(pi);
    return "((kv_leaf_word(P, N, " + n + ", " + u32(slot / 32) + ") >> " + u32(slot % 32) + ") & 1u) != 0u";
  }

  // ---------------------------------------------------------------- globs
  // word compare of segment `sg` against value bytes [k, k + len) (base 4-byte aligned)
  std::string seg_expr(const GSeg& sg, const std::string& k, bool aligned0) {
    const uint32_t nw = (sg.len + 3) / 4;
    std::ostringstream e;
    e << "([&]() -> bool { ";
    if (aligned0) {
      e << "uint32_t x = 0u; ";
      for (uint32_t i = 0; i < nw; i++) {
        const GWord& g = ps.gwords[sg.wfirst + i];
        if (g.mask == 0) continue;
        e << "x |= (base[" << i << "] ^ " << hex32(g.w) << ") & " << hex32(g.mask) << "; ";
      }
      e << "return x == 0u; })()";
      return e.str();
    }
    e << "const uint32_t k_ = " << k << ", a_ = k_ >> 2, sh_ = k_ & 3u; uint32_t lo_ = base[a_], hi_, x = 0u; ";
    for (uint32_t i = 0; i < nw; i++) {
      const GWord& g = ps.gwords[sg.wfirst + i];
      e << "hi_ = base[a_ + " << (i + 1) << "]; ";
      if (g.mask) e << "x |= (__builtin_amdgcn_alignbyte(hi_, lo_, sh_) ^ " << hex32(g.w) << ") & " << hex32(g.mask) << "; ";
      e << "lo_ = hi_; ";
    }
    e << "return x == 0u; })()";
    return e.str();
  }

  std::set<uint32_t> globs_done;
  void glob_once(uint32_t ai) {
    if (globs_done.insert(ai).second) glob_fn(ai);
  }

  void glob_fn(uint32_t ai) {
    const Atom& A = ps.atoms[ai];
    o << "__device__ __forceinline__ bool g_glob_" << ai
      << "(const uint8_t* __restrict__ s, uint32_t sl, bool ascii, const uint8_t* __restrict__ pstr) {\n";
    const uint32_t fl = A.gflags;
    if (fl & G_ALL) { o << "  return true;\n}\n"; return; }
    if (fl & G_EMPTY) { o << "  return sl == 0u;\n}\n"; return; }
    if (fl & G_HASQ)
      o << "  if (!ascii) return kv_glob(pstr + " << u32(A.s_off) << ", " << u32(A.s_len & 0x7FFFFFFFu) << ", s, sl);\n";
    o << "  if (sl < " << u32(A.gmin) << ") return false;\n";
    o << "  const uint32_t* __restrict__ base = (const uint32_t*)s;\n";
    const uint32_t n = A.gcount;
    const GSeg* segs = ps.gsegs.data() + A.gfirst;
    uint32_t i0 = 0, i1 = n;
    o << "  uint32_t pos = 0u, end = sl;\n";
    if (!(fl & G_LEAD)) {
      const GSeg& s0 = segs[0];
      if (n == 1 && !(fl & G_TRAIL)) {
        o << "  return sl == " << u32(s0.len) << " && " << seg_expr(s0, "0u", true) << ";\n}\n";
        return;
      }
      o << "  if (!" << seg_expr(s0, "0u", true) << ") return false;\n";
      o << "  pos = " << u32(s0.len) << ";\n";
      i0 = 1;
    }
    if (!(fl & G_TRAIL)) {
      const GSeg& st = segs[n - 1];
      o << "  if (end < pos + " << u32(st.len) << ") return false;\n";
      o << "  if (!" << seg_expr(st, "end - " + u32(st.len), false) << ") return false;\n";
      o << "  end -= " << u32(st.len) << ";\n";
      i1 = n - 1;
    }
    for (uint32_t i = i0; i < i1; i++) {
      const GSeg& sg = segs[i];
      // leftmost occurrence of the segment in [pos, end): candidates are the
      // positions of its first literal byte, found 4 bytes at a time (SWAR
      // zero-byte test, exact: it never misses a match, false candidates are
      // rejected by the full word compare)
      int32_t j = -1;
      uint32_t cbyte = 0;
      for (uint32_t q = 0; q < sg.len && j < 0; q++) {
        const GWord& gw = ps.gwords[sg.wfirst + q / 4];
        if ((gw.mask >> (8 * (q % 4))) & 0xFFu) {
          j = (int32_t)q;
          cbyte = (gw.w >> (8 * (q % 4))) & 0xFFu;
        }
      }
      if (j < 0) {  // all-'?' segment: plain scan
        o << "  { bool found = false;\n"
          << "    for (uint32_t k = pos; k + " << u32(sg.len) << " <= end; k++)\n"
          << "      if (" << seg_expr(sg, "k", false) << ") { pos = k + " << u32(sg.len) << "; found = true; break; }\n"
          << "    if (!found) return false; }\n";
        continue;
      }
      o << "  { if (end < pos + " << u32(sg.len) << ") return false;\n"
        << "    const uint32_t plo = pos + " << u32(j) << ", phi = end - " << u32(sg.len) << " + " << u32(j) << ";\n"
        << "    bool found = false;\n"
        << "    for (uint32_t wa = plo >> 2; wa <= (phi >> 2) && !found; wa++) {\n"
        << "      const uint32_t w = base[wa] ^ " << hex32(cbyte * 0x01010101u) << ";\n"
        << "      uint32_t m = (w - 0x01010101u) & ~w & 0x80808080u;\n"
        << "      while (m) {\n"
        << "        const uint32_t p = wa * 4u + ((uint32_t)__builtin_ctz(m) >> 3); m &= m - 1u;\n"
        << "        if (p < plo || p > phi) continue;\n"
        << "        const uint32_t k = p - " << u32(j) << ";\n"
        << "        if (" << seg_expr(sg, "k", false) << ") { pos = k + " << u32(sg.len) << "; found = true; break; }\n"
        << "      }\n"
        << "    }\n"
        << "    if (!found) return false; }\n";
    }
    o << "  (void)pos; (void)end;\n  return true;\n}\n";
  }

  // ---------------------------------------------------------------- kvj_ptab globs (register path)
  // In kvj_ptab a value's bytes (<= 64) sit in 16 registers `w` (plus an LDS copy
  // `lw` for reads at a per-lane offset). A middle segment's candidates are the
  // positions of one of its literal bytes, taken from a 64-bit byte mask `bm[slot]`
  // that the row computes once per distinct byte (kv_bmask: straight-line SWAR over
  // the 16 words) and that every glob of the row sharing that byte reuses; the
  // leftmost verified candidate at or after `pos` wins (the same leftmost-occurrence
  // search as glob_fn, without the per-lane word loop that made the kernel
  // scalar-issue bound: 2.1e8 SALU against 6.0e7 VALU instructions per pass on C2).
  std::map<uint32_t, uint32_t> bslot;  // byte -> slot of bm[]
  std::map<uint32_t, std::set<uint32_t>> glob_bytes;  // atom -> bytes its middle segments search
  std::set<std::pair<char, uint32_t>> qglobs_done, qatoms_done, qpreds_done;
  static constexpr uint32_t kMaxBSlots = 48;
  // register-path variants: values of <= 64 bytes (16 words, 64-bit masks, prefix q_) and
  // of <= 128 bytes (32 words, two-word masks KvM2, prefix r_); the mask helpers
  // (kv_mrange / kv_mctz / kv_mpop) are overloaded on the mask type
  struct QV {
    char pfx;
    const char* mt;   // mask type
    const char* bmk;  // mask builder
    uint32_t words;
  };
  static constexpr QV kQ64{'q', "uint64_t", "kv_bmask", 16}, kQ128{'r', "KvM2", "kv_bmask2", 32};

  // first literal byte of segment `sg` and its offset in the segment (-1: all '?')
  std::pair<int32_t, uint32_t> seg_key(const GSeg& sg) const {
    for (uint32_t q = 0; q < sg.len; q++) {
      const GWord& gw = ps.gwords[sg.wfirst + q / 4];
      if ((gw.mask >> (8 * (q % 4))) & 0xFFu) return {(int32_t)q, (gw.w >> (8 * (q % 4))) & 0xFFu};
    }
    return {-1, 0u};
  }

  std::string qsig(const QV& v) const {
    return std::string("(const Val* __restrict__ V, const uint8_t* __restrict__ S, const uint32_t* w, const uint32_t* lw, const ") +
           v.mt + "* bm, const uint8_t* __restrict__ pstr, uint32_t type, const Node& n)";
  }

  void qglob_fn(uint32_t ai, const QV& v) {
    if (!qglobs_done.insert({v.pfx, ai}).second) return;
    const Atom& A = ps.atoms[ai];
    std::ostringstream& q = o;
    // branch-free: every step folds into `ok` (indices clamped so a failed step reads in
    // bounds); only a segment whose leftmost candidate fails verification loops over the rest
    q << "__device__ __forceinline__ bool " << v.pfx << "_glob_" << ai
      << "(const uint32_t* w, const uint32_t* lw, const " << v.mt << "* bm, uint32_t sl, bool ascii, "
         "const uint8_t* __restrict__ pstr) {\n";
    const uint32_t fl = A.gflags;
    if (fl & G_ALL) { q << "  return true;\n}\n"; return; }
    if (fl & G_EMPTY) { q << "  return sl == 0u;\n}\n"; return; }
    if (fl & G_HASQ)
      q << "  if (!ascii) return kv_glob(pstr + " << u32(A.s_off) << ", " << u32(A.s_len & 0x7FFFFFFFu)
        << ", (const uint8_t*)lw, sl);\n";
    const uint32_t n = A.gcount;
    const GSeg* segs = ps.gsegs.data() + A.gfirst;
    uint32_t i0 = 0, i1 = n;
    q << "  const uint32_t* base = lw;\n  bool ok = sl >= " << u32(A.gmin) << ";\n  uint32_t pos = 0u, end = sl;\n";
    auto prefix_expr = [&](const GSeg& sg) {  // aligned compare at 0 from the registers
      std::ostringstream e;
      e << "((0u";
      for (uint32_t i = 0; i < (sg.len + 3) / 4; i++) {
        const GWord& g = ps.gwords[sg.wfirst + i];
        if (g.mask) e << " | ((w[" << i << "] ^ " << hex32(g.w) << ") & " << hex32(g.mask) << ")";
      }
      e << ") == 0u)";
      return e.str();
    };
    if (!(fl & G_LEAD)) {
      const GSeg& s0 = segs[0];
      if (n == 1 && !(fl & G_TRAIL)) {
        q << "  return (sl == " << u32(s0.len) << ") & " << prefix_expr(s0) << ";\n}\n";
        return;
      }
      q << "  ok &= " << prefix_expr(s0) << ";\n  pos = " << u32(s0.len) << ";\n";
      i0 = 1;
    }
    if (!(fl & G_TRAIL)) {
      const GSeg& st = segs[n - 1];
      q << "  { const bool fit_ = ok & (end >= pos + " << u32(st.len) << ");\n"
        << "    const uint32_t ks_ = fit_ ? end - " << u32(st.len) << " : 0u;\n"
        << "    ok = fit_ & " << seg_expr(st, "ks_", false) << ";\n"
        << "    end = ks_; }\n";
      i1 = n - 1;
    }
    for (uint32_t i = i0; i < i1; i++) {
      const GSeg& sg = segs[i];
      const auto [j, cb] = seg_key(sg);
      if (j < 0) {  // all-'?' segment: its leftmost occurrence is pos itself
        q << "  ok &= end >= pos + " << u32(sg.len) << ";\n  pos += " << u32(sg.len) << ";\n";
        continue;
      }
      auto it = bslot.find(cb);
      if (it == bslot.end() && bslot.size() < kMaxBSlots) it = bslot.emplace(cb, (uint32_t)bslot.size()).first;
      const std::string mask =
          it != bslot.end() ? "bm[" + u32(it->second) + "]" : std::string(v.bmk) + "(w, " + hex32(cb * 0x01010101u) + ")";
      if (it != bslot.end()) glob_bytes[ai].insert(cb);
      // candidates p in [plo, phi] (phi < 4 * words: end <= sl and j < len)
      q << "  { ok &= end >= pos + " << u32(sg.len) << ";\n"
        << "    const uint32_t plo = ok ? pos + " << u32(j) << " : 0u, phi = ok ? end - " << u32(sg.len) << " + " << u32(j)
        << " : 0u;\n"
        << "    " << v.mt << " cm = kv_mrange(" << mask << ", plo, phi, ok);\n"
        << "    uint32_t kf = kv_mnz(cm) ? kv_mctz(cm) - " << u32(j) << " : 0u;\n"
        << "    bool found = kv_mnz(cm) & " << seg_expr(sg, "kf", false) << ";\n"
        << "    cm = kv_mpop(cm);\n"
        << "    if (!found && kv_mnz(cm)) {\n"
        << "      while (kv_mnz(cm)) {\n"
        << "        const uint32_t k = kv_mctz(cm) - " << u32(j) << "; cm = kv_mpop(cm);\n"
        << "        if (" << seg_expr(sg, "k", false) << ") { kf = k; found = true; break; }\n"
        << "      }\n"
        << "    }\n"
        << "    ok &= found;\n"
        << "    pos = kf + " << u32(sg.len) << "; }\n";
    }
    q << "  (void)pos; (void)end; (void)base;\n  return ok;\n}\n";
  }

  void qatom_fn(uint32_t ai, const QV& v) {
    if (!qatoms_done.insert({v.pfx, ai}).second) return;
    const Atom& A = ps.atoms[ai];
    atom_fn(ai);
    if (A.kind == AT_GLOB_E || A.kind == AT_GLOB_N) qglob_fn(ai, v);
    const std::string g = std::string(1, v.pfx) + "_glob_" + std::to_string(ai);
    o << "__device__ __forceinline__ bool " << v.pfx << "_atom_" << ai << qsig(v) << " {\n";
    switch (A.kind) {
      case AT_GLOB_E:
        o << "  const bool r = " << g << "(w, lw, bm, n.c & NC_LEN_MASK, (n.c & NC_ASCII_E) != 0u, pstr);\n"
          << "  return (type != NT_MAP) & (type != NT_ARR) & (type != NT_NULL) & " << (A.op == CO_NE ? "!r" : "r") << ";\n";
        break;
      case AT_GLOB_N:
        o << "  if (type != NT_FLOAT && type != NT_MAP && type != NT_ARR && type != NT_BOOL && type != NT_NULL)\n"
          << "    return " << g << "(w, lw, bm, n.c & NC_LEN_MASK, (n.c & NC_ASCII_E) != 0u, pstr);\n"
          << "  return g_atom_" << ai << "(V, S, (const uint8_t*)lw, pstr, type, n);\n";
        break;
      default:
        o << "  return g_atom_" << ai << "(V, S, (const uint8_t*)lw, pstr, type, n);\n";
        break;
    }
    o << "}\n";
  }

  // the row's predicates on the register copy; non-string predicates are the g_pred ones
  void qpred_fn(uint32_t pi, const QV& v) {
    if (!qpreds_done.insert({v.pfx, pi}).second) return;
    const Pred& pr = ps.preds[pi];
    if (pr.kind == PK_STRING)
      for (uint32_t a = pr.first; a < pr.first + pr.count; a++) {
        const Alt& al = ps.alts[a];
        for (uint32_t c = al.first; c < al.first + al.count; c++) {
          qatom_fn(ps.conjs[c].a0, v);
          if (ps.conjs[c].kind != CJ_ATOM) qatom_fn(ps.conjs[c].a1, v);
        }
      }
    o << "__device__ __forceinline__ bool " << v.pfx << "_pred_" << pi << qsig(v) << " {\n";
    if (pr.kind != PK_STRING) {
      o << "  return g_pred_" << pi << "(V, S, (const uint8_t*)lw, pstr, type, n);\n}\n";
      return;
    }
    // every alternative and conjunct evaluated (straight-line atoms), combined without branches
    o << "  return false";
    for (uint32_t a = pr.first; a < pr.first + pr.count; a++) {
      const Alt& al = ps.alts[a];
      o << "\n    | (true";
      for (uint32_t c = al.first; c < al.first + al.count; c++) {
        const Conj& cj = ps.conjs[c];
        auto call = [&](uint32_t at) {
          return std::string(1, v.pfx) + "_atom_" + std::to_string(at) + "(V, S, w, lw, bm, pstr, type, n)";
        };
        if (cj.kind == CJ_INRANGE) o << " & (" << call(cj.a0) << " & " << call(cj.a1) << ")";
        else if (cj.kind == CJ_NOTINRANGE) o << " & (" << call(cj.a0) << " | " << call(cj.a1) << ")";
        else o << " & " << call(cj.a0);
      }
      o << ")";
    }
    o << ";\n}\n";
  }

  // bytes whose masks the q_pred / r_pred of `pi` reads
  void pred_bytes(uint32_t pi, std::set<uint32_t>* out) {
    const Pred& pr = ps.preds[pi];
    if (pr.kind != PK_STRING) return;
    for (uint32_t a = pr.first; a < pr.first + pr.count; a++) {
      const Alt& al = ps.alts[a];
      for (uint32_t c = al.first; c < al.first + al.count; c++) {
        for (uint32_t at : {ps.conjs[c].a0, ps.conjs[c].kind != CJ_ATOM ? ps.conjs[c].a1 : ps.conjs[c].a0}) {
          auto it = glob_bytes.find(at);
          if (it != glob_bytes.end()) out->insert(it->second.begin(), it->second.end());
        }
      }
    }
  }

  // ---------------------------------------------------------------- atoms / predicates
  void atom_fn(uint32_t ai) {
    if (!atoms_done.insert(ai).second) return;
    const Atom& A = ps.atoms[ai];
    if (A.kind == AT_GLOB_E || A.kind == AT_GLOB_N) glob_once(ai);
    o << "__device__ __forceinline__ bool g_atom_" << ai
      << "(const Val* __restrict__ V, const uint8_t* __restrict__ S, const uint8_t* __restrict__ E, "
         "const uint8_t* __restrict__ pstr, uint32_t type, const Node& n) {\n";
    switch (A.kind) {
      case AT_FALSE: o << "  return false;\n"; break;
      case AT_GLOB_E:
        o << "  if (type == NT_MAP || type == NT_ARR || type == NT_NULL) return false;\n"
          << "  const bool r = g_glob_" << ai << "(E, n.c & NC_LEN_MASK, (n.c & NC_ASCII_E) != 0u, pstr);\n"
          << "  return " << (A.op == CO_NE ? "!r" : "r") << ";\n";
        break;
      case AT_GLOB_N:
        o << "  if (type == NT_MAP || type == NT_ARR || type == NT_BOOL) return false;\n"
          << "  if (type == NT_NULL) return g_glob_" << ai << "(S, 1u, true, pstr);\n"
          << "  if (type != NT_FLOAT) return g_glob_" << ai << "(E, n.c & NC_LEN_MASK, (n.c & NC_ASCII_E) != 0u, pstr);\n"
          << "  const Val& v = V[n.a];\n"
          << "  return g_glob_" << ai << "(S + v.n_off, v.n_len, (v.flags & VF_ASCII_N) != 0u, pstr);\n";
        break;
      default: {  // AT_QCMP
        o << "  if (type == NT_MAP || type == NT_ARR || type == NT_BOOL) return false;\n"
          << "  int r;\n"
          << "  if (type == NT_NULL) {\n"
          << "    r = q_cmp(VF_Q_ZERO, 0, 0ull, 0ull, " << u32(A.q_flags) << ", " << A.q_exp << ", " << u64(A.q_hi) << ", "
          << u64(A.q_lo) << ");\n"
          << "  } else {\n"
          << "    const Val& v = V[n.a];\n"
          << "    if (!(v.flags & VF_Q_VALID)) return false;\n"
          << "    r = q_cmp(v.flags, v.q_exp, v.q_hi, v.q_lo, " << u32(A.q_flags) << ", " << A.q_exp << ", " << u64(A.q_hi)
          << ", " << u64(A.q_lo) << ");\n"
          << "  }\n"
          << "  return cmp_ok(" << u32(A.op) << ", r);\n";
        break;
      }
    }
    o << "}\n";
  }

  void pred_fn(uint32_t pi) {
    if (!preds_done.insert(pi).second) return;
    const Pred& pr = ps.preds[pi];
    if (pr.kind == PK_STRING) {
      for (uint32_t a = pr.first; a < pr.first + pr.count; a++) {
        const Alt& al = ps.alts[a];
        for (uint32_t c = al.first; c < al.first + al.count; c++) {
          atom_fn(ps.conjs[c].a0);
          if (ps.conjs[c].kind != CJ_ATOM) atom_fn(ps.conjs[c].a1);
        }
      }
    }
    // E: the validateString (e-form) bytes of the value, S + n.b in the rule kernels (a staged copy in kvj_ptab)
    o << "__device__ __forceinline__ bool g_pred_" << pi
      << "(const Val* __restrict__ V, const uint8_t* __restrict__ S, const uint8_t* __restrict__ E, "
         "const uint8_t* __restrict__ pstr, uint32_t type, const Node& n) {\n";
    switch (pr.kind) {
      case PK_BOOL: o << "  return type == NT_BOOL && ((n.c & NC_BOOLV) != 0u) == " << (pr.flags ? "true" : "false") << ";\n"; break;
      case PK_FLOAT:
        o << "  if (type == NT_INT) return " << (pr.flags ? "V[n.a].i == " + i64(pr.fi) : std::string("false")) << ";\n"
          << "  if (type == NT_FLOAT) return V[n.a].f == " << f64(pr.f) << ";\n"
          << "  if (type == NT_STR) { const Val& v = V[n.a]; return (v.flags & VF_PF_OK) && v.f == " << f64(pr.f) << "; }\n"
          << "  return false;\n";
        break;
      case PK_NIL:
        o << "  if (type == NT_NULL) return true;\n"
          << "  if (type == NT_MAP || type == NT_ARR) return false;\n"
          << "  return (n.c & NC_NILLIKE) != 0u;\n";
        break;
      case PK_MAPTYPE: o << "  return type == NT_MAP;\n"; break;
      case PK_STRING: {
        for (uint32_t a = pr.first; a < pr.first + pr.count; a++) {
          const Alt& al = ps.alts[a];
          o << "  if (true";
          for (uint32_t c = al.first; c < al.first + al.count; c++) {
            const Conj& cj = ps.conjs[c];
            auto call = [&](uint32_t at) { return "g_atom_" + std::to_string(at) + "(V, S, E, pstr, type, n)"; };
            if (cj.kind == CJ_INRANGE) o << " && (" << call(cj.a0) << " && " << call(cj.a1) << ")";
            else if (cj.kind == CJ_NOTINRANGE) o << " && (" << call(cj.a0) << " || " << call(cj.a1) << ")";
            else o << " && " << call(cj.a0);
          }
          o << ") return true;\n";
        }
        o << "  return false;\n";
        break;
      }
      default: o << "  return false;\n"; break;
    }
    o << "}\n";
  }

  // memo slot of leaf predicate `pi` (one per predicate for single rules, assigned on first use)
  uint32_t slot_for(uint32_t pi) {
    auto it = pslot.find(pi);
    if (it != pslot.end()) return it->second;
    const uint32_t slot = (uint32_t)mpreds.size();
    mpreds.push_back(pi);
    pslot[pi] = slot;
    return slot;
  }
  // consecutive memo slots inside one table word for the leaf predicates of a rule group's
  // members (member j = bit base + j; a word's unused tail is padded with the first predicate)
  uint32_t group_slots(const std::vector<uint32_t>& preds) {
    if ((mpreds.size() % 32) + preds.size() > 32)
      while (mpreds.size() % 32) mpreds.push_back(preds[0]);
    const uint32_t base = (uint32_t)mpreds.size();
    for (uint32_t p : preds) mpreds.push_back(p);
    return base;
  }

  // Position classes of every leaf predicate: the projection-trie node of each
  // cursor is followed through the rule program (KEY: slot child, LOOP/EXIST/
  // INDEX: element node, keep-all scans: leaf-only positions, KEYGLOB: unknown),
  // and a predicate gets the class bit of every position it tests (its cursor,
  // and the element position when the value is an array). Ingest marks each
  // value with the class bits of the positions holding it (Val::cls), so the
  // table bit of (pred, value) is computed exactly when some node could read it.
  std::map<uint32_t, uint32_t> pmask;
  void leaf_classes(uint32_t ri) {
    // per cursor depth: projection-trie node (child lookups) and position id (value classes,
    // kv_pos_elem); -2 = unknown (every class)
    std::vector<int32_t> tn(8, -2), pos(8, -2);
    tn[0] = 0;
    pos[0] = 0;
    auto cls = [&](int32_t p) -> uint32_t { return p == -2 ? 0xFFFFFFFFu : kv_tcls(p); };
    auto epos = [&](int32_t p) -> int32_t { return p == -2 ? -2 : kv_pos_elem(p, 0); };
    for (uint32_t pc = ps.rules[ri].prog; pc < ps.prog.size(); pc++) {
      const Inst& in = ps.prog[pc];
      const uint32_t op = in.op & 0xFF, d = (in.op >> 8) & 0xFF, aux = (in.op >> 16) & 0xFF;
      if (op == OP_DONE) break;
      if (d + 2 > tn.size()) { tn.resize(d + 2, -2); pos.resize(d + 2, -2); }
      switch (op) {
        case OP_KEY:
        case OP_KEYV: {
          const int32_t t = tn[d];
          if (aux & AUX_SCAN) {  // children of keep-all maps: leaf-only positions
            tn[d + 1] = t == -2 ? -2 : -1;
            pos[d + 1] = t == -2 ? -2 : -1;
          } else if (t >= 0 && in.a < ps.trie.nodes[t].slot_keys.size()) {
            tn[d + 1] = pos[d + 1] = (int32_t)ps.trie.nodes[t].kids.at(ps.trie.nodes[t].slot_keys[in.a]);
          } else {
            tn[d + 1] = pos[d + 1] = -2;
          }
          break;
        }
        case OP_KEYGLOB: {  // a resolved label / annotation key: a child of a keep-all map (pos -1)
          const int32_t t = tn[d];
          tn[d + 1] = pos[d + 1] = t >= 0 && ps.trie.nodes[t].keep_all ? -1 : -2;
          break;
        }
        case OP_LOOP_BEGIN:
        case OP_EXIST_BEGIN:
        case OP_INDEX:
          tn[d + 1] = tn[d] >= 0 ? ps.trie.nodes[tn[d]].elem : tn[d];
          pos[d + 1] = epos(pos[d]);
          break;
        case OP_LEAF: pmask[in.a] |= cls(pos[d]) | cls(epos(pos[d])); break;
        default: break;
      }
    }
  }

  // kvj_ptab: one lane per distinct scalar Val of the batch; evaluates every memo
  // slot's predicate on the scalar node ingest builds for that value
  // (kvingest.cpp scalar(): a = val id, b = e_off, c = e_len | NC_* flags)
  // kernel texts (name, source): each one is compiled as its own hiprtc program
  // after the helpers every kernel may use (Gen::o, the common part)
  std::vector<std::pair<std::string, std::string>> kernels;
  struct KernelText {  // redirects Gen::o into a kernel's own text for its lifetime
    Gen& g;
    std::string name;
    std::ostringstream saved;
    KernelText(Gen& gg, std::string n) : g(gg), name(std::move(n)) { std::swap(g.o, saved); }
    ~KernelText() {
      std::swap(g.o, saved);
      g.kernels.push_back({name, saved.str()});
    }
  };

  // the slots `ks` by predicate (a predicate holds several slots when rule groups share it):
  // predicate -> (table word -> bits), in first-slot order
  std::vector<std::pair<uint32_t, std::map<uint32_t, uint32_t>>> pred_words(const std::vector<uint32_t>& ks) const {
    std::vector<std::pair<uint32_t, std::map<uint32_t, uint32_t>>> out;
    std::map<uint32_t, size_t> at;
    for (uint32_t k : ks) {
      auto it = at.find(mpreds[k]);
      if (it == at.end()) {
        it = at.emplace(mpreds[k], out.size()).first;
        out.push_back({mpreds[k], {}});
      }
      out[it->second].second[k / 32] |= 1u << (k % 32);
    }
    return out;
  }

  // predicates per kvj_ptab thread: all of them (one grid row)
  uint32_t ptab_row_out() const { return std::max<uint32_t>(1u, (uint32_t)mpreds.size()); }

  void ptab_kernel() {
    // register-path predicates (helpers: emitted before the kernel text)
    for (uint32_t k = 0; k < mpreds.size(); k++) qpred_fn(mpreds[k], kQ64);
    for (uint32_t k = 0; k < mpreds.size(); k++) qpred_fn(mpreds[k], kQ128);
    KernelText kt(*this, "kvj_ptab");
    const uint32_t nw = (uint32_t)((mpreds.size() + 31) / 32);
    auto pm = [&](uint32_t k) { auto it = pmask.find(mpreds[k]); return it == pmask.end() ? 0xFFFFFFFFu : it->second; };
    // predicates grouped by position class: a value runs the groups its class bits select
    // (Vals are numbered by class, kvingest.cpp val_order_key, so the tests are uniform in
    // most waves); one thread per value writes every word of its table column
    std::map<uint32_t, std::vector<uint32_t>> groups;  // class mask -> memo slots
    uint32_t all = 0;
    for (uint32_t k = 0; k < mpreds.size(); k++) {
      groups[pm(k)].push_back(k);
      all |= pm(k);
    }
    o << "extern \"C\" __global__ __launch_bounds__(KV_WG) void kvj_ptab(const DevPS* __restrict__ Pp, "
         "const Val* __restrict__ V, const uint8_t* __restrict__ S, uint32_t NV, uint32_t* __restrict__ PT) {\n"
      << "  const uint32_t v = blockIdx.x * KV_WG + threadIdx.x;\n"
      << "  const uint32_t NP = NV + KV_PTAB_PSEUDO;  // table pitch\n"
      << "  if (v >= NP) return;\n"
      << "  uint32_t w[" << nw << "] = {};\n"
      << "  if (v >= NV) {  // pseudo columns: every predicate on a null / map / array node\n"
      << "    const uint8_t* __restrict__ pstr = Pp->pstr;\n"
      << "    const uint32_t type = v == NV ? NT_NULL : v == NV + 1u ? NT_MAP : NT_ARR;\n"
      << "    const Node n{type, 0u, 0u, 0u};\n";
    {
      std::vector<uint32_t> all_k(mpreds.size());
      for (uint32_t k = 0; k < mpreds.size(); k++) all_k[k] = k;
      for (const auto& [pi, wb] : pred_words(all_k)) {
        o << "    if (g_pred_" << pi << "(V, S, S, pstr, type, n)) {";
        for (const auto& [wi, bits] : wb) o << " w[" << wi << "] |= " << u32(bits) << ";";
        o << " }\n";
      }
    }
    for (uint32_t i = 0; i < nw; i++) o << "    PT[(size_t)" << i << "u * NP + v] = w[" << i << "];\n";
    o << "    return;\n  }\n"
      << "  const uint32_t vc = V[v].cls;\n"
      << "  if (vc & " << u32(all) << ") {\n"
      << "  const uint8_t* __restrict__ pstr = Pp->pstr;\n"
      << "  const Val& val = V[v];\n"
      << "  const uint32_t type = val.type;\n"
      << "  Node n{type, v, val.e_off, val.e_len};\n"
      << "  if (val.flags & VF_ASCII_E) n.c |= NC_ASCII_E;\n"
      << "  if (val.flags & VF_BOOLV) n.c |= NC_BOOLV;\n"
      << "  if (val.flags & VF_NILLIKE) n.c |= NC_NILLIKE;\n"
      << "  const uint8_t* __restrict__ E = S + val.e_off;\n"
      // values of <= 64 (<= 128) bytes: 16 (32) words in registers (loads clamped to the
      // word after the string, which the word-wise readers already touch) and an LDS copy of
      // 33 words (odd stride: no bank conflicts) for the reads at a per-lane offset; values
      // are numbered by length bucket within their class, so a wave runs one of the paths
      << "  __shared__ uint32_t lds_e[KV_WG * 33];\n"
      << "  uint32_t* lw = lds_e + threadIdx.x * 33u;\n";
    for (const QV* qv : {&kQ64, &kQ128}) {
      const uint32_t W = qv->words;
      o << (W == 16 ? "  if (val.e_len <= 64u) {\n" : "  } else if (val.e_len <= 128u) {\n")
        << "    uint32_t sw[" << W << "];\n"
        << "    const uint32_t* __restrict__ src = (const uint32_t*)E;\n"
        << "    const uint32_t lastw = (val.e_len + 3u) >> 2;\n"
        << "#pragma unroll\n"
        << "    for (uint32_t i = 0; i < " << W << "u; i++) sw[i] = src[i < lastw ? i : lastw];\n"
        << "#pragma unroll\n"
        << "    for (uint32_t i = 0; i < " << W << "u; i++) lw[i] = sw[i];\n"
        << "    lw[" << W << "] = src[lastw];\n"
        // byte masks only over the words the wave's values occupy
        << "    const uint32_t nwu_ = kv_wave_words(lastw, " << W << "u);\n";
      for (auto& [m, ks] : groups) {
        std::set<uint32_t> bytes;
        for (uint32_t k : ks) pred_bytes(mpreds[k], &bytes);
        o << "    if (vc & " << u32(m) << ") {\n";
        if (!bytes.empty()) {
          o << "      " << qv->mt << " bm[" << kMaxBSlots << "];\n";
          for (uint32_t c : bytes)
            o << "      bm[" << bslot.at(c) << "] = " << qv->bmk << "_n(sw, " << hex32(c * 0x01010101u) << ", nwu_);\n";
        } else {
          o << "      const " << qv->mt << "* bm = nullptr;\n";
        }
        for (const auto& [pi, wb] : pred_words(ks)) {  // each predicate once, into every slot it has
          o << "      { const bool p_ = " << qv->pfx << "_pred_" << pi << "(V, S, sw, lw, bm, pstr, type, n);";
          for (const auto& [wi, bits] : wb) o << " w[" << wi << "] |= p_ ? " << u32(bits) << " : 0u;";
          o << " }\n";
        }
        o << "    }\n";
      }
    }
    o << "  } else {\n";
    for (auto& [m, ks] : groups) {
      o << "    if (vc & " << u32(m) << ") {\n";
      for (const auto& [pi, wb] : pred_words(ks)) {
        o << "      if (g_pred_" << pi << "(V, S, E, pstr, type, n)) {";
        for (const auto& [wi, bits] : wb) o << " w[" << wi << "] |= " << u32(bits) << ";";
        o << " }\n";
      }
      o << "    }\n";
    }
    o << "  }\n  }\n";
    for (uint32_t i = 0; i < nw; i++) o << "  PT[(size_t)" << i << "u * NP + v] = w[" << i << "];\n";
    o << "}\n\n";
  }

  // dynamic leaves (pattern variables, kvvars.cpp): the generic predicate evaluator on the
  // batch table, out of line (one copy per program; inlined per leaf it multiplies the
  // kernel's code and its compile time)
  bool dleaf_done = false;
  void dleaf_fn() {
    if (dleaf_done) return;
    dleaf_done = true;
    o << "__device__ __forceinline__ bool g_dleaf_0(const DevBatch& B, const Node* __restrict__ N, uint32_t dp, "
         "const Node& vn) { return kv_dleaf_impl(B, N, dp, vn); }\n"
      << "__device__ __noinline__ bool kv_dleaf_impl(const DevBatch& B, const Node* __restrict__ N, uint32_t dp, Node vn) {\n"
      << "  const uint32_t vt = node_type(vn.kt);\n"
      << "  if (vt == NT_ARR) {\n"
      << "    for (uint32_t k = 0; k < vn.b; k++) if (!pred_node(*B.dps, B, N, dp, ni(vn.a + k))) return false;\n"
      << "    return true;\n  }\n"
      << "  return pred_eval(*B.dps, B, dp, vt, vn);\n}\n";
  }

  // ---------------------------------------------------------------- match / exclude
  // blk_ok(f) == !(MF_EMPTY) && doesResourceMatchConditionBlock(f) has no errors
  // (pkg/engine/utils.go:265-336); MF_EMPTY / MF_UI_FAIL are folded per launch
  // (user info), so they are read from P.fflags; every other criterion is static.
  std::set<uint32_t> blks_done;
  void blk_fn(uint32_t f) {
    if (!blks_done.insert(f).second) return;
    const MFilter& F = ps.filters[f];
    for (uint32_t a : ps.filter_name_atoms.at(f)) glob_once(a);  // before this function's text
    o << "__device__ __forceinline__ bool g_blk_" << f
      << "(const DevPS& P, const DevBatch& B, const Res* __restrict__ R, uint32_t rkind, uint32_t rflags) {\n"
      << "  if (sld(P.fflags + " << f << "u) & (MF_EMPTY | MF_UI_FAIL)) return false;\n";
    if (F.flags & MF_KINDS) {
      bool any_star = false;
      std::ostringstream k;
      k << "false";
      for (uint32_t i = F.kinds_first; i < F.kinds_first + F.kinds_count; i++) {
        const KindSpec& ks = ps.kinds[i];
        switch (ks.form) {
          case 3: any_star = true; break;
          case 0: k << " || rkind == " << u32(ks.kind); break;
          case 1: k << " || (rkind == " << u32(ks.kind) << " && R->version == " << u32(ks.version) << ")"; break;
          default:
            k << " || (R->group == " << u32(ks.group) << " && rkind == " << u32(ks.kind) << " && (R->version == "
              << u32(ks.version) << " || R->version == P.star_id))";
            break;
        }
      }
      if (!any_star) o << "  if (!(" << k.str() << ")) return false;\n";
    }
    // name / names: compiled word globs over the resource name (no calls)
    const std::vector<uint32_t>& na = ps.filter_name_atoms.at(f);
    auto name_glob = [&](uint32_t a) {
      return "g_glob_" + std::to_string(a) + "(B.bstr + R->name_off, R->name_len, (rflags & RF_NAME_ASCII) != 0u, P.pstr)";
    };
    size_t k = 0;
    if (F.flags & MF_NAME) o << "  if (!" << name_glob(na.at(k++)) << ") return false;\n";
    if (F.flags & MF_NAMES) {
      o << "  if (!(false";
      for (; k < na.size(); k++) o << " || " << name_glob(na[k]);
      o << ")) return false;\n";
    }
    // namespace globs, annotations, label selectors: bits of the pass's match tables (kv_mtab)
    if (F.flags & MF_NSS) o << "  if (!mt_bit(P.mt_ns, " << u32(F.nss_bit) << ", B.n_nsm, R->nsm)) return false;\n";
    if (F.flags & MF_ANN) o << "  if (!mt_bit(P.mt_ann, " << u32(F.ann_bit) << ", B.n_asets, R->aset)) return false;\n";
    if (F.flags & MF_SEL) o << "  if (!mt_bit(P.mt_sel, " << u32(F.sel) << ", B.n_lsets, R->lset)) return false;\n";
    if (F.flags & MF_NSSEL)
      o << "  if (!(rflags & (RF_KIND_NAMESPACE | RF_KIND_EMPTY)) && !((B.ns_bits[R->ns_index * B.ns_words + "
        << (F.nssel_bit / 32) << "u] >> " << (F.nssel_bit % 32) << "u) & 1u)) return false;\n";
    o << "  return true;\n}\n";
  }

  // rule_matches (kvdevfn.h) for one rule, with its filter list unrolled
  void match_fn(uint32_t ri) {
    const RuleRec& rr = ps.rules[ri];
    for (uint32_t f = rr.m_first; f < rr.m_first + rr.m_count; f++) blk_fn(f);
    for (uint32_t f = rr.x_first; f < rr.x_first + rr.x_count; f++) blk_fn(f);
    auto call = [&](uint32_t f) { return "g_blk_" + std::to_string(f) + "(P, B, R, rkind, rflags)"; };
    auto combine = [&](uint32_t mode, uint32_t first, uint32_t count) {
      std::ostringstream e;
      if (mode == 0 || count == 0) {
        e << call(first);
      } else {
        e << "(";
        for (uint32_t f = first; f < first + count; f++) e << (f > first ? (mode == 1 ? " || " : " && ") : "") << call(f);
        e << ")";
      }
      return e.str();
    };
    o << "__device__ __forceinline__ bool g_match_" << ri
      << "(const DevPS& P, const DevBatch& B, const Res* __restrict__ R, uint32_t rkind, uint32_t rflags) {\n"
      << "  if (!" << combine(rr.m_mode, rr.m_first, rr.m_count) << ") return false;\n"
      << "  return !" << combine(rr.x_mode, rr.x_first, rr.x_count) << ";\n}\n";
  }

  // ---------------------------------------------------------------- rule programs
  static uint32_t prog_end(const PolicySet& ps, uint32_t pc) {
    while ((ps.prog[pc].op & 0xFF) != OP_DONE) pc++;
    return pc;
  }

  // ================================================================ fused chunk kernels
  // All rules of a chunk run in one kernel body as interleaved sequential
  // programs. Rules never interact, so any interleaving that keeps each rule's
  // own op order is exact; the interleaving is chosen to share memory traffic:
  //  * cursor lookups whose path from the resource root (or from the element
  //    of a shared array loop) is known statically are hoisted: computed once
  //    (per kernel, or per loop iteration), just before the first rule that
  //    walks them, together with the 16-B node they land on;
  //  * every rule program is split at its top-level array loops into stages;
  //    at stage k the k-th loops of all rules iterating the same array
  //    (e.g. spec.containers) become ONE loop whose body runs each active
  //    rule's loop body for that element.
  // Per-rule registers: rs (resume pc between stages | ACTIVE bit, or FIN |
  // status once the rule's DONE ran), ek (error kind | flags << 4 | pattern
  // node << 8), loop indices of the raise (ei0..), anchor bitsets when used.
  static constexpr uint32_t FIN = 0x7F000000u, ACT = 0x80000000u;

  struct HVar { std::string idx, node; };  // hoisted cursor: node index var + Node var
  struct HoistTable {
    std::string prefix;
    std::map<std::string, HVar> vars;
    std::vector<std::string> code;  // one statement group per entry, dependency order
    std::set<std::string> words;    // hoisted table-word loads (Gen::pw)
    size_t flushed = 0;
    uint32_t n = 0;
    // path columns: the family its lookups read (-1: none, walk the node rows), the root token
    // of its exprs (an element family) and the cell-offset expression of its lane's column 0
    int fam = -1;
    std::string troot, cell0;
    std::string flush() {
      std::string s;
      for (; flushed < code.size(); flushed++) s += code[flushed];
      return s;
    }
  };

  struct RGen {  // per-rule generation state
    uint32_t ri = 0, b = 0, e = 0, maxd = 1;
    std::vector<std::pair<uint32_t, uint32_t>> loops;  // stage loops (LOOP_BEGIN pc, LOOP_END pc)
    std::vector<std::string> expr;                      // symbolic cursor per depth ("" = unknown)
    std::vector<HVar> hv;                               // hoisted vars per depth (when expr known)
    std::set<uint32_t> resume;                          // resume targets of later segments
    // targets past the segment being emitted, reached without / with a pending error
    std::set<uint32_t> seg_jumps, seg_err_jumps;
    // resume targets set by earlier stages and not consumed yet (the segment holding them lies
    // further on), reached without / with a pending error
    std::set<uint32_t> carry_ok, carry_err;
    // per stage loop k: the rule is "lean" there (its state is one bit of the block's stage-k
    // masks and a failing element decides its status at once), the status its post chain adds
    // to the error (flags) and whether that chain ends at the last anyPattern alternative
    std::vector<char> lean;
    std::vector<uint32_t> post_flags, skip_to, skip_flags;
    std::vector<char> post_alt, skip_alt;
    uint32_t q = 0;                                     // position in the block (mask bit, LDS row)
    bool uses_anchor = false, uses_keyglob = false;
    // rule group: the representative's program run once for all members (bit j of `al` = member
    // j alive on this lane); every error is decided where it is raised (kv_gfin)
    bool grp = false;
    uint32_t gn = 1, grow = 0, gsri = 0, gspn = 0;      // members, LDS row of member 0, steps
    std::vector<uint32_t> gri, gdpn;                    // member rule ids, pattern-node shifts
    std::map<uint32_t, uint32_t> gslot;                 // representative LEAF pc -> slot of member 0
    std::string gtab;                                   // member table (empty: arithmetic)
    bool gsite = false;                                 // site records (gl: its counter in the kernel)
    uint32_t gl = 0, gpre = 0;
    uint32_t max_level = 0;
    std::string s;                                      // "_<ri>"
  };

  HVar hoist(HoistTable& T, const std::string& pexpr, const HVar& p, uint32_t a, uint32_t aux) {
    const bool scan = (aux & AUX_SCAN) != 0;
    const std::string ex = pexpr + (scan ? "/k" : "/s") + std::to_string(a);
    auto it = T.vars.find(ex);
    if (it != T.vars.end()) return it->second;
    HVar h{T.prefix + "h" + std::to_string(T.n), T.prefix + "hn" + std::to_string(T.n)};
    T.n++;
    std::ostringstream c;
    const uint32_t j = T.fam >= 0 ? col_of((uint32_t)T.fam, T.fam == 0 ? ex : ex.substr(T.troot.size())) : kNoCol;
    if (j != kNoCol) {
      // the node from its path column (absent: the zero cell); the index only where the
      // lookup's presence (or a map's own index: wildcard keys) is asked for
      c << "  const Node " << h.node << " = kv_ldc(PC, PCB, " << T.cell0 << " + " << u32(j * KV_LANES) << ");\n"
        << "  const uint32_t " << h.idx << " = " << h.node << ".kt == 0u ? ABSENT : node_type(" << h.node
        << ".kt) == NT_MAP ? " << h.node << ".c : 0u;\n";
      T.code.push_back(c.str());
      T.vars.emplace(ex, h);
      return h;
    }
    c << "  uint32_t " << h.idx << " = ABSENT; Node " << h.node << "{0u, 0u, 0u, 0u};\n";
    if (scan) {
      c << "  if (node_type(" << p.node << ".kt) == NT_MAP) for (uint32_t q_ = 0u; q_ < " << p.node << ".b; q_++) { "
        << "const uint32_t c_ = ni(" << p.node << ".a + q_); const Node t_ = N[c_]; if (node_key(t_.kt) == " << u32(a)
        << ") { " << h.idx << " = c_; " << h.node << " = t_; break; } }\n";
    } else {
      // the loaded node passes through v_perm (keep / zero) instead of a select,
      // which the compiler would turn into a branch around a narrowed reload
      c << "  { const bool ok_ = node_type(" << p.node << ".kt) == NT_MAP && " << u32(a) << " < " << p.node << ".b; "
        << "const uint32_t c_ = ok_ ? ni(" << p.node << ".a + " << u32(a) << ") : 0u; const Node t_ = N[c_]; "
        << "const bool hit_ = ok_ && node_type(t_.kt) != NT_ABSENT; const uint32_t m_ = hit_ ? 0x07060504u : 0x0c0c0c0cu; "
        << h.idx << " = hit_ ? c_ : ABSENT; " << h.node << " = Node{__builtin_amdgcn_perm(t_.kt, 0u, m_), "
        << "__builtin_amdgcn_perm(t_.a, 0u, m_), __builtin_amdgcn_perm(t_.b, 0u, m_), __builtin_amdgcn_perm(t_.c, 0u, m_)}; }\n";
    }
    T.code.push_back(c.str());
    T.vars.emplace(ex, h);
    return h;
  }

  // a region of one rule's program: a segment between stage loops (kind 0) or
  // the body of a fused loop (kind 1)
  struct Region {
    int kind = 0;
    uint32_t rb = 0, re = 0;  // ops emitted: [rb, re)
    uint32_t jre = 0;         // local jump targets: [rb, jre)
    std::string se;           // segment end label
    std::string li0;          // level-0 loop index expression
    HoistTable* T = nullptr;  // hoist table for exprs rooted at this region's loop element
    std::string troot;        // expr root of T
  };

  HoistTable* gT = nullptr;  // global (root-derived) hoist table of the current chunk
  // per-rule histogram of a rule kernel from its statuses staged in LDS (one byte per rule and
  // lane, counted once when the kernel ends: kv_end_flush); otherwise (store_result2) with ballots
  // + LDS atomics per rule and wave
  bool hist_lds = false;

  void emit_region(RGen& g, const Region& R, std::ostringstream& wout) {
    struct OpOut {
      std::string code;
    };
    std::vector<OpOut> outs;
    const std::string& s = g.s;
    auto C = [&](uint32_t d) { return "c" + std::to_string(d) + s; };
    auto L = [&](uint32_t pc) { return "R" + std::to_string(g.ri) + "_L" + std::to_string(pc); };
    // err: the jump carries a pending error (a raise, or an error passed on by a scope end)
    auto jump = [&](uint32_t t, bool err = false) -> std::string {
      if (t >= R.rb && t < R.jre) return "goto " + L(t) + ";";
      if (R.kind == 0 && t >= R.jre) {
        g.resume.insert(t);
        (err ? g.seg_err_jumps : g.seg_jumps).insert(t);
        return "{ rs" + s + " = " + u32(t) + "; goto " + R.se + "; }";
      }
      throw std::runtime_error("kvjit: jump out of a fused region (rule " + std::to_string(g.ri) + ")");
    };
    auto finish = [&](const std::string& st) {
      if (R.kind != 0) throw std::runtime_error("kvjit: rule end inside a fused loop");
      return "{ rs" + s + " = FIN_ | " + st + "; goto " + R.se + "; }";
    };
    auto li = [&](uint32_t lv) { return lv == 0 && R.kind == 1 ? R.li0 : "li" + std::to_string(lv) + s; };
    const bool G = g.grp;
    const std::string al = "al" + s;
    // a group with no member left on this lane leaves the region
    auto gdone = [&]() -> std::string {
      if (R.kind == 0) return "{ rs" + s + " = FIN_ | ST_STORED_; goto " + R.se + "; }";
      return "goto " + L(R.re) + ";";
    };
    // members `m` of a group fail with the representative's error (kind, pn) raised here: their
    // status is the error's, carried statically through the scope ends to DONE (post_chain)
    auto gfin = [&](const std::string& m, uint32_t kind, uint32_t pn, uint32_t catch_pc) {
      const PostChain pcn = post_chain(g, catch_pc);
      if (!pcn.pure || pcn.alt) throw std::runtime_error("kvjit: impure error chain in rule group");
      std::string st;
      if (kind == E_CPU) st = "ST_CPU";
      else if (pcn.flags & (EF_COND | EF_GLOBAL)) st = "ST_SKIP";
      else {
        st = kind == E_LEN ? "ST_ERROR" : "ST_FAIL";
        if (g.uses_anchor) st = "((areg" + s + " & ~apres" + s + ") ? ST_ERROR : " + st + ")";
      }
      std::ostringstream r;
      r << "kv_gfin<" << (g.gtab.empty() ? "false" : "true") << ", " << (g.gsite ? "true" : "false")
        << ">(O, n_res, r, valid, " << m << ", " << st << ", " << u32(kind | (pcn.flags << 4) | (pn << 8));
      for (uint32_t lv = 0; lv < 4; lv++) r << ", " << (lv <= g.max_level ? li(lv) : std::string("0u"));
      r << ", s_w + " << u32(KV_ROW0 + g.grow * KV_RSTRIDE) << ", " << u32(g.grow) << ", " << (g.gtab.empty() ? std::string("nullptr") : g.gtab) << ", "
        << u32(g.gn) << ", " << u32(g.gri[0]) << ", " << u32(g.gsri) << ", " << u32(g.gspn) << ", "
        << (!g.gsite && g.gn >= gslot_members() ? "true" : "false");
      if (g.gsite) r << ", s_gc_ + " << u32(KV_RWAVES * g.gl) << ", " << u32(g.gpre);
      r << ");";
      return r.str();
    };
    auto raise = [&](uint32_t kind, uint32_t pn, uint32_t catch_pc) {
      if (pn >= (1u << 24)) throw std::runtime_error("kvjit: pattern node id exceeds 24 bits");
      if (G) return "{ " + gfin(al, kind, pn, catch_pc) + " " + al + " = 0u; " + gdone() + " }";
      std::ostringstream r;
      r << "{ ek" << s << " = " << u32(kind) << " | " << u32(pn << 8) << ";";
      for (uint32_t lv = 0; lv <= g.max_level && lv < 4; lv++) r << " ei" << lv << s << " = " << li(lv) << ";";
      if (g.uses_keyglob) r << " ekn" << s << " = kn" << s << ";";
      r << " " << jump(catch_pc, true) << " }";
      return r.str();
    };
    auto known = [&](uint32_t d) {
      if (d >= g.expr.size() || g.expr[d].empty()) return false;
      const std::string& ex = g.expr[d];
      return ex[0] == 'R' || (R.T && ex.compare(0, R.troot.size(), R.troot) == 0);
    };
    auto NODE = [&](uint32_t d) -> std::string {
      if (known(d)) return g.hv[d].node;
      return "N[" + C(d) + "]";
    };
    auto table_for = [&](uint32_t d) -> HoistTable* {
      const std::string& ex = g.expr[d];
      if (ex[0] == 'R') return gT;
      if (R.T && ex.compare(0, R.troot.size(), R.troot) == 0) return R.T;
      return nullptr;
    };
    auto set_unknown = [&](uint32_t from) {
      for (uint32_t x = from; x < g.expr.size(); x++) g.expr[x].clear();
    };
    // key lookup: returns the index expression; records the child cursor expr at d+1 when assign
    auto lookup = [&](uint32_t d, uint32_t a, uint32_t aux, bool assign) -> std::string {
      const uint32_t laux = aux & AUX_SCAN;
      HoistTable* T = known(d) ? table_for(d) : nullptr;
      if (T) {
        HVar h = hoist(*T, g.expr[d], g.hv[d], a, laux);
        if (assign) {
          set_unknown(d + 1);
          g.expr[d + 1] = g.expr[d] + (laux ? "/k" : "/s") + std::to_string(a);
          g.hv[d + 1] = h;
        }
        return h.idx;
      }
      if (assign) set_unknown(d + 1);
      return "lookup_op(N, " + C(d) + ", " + u32(a) + ", " + u32(laux) + ")";
    };
    const std::string ek = "ek" + s;
    const std::string kindof = "(" + ek + " & 15u)";

    for (uint32_t pc = R.rb; pc < R.re; pc++) {
      const Inst& in = ps.prog[pc];
      const uint32_t op = in.op & 0xFF, d = (in.op >> 8) & 0xFF, aux = (in.op >> 16) & 0xFF;
      const std::string cd = C(d), cn = C(d + 1);
      const uint32_t lv = aux & 3;
      const std::string L_lv = std::to_string(lv);
      std::ostringstream w;
      OpOut oo;  // this op's code and, for the fast-path guards, its exit condition / assignments
      w << L(pc) << ":;\n";
      switch (op) {
        case OP_MAPCHK:
        case OP_ARRCHK: {
          const char* t = op == OP_MAPCHK ? "NT_MAP" : "NT_ARR";
          if (known(d)) {
            w << "  if (node_type(" << NODE(d) << ".kt) != " << t << ") ";
          } else {
            w << "  if (" << cd << " == ABSENT || node_type(N[" << cd << "].kt) != " << t << ") ";
          }
          w << raise(op == OP_MAPCHK ? E_TYPE_MAP : E_TYPE_ARR, in.a, in.c) << "\n";
          break;
        }
        case OP_AREG: {
          const std::string bit = "(1ull << " + std::to_string(aux & 63) + ")";
          const bool h = known(d) && table_for(d);
          const std::string st = "  areg" + s + " |= " + bit + "; if (" + lookup(d, in.a, aux, false) + " != ABSENT) apres" +
                                 s + " |= " + bit + ";\n";
          w << st;
          if (h) {
          }
          break;
        }
        case OP_KEY: {
          const bool h = known(d) && table_for(d);
          std::string x = lookup(d, in.a, aux, true);
          w << "  " << cn << " = " << x << "; if (" << cn << " == ABSENT) " << jump(in.b) << "\n";
          if (h) {
          }
          break;
        }
        case OP_KEYV: {
          const bool h = known(d) && table_for(d);
          std::string x = lookup(d, in.a, aux, true);
          w << "  " << cn << " = " << x << ";\n";
          if (h) {
          }
          break;
        }
        case OP_KEYGLOB:
          if (G) throw std::runtime_error("kvjit: KEYGLOB in a rule group");
          set_unknown(d + 1);
          w << "  { uint32_t nd_; if (!keyglob_op(P, B, N, " << cd << ", " << u32(in.op) << ", " << u32(in.a) << ", "
            << u32(in.c) << ", &nd_, &kn" << s << ")) " << jump(in.b) << " " << cn << " = nd_; }\n";
          break;
        case OP_SCOPE_END:
          if (G) {  // groups carry no pending error (decided where raised)
            break;
          }
          if (in.c == 0) w << "  if (" << kindof << ") " << ek << " |= " << u32(aux << 4) << ";\n";
          else w << "  if (" << kindof << ") { " << ek << " |= " << u32(aux << 4) << "; " << jump(in.c, true) << " }\n";
          break;
        case OP_POS_END:
          if (G) throw std::runtime_error("kvjit: POS_END in a rule group");
          w << "  if (" << kindof << ") { if (" << ek << " & " << u32(EF_COND << 4) << ") " << ek << " = 0u; else "
            << jump(in.c, true) << " }\n";
          break;
        case OP_NEG: {
          const bool h = known(d) && table_for(d);
          const std::string x = lookup(d, in.a, aux, false);
          w << "  if (" << x << " != ABSENT) " << raise(E_NEG, in.b, in.c) << "\n";
          if (h) {
          }
          break;
        }
        case OP_STAR:
          if (known(d + 1)) {
            w << "  if (node_type(" << NODE(d + 1) << ".kt) == NT_NULL) ";
          } else {
            w << "  if (" << cn << " == ABSENT || node_type(N[" << cn << "].kt) == NT_NULL) ";
          }
          w << raise(E_STAR, in.b, in.c) << "\n";
          break;
        case OP_LEAF: {
          // one bit of the leaf's table word (a group: one bit per member, consecutive): hoisted
          // leaves read the word loaded (and, for an array, AND-ed over its elements) once per
          // region; others load it here
          const uint32_t slot = G ? g.gslot.at(pc) : slot_for(in.a);
          const uint32_t word = slot / 32;
          HoistTable* T = known(d) ? table_for(d) : nullptr;
          std::string wx;
          if (T) {
            const std::string hn = g.hv[d].node;
            wx = hn + "_w" + std::to_string(word);
            if (T->words.insert(wx).second)
              T->code.push_back("  const uint32_t " + wx + " = kv_leaf_word(P, N, " + hn + ", " + u32(word) + ");\n");
          } else {
            wx = "kv_leaf_word(P, N, (" + cd + " != ABSENT ? N[" + cd + "] : Node{0u, 0u, 0u, 0u}), " + u32(word) + ")";
          }
          if (G) {
            const uint32_t mask = g.gn >= 32 ? 0xFFFFFFFFu : (1u << g.gn) - 1u;
            w << "  { const uint32_t f_ = " << al << " & ~((" << wx << " >> " << u32(slot % 32) << ") & " << hex32(mask)
              << ");\n    if (f_) { " << gfin("f_", E_VALUE, in.b, in.c) << " " << al << " &= ~f_; if (!" << al << ") "
              << gdone() << " } }\n";
            if (T) {
            }
          } else {
            w << "  if (!(((" << wx << " >> " << u32(slot % 32) << ") & 1u) != 0u)) " << raise(E_VALUE, in.b, in.c) << "\n";
            if (T) {
            }
          }
          break;
        }
        case OP_VLEAF:  // pattern variables: the resource's substituted value (kvvars.cpp)
          if (G) throw std::runtime_error("kvjit: VLEAF in a rule group");
          if (known(d)) w << "  { const Node vn_ = " << NODE(d) << ";\n";
          else w << "  { Node vn_{0u, 0u, 0u, 0u}; if (" << cd << " != ABSENT) vn_ = N[" << cd << "];\n";
          dleaf_fn();
          w << "    if (!g_dleaf_0(B, N, B.dleaf[(size_t)" << u32(in.a) << " * n_res + r], vn_)) "
            << raise(E_VALUE, in.b, in.c) << " }\n";
          break;
        case OP_RAISE:
          w << "  " << raise(in.b, in.a, in.c) << "\n";
          break;
        case OP_EXISTCHK:
          if (known(d)) {
            w << "  if (node_type(" << NODE(d) << ".kt) != NT_ARR) ";
          } else {
            w << "  if (" << cd << " == ABSENT || node_type(N[" << cd << "].kt) != NT_ARR) ";
          }
          w << raise(E_EXIST_RESTYPE, in.a, in.c) << "\n";
          break;
        case OP_LENCHK:
          w << "  if (" << NODE(d) << ".b < " << u32(in.a) << ") " << raise(E_LEN, in.b, in.c) << "\n";
          if (known(d)) {
          }
          break;
        case OP_INDEX:
          w << "  " << cn << " = ni(" << NODE(d) << ".a + " << u32(in.a) << ");\n";
          if (known(d)) {
          }
          set_unknown(d + 1);
          break;
        case OP_LOOP_BEGIN:
          if (R.kind == 0 && lv == 0) {  // stage loop: hand over to the fused loop
            set_unknown(d + 1);
            w << "  { rs" << s << " = " << u32(in.a + 1) << " | ACT_; goto " << R.se << "; }\n";
            break;
          }
          [[fallthrough]];  // nested loop, per rule
        case OP_EXIST_BEGIN:
          if (G && op == OP_EXIST_BEGIN) throw std::runtime_error("kvjit: EXIST in a rule group");
          set_unknown(d + 1);
          w << "  { const Node an_ = " << NODE(d) << "; lf" << L_lv << s << " = an_.a; ll" << L_lv << s << " = an_.b; li"
            << L_lv << s << " = 0u;\n    if (an_.b == 0u) ";
          if (op == OP_LOOP_BEGIN) w << jump(in.a + 1);
          else w << raise(E_EXIST_FAIL, in.b, in.c);
          w << "\n    " << cn << " = ni(an_.a); }\n";
          break;
        case OP_LOOP_END:
          if (!G)  // groups carry no pending error
            w << "  if (" << kindof << ") { if (" << ek << " & " << u32(EF_COND << 4) << ") " << ek << " = 0u; else "
              << jump(in.c, true) << " }\n";
          w << "  if (li" << L_lv << s << " + 1u < ll" << L_lv << s << ") { li" << L_lv << s << "++; " << cn << " = ni(lf"
            << L_lv << s << " + li" << L_lv << s << "); " << jump(in.a + 1) << " }\n";
          set_unknown(d + 1);
          break;
        case OP_EXIST_END:
          if (G) throw std::runtime_error("kvjit: EXIST in a rule group");
          w << "  if (!" << kindof << ") " << jump(pc + 1) << "\n  " << ek << " = 0u;\n"
            << "  if (li" << L_lv << s << " + 1u < ll" << L_lv << s << ") { li" << L_lv << s << "++; " << cn << " = ni(lf"
            << L_lv << s << " + li" << L_lv << s << "); " << jump(in.a + 1) << " }\n"
            << "  " << raise(E_EXIST_FAIL, in.b, in.c) << "\n";
          set_unknown(d + 1);
          break;
        case OP_ALT_BEGIN:
          if (G) throw std::runtime_error("kvjit: anyPattern in a rule group");
          w << "  " << ek << " = 0u;";
          if (g.uses_anchor) w << " areg" << s << " = 0ull; apres" << s << " = 0ull;";
          w << "\n";
          break;
        case OP_ALT_END:
          if (G) throw std::runtime_error("kvjit: anyPattern in a rule group");
          w << "  if (" << kindof << " == 0u) " << finish("ST_PASS") << "\n  if (" << kindof << " == E_CPU) "
            << finish("ST_CPU") << "\n";
          if (in.b) w << "  " << finish("ST_FAIL") << "\n";
          else {
            w << "  " << ek << " = 0u;";
            if (g.uses_anchor) w << " areg" << s << " = 0ull; apres" << s << " = 0ull;";
            w << "\n";
          }
          break;
        case OP_DONE:  // the MatchPattern epilogue as one select chain (no per-lane branches)
          if (R.kind != 0) throw std::runtime_error("kvjit: rule end inside a fused loop");
          if (G) {  // the members alive here passed (no error: the anchor-key check does not apply)
            w << "  { rs" << s << " = FIN_ | ST_PASS; goto " << R.se << "; }\n";
            break;
          }
          w << "  { const uint32_t k_ = " << kindof << ";\n    rs" << s << " = FIN_ | (k_ == 0u ? ST_PASS : k_ == E_CPU ? ST_CPU : ("
            << ek << " & " << u32((EF_COND | EF_GLOBAL) << 4) << ") ? ST_SKIP : ";
          if (g.uses_anchor) w << "(areg" << s << " & ~apres" << s << ") ? ST_ERROR : ";
          w << "k_ == E_LEN ? ST_ERROR : ST_FAIL);\n    goto " << R.se << "; }\n";
          break;
        default:  // OP_NOP, OP_METACHK (handled per resource by RF_BAD_META)
          break;
      }
      oo.code = w.str();
      outs.push_back(std::move(oo));
    }
    for (const auto& x : outs) wout << x.code;
  }

  RGen analyze(uint32_t ri) {
    RGen g;
    g.ri = ri;
    g.s = "_" + std::to_string(ri);
    g.b = ps.rules[ri].prog;
    g.e = prog_end(ps, g.b);
    int nest = 0;
    for (uint32_t pc = g.b; pc <= g.e; pc++) {
      const Inst& in = ps.prog[pc];
      const uint32_t op = in.op & 0xFF, d = (in.op >> 8) & 0xFF, aux = (in.op >> 16) & 0xFF;
      g.maxd = std::max(g.maxd, d + 2);
      if (op == OP_AREG) g.uses_anchor = true;
      if (op == OP_KEYGLOB) g.uses_keyglob = true;
      if (op == OP_LOOP_BEGIN || op == OP_EXIST_BEGIN) {
        if (op == OP_LOOP_BEGIN && nest == 0 && (aux & 3) == 0) g.loops.push_back({pc, in.a});
        g.max_level = std::max(g.max_level, aux & 3);
        nest++;
      } else if (op == OP_LOOP_END || op == OP_EXIST_END) {
        nest--;
      }
    }
    g.expr.assign(g.maxd + 1, "");
    g.hv.assign(g.maxd + 1, HVar{});
    g.expr[0] = "R";
    g.hv[0] = HVar{"root", "rootn"};
    return g;
  }

  // The ops a lane runs after leaving stage loop k of `g` with a (non-condition) error,
  // from the LOOP_END's catch target: pure when it only carries the error through scope
  // ends to DONE (or to the end of the last anyPattern alternative), adding `flags`. The
  // rule's status is then a function of the error alone, decided at the failing element.
  struct PostChain {
    bool pure = false, alt = false;
    uint32_t flags = 0;
  };
  PostChain post_chain(const RGen& g, uint32_t pc, bool cond = false) const {
    PostChain r;
    for (int steps = 0; steps < 100000 && pc >= g.b && pc <= g.e; steps++) {
      const Inst& in = ps.prog[pc];
      const uint32_t op = in.op & 0xFF, aux = (in.op >> 16) & 0xFF;
      switch (op) {
        case OP_SCOPE_END:
          r.flags |= aux;
          cond |= (aux & EF_COND) != 0;
          pc = in.c ? in.c : pc + 1;
          continue;
        case OP_POS_END:
        case OP_LOOP_END:
          if (cond) return r;  // a condition error is cleared there: the walk goes on
          pc = in.c;
          continue;
        case OP_NOP:
        case OP_METACHK:
          pc++;
          continue;
        case OP_DONE:
          r.pure = true;
          return r;
        case OP_ALT_END:
          if (in.b) r.pure = r.alt = true;  // the last alternative: FAIL (or CPU)
          return r;
        default:
          return r;
      }
    }
    return r;
  }

  // Status of a rule whose error `ekx` reached DONE (or the last alternative's end): the
  // MatchPattern epilogue as one select chain
  std::string done_status(const RGen& g, const std::string& ekx, bool alt) const {
    std::ostringstream w;
    const std::string k = "(" + ekx + " & 15u)";
    if (alt) {
      w << "(" << k << " == 0u ? ST_PASS : " << k << " == E_CPU ? ST_CPU : ST_FAIL)";
      return w.str();
    }
    w << "(" << k << " == 0u ? ST_PASS : " << k << " == E_CPU ? ST_CPU : (" << ekx << " & "
      << u32((EF_COND | EF_GLOBAL) << 4) << ") ? ST_SKIP : ";
    if (g.uses_anchor) w << "(areg" << g.s << " & ~apres" << g.s << ") ? ST_ERROR : ";
    w << k << " == E_LEN ? ST_ERROR : ST_FAIL)";
    return w.str();
  }

  // Structural form of rule ri's program for rule groups: its ops with their operands, jump
  // targets relative to the program start; the pattern nodes and leaf predicates are left out
  // (listed in pns / preds, the LEAF pcs relative to the start in leafpcs). Empty when the
  // program holds an op a group cannot run: condition anchors (errors cleared later), existence
  // anchors, anyPattern, wildcard keys, pattern variables.
  std::string group_form(uint32_t ri, std::vector<uint32_t>* preds, std::vector<uint32_t>* pns,
                         std::vector<uint32_t>* leafpcs) const {
    const RuleRec& rr = ps.rules[ri];
    // (pattern-variable rules stay out of groups: their substitution status is decided per
    // member before the walk, and a group's record layout may be per resource slot)
    if (rr.route != 0 || rr.dyn) return "";
    const uint32_t b = rr.prog, e = prog_end(ps, b);
    std::ostringstream f;
    auto rel = [&](uint32_t t) { return (int64_t)t - (int64_t)b; };
    for (uint32_t pc = b; pc <= e; pc++) {
      const Inst& in = ps.prog[pc];
      const uint32_t op = in.op & 0xFF, aux = (in.op >> 16) & 0xFF;
      f << (in.op & 0xFFFFFFu) << ':';  // op | depth << 8 | aux << 16
      switch (op) {
        case OP_MAPCHK:
        case OP_ARRCHK: pns->push_back(in.a); f << rel(in.c); break;
        case OP_AREG:
        case OP_KEYV:
        case OP_INDEX: f << in.a; break;
        case OP_KEY: f << in.a << ',' << rel(in.b); break;
        case OP_SCOPE_END:
          if (aux & EF_COND) return "";
          f << (in.c ? rel(in.c) : -1);
          break;
        case OP_NEG: f << in.a << ','; pns->push_back(in.b); f << rel(in.c); break;
        case OP_STAR: pns->push_back(in.b); f << rel(in.c); break;
        case OP_LEAF:
          preds->push_back(in.a);
          leafpcs->push_back(pc - b);
          pns->push_back(in.b);
          f << rel(in.c);
          break;
        case OP_RAISE: f << in.b << ','; pns->push_back(in.a); f << rel(in.c); break;
        case OP_LENCHK: f << in.a << ','; pns->push_back(in.b); f << rel(in.c); break;
        case OP_LOOP_BEGIN: f << rel(in.a); break;
        case OP_LOOP_END: f << rel(in.a) << ',' << rel(in.c); break;
        case OP_DONE:
        case OP_NOP:
        case OP_METACHK: break;
        default: return "";
      }
      f << ';';
    }
    return f.str();
  }

  // Match bits (kv_mtup_kernel): the rule at LDS row q of the kernel being generated has bit
  // position 32 * mt_kbase + q; mt_bits[p] = the rule at bit position p (KV_SENT: padding).
  // A rule whose match reads the resource name is evaluated per resource behind its bit (which
  // the tuple kernel sets to 1).
  uint32_t mt_kbase = 0;
  std::vector<uint32_t> mt_bits;
  std::vector<uint8_t> rec_slot;  // rules whose records go to their resource slot (gslot_members)
  bool name_dependent(uint32_t ri) const {
    const RuleRec& rr = ps.rules[ri];
    for (uint32_t f = rr.m_first; f < rr.m_first + rr.m_count; f++)
      if (ps.filters[f].flags & (MF_NAME | MF_NAMES)) return true;
    for (uint32_t f = rr.x_first; f < rr.x_first + rr.x_count; f++)
      if (ps.filters[f].flags & (MF_NAME | MF_NAMES)) return true;
    return false;
  }
  std::string mt_cond(uint32_t ri, uint32_t row) const {
    const uint32_t p = mt_kbase * 32u + row;
    std::string c = "((mw" + std::to_string(p / 32u) + " >> " + std::to_string(p % 32u) + "u) & 1u)";
    if (name_dependent(ri)) c += " && g_match_" + std::to_string(ri) + "(P, B, R, rkind, rflags)";
    return c;
  }

  uint32_t gtab_n = 0;          // member tables emitted so far (per generated program text)
  std::string block_decls;      // declarations the current kernel's blocks need (member tables)

  // Code block of one fused chunk inside a kernel body (its own C++ scope); the
  // chunk's status rows are s_stw rows [hbase, hbase + rules) (KV_RSTRIDE bytes each).
  //
  // Lean rules (hist_lds kernels): at the end of stage segment k a rule that enters stage
  // loop k keeps only one bit (am<k>_<w>, bit q of its block position), one that jumps past
  // the loop one bit of sk<k>_<w> (its single target), and one that finished stores its
  // status at once; inside the fused loop its error state is local to the element and an
  // element that fails decides the status there (post_chain), so no per-rule register lives
  // across the loop. After the loops the resume pc is rebuilt from the bits.
  //
  // Rule groups (hist_lds kernels): rules of one structural form (group_form) whose pattern
  // nodes differ by one constant run the representative's program once, with one bit per
  // member; their leaf predicates take consecutive bits of one table word, so a leaf tests
  // every member with one shift and mask. The members take consecutive block positions.
  // `order` receives the block's rules in block position order.
  std::string fused_block(const JitChunk& ch_in, uint32_t hbase, std::vector<uint32_t>* order) {
    struct GInfo {
      std::vector<uint32_t> members, pns0, leafpcs;
      std::vector<uint32_t> dpn;                 // pattern-node shift of each member
      std::vector<std::vector<uint32_t>> preds;  // leaf predicates of each member
    };
    std::vector<GInfo> ginfo;
    std::map<uint32_t, size_t> gof;  // rule -> group
    if (hist_lds) {
      std::map<std::string, size_t> open;
      for (uint32_t ri : ch_in.rules) {
        std::vector<uint32_t> pr, pn, lp;
        const std::string f = group_form(ri, &pr, &pn, &lp);
        if (f.empty()) continue;
        auto it = open.find(f);
        if (it != open.end()) {
          GInfo& G = ginfo[it->second];
          const uint32_t dp = pn.empty() ? 0u : pn[0] - G.pns0[0];
          bool ok = G.members.size() < 32;
          for (size_t i = 0; i < pn.size() && ok; i++) ok = pn[i] - G.pns0[i] == dp;
          if (ok) {
            G.members.push_back(ri);
            G.dpn.push_back(dp);
            G.preds.push_back(pr);
            gof[ri] = it->second;
            continue;
          }
        }
        GInfo G;
        G.members = {ri};
        G.pns0 = pn;
        G.leafpcs = lp;
        G.dpn = {0u};
        G.preds = {pr};
        open[f] = ginfo.size();
        gof[ri] = ginfo.size();
        ginfo.push_back(std::move(G));
      }
    }
    JitChunk ch;  // block order: a group's members together, at its first member's place
    for (uint32_t ri : ch_in.rules) {
      auto it = gof.find(ri);
      if (it == gof.end()) ch.rules.push_back(ri);
      else if (ginfo[it->second].members[0] == ri)
        ch.rules.insert(ch.rules.end(), ginfo[it->second].members.begin(), ginfo[it->second].members.end());
    }
    *order = ch.rules;
    const uint32_t nr = (uint32_t)ch.rules.size();
    std::vector<RGen> gs;
    HoistTable global;
    global.prefix = "g";
    global.fam = 0;
    global.cell0 = "gc_";
    gT = &global;
    size_t K = 0;
    for (uint32_t q = 0; q < nr; q++) {
      const uint32_t ri = ch.rules[q];
      if (ps.rules[ri].route != 0) continue;
      auto git = gof.find(ri);
      if (git != gof.end() && ginfo[git->second].members[0] != ri) continue;  // a group member
      RGen g = analyze(ri);
      g.q = q;
      for (uint32_t pc = g.b; pc <= g.e; pc++)
        if ((ps.prog[pc].op & 0xFF) == OP_LEAF) pred_fn(ps.prog[pc].a);
      if (git != gof.end()) {
        const GInfo& G = ginfo[git->second];
        g.grp = true;
        g.s = "_G" + std::to_string(hbase + q);
        g.gn = (uint32_t)G.members.size();
        g.gri = G.members;
        g.gdpn = G.dpn;
        if (g.gn >= 2u) {
          g.gsite = true;
          g.gl = k_gsn++;
          g.gpre = gs_members;
          gs_desc.insert(gs_desc.end(), {g.gn, gs_members, (uint32_t)(gs_mem.size() / 2u), 0u});
          for (uint32_t j = 0; j < g.gn; j++) gs_mem.insert(gs_mem.end(), {G.members[j], G.dpn[j]});
          gs_members += g.gn;
        }
        // (site-record members get their records expanded to their resource slots at fetch)
        if (g.gsite || g.gn >= gslot_members())
          for (uint32_t m : G.members) rec_slot.at(m) = 1;
        g.grow = hbase + q;
        for (const auto& m : G.preds)
          for (uint32_t pi : m) pred_fn(pi);
        for (size_t i = 0; i < G.leafpcs.size(); i++) {
          std::vector<uint32_t> lp;
          for (const auto& m : G.preds) lp.push_back(m[i]);
          g.gslot[g.b + G.leafpcs[i]] = group_slots(lp);
        }
        // members as arithmetic progressions (rule ids, node shifts), else a table
        bool arith = true;
        g.gsri = g.gn > 1 ? g.gri[1] - g.gri[0] : 0u;
        g.gspn = g.gn > 1 ? g.gdpn[1] : 0u;
        for (uint32_t j = 0; j < g.gn && arith; j++) arith = g.gri[j] == g.gri[0] + j * g.gsri && g.gdpn[j] == j * g.gspn;
        if (!arith) {
          g.gtab = "kvg_t" + std::to_string(gtab_n++);
          std::ostringstream t;
          t << "__device__ const uint32_t " << g.gtab << "[" << 2 * g.gn << "] = {";
          for (uint32_t j = 0; j < g.gn; j++) t << u32(g.gri[j]) << ", ";
          for (uint32_t j = 0; j < g.gn; j++) t << u32(g.gdpn[j]) << (j + 1 < g.gn ? ", " : "");
          t << "};\n";
          block_decls += t.str();
        }
      }
      K = std::max(K, g.loops.size());
      g.lean.assign(g.loops.size(), 0);
      g.post_flags.assign(g.loops.size(), 0);
      g.post_alt.assign(g.loops.size(), 0);
      g.skip_to.assign(g.loops.size(), 0xFFFFFFFFu);
      g.skip_flags.assign(g.loops.size(), 0);
      g.skip_alt.assign(g.loops.size(), 0);
      gs.push_back(std::move(g));
    }
    const uint32_t nw = (nr + 31) / 32;
    auto mword = [&](const char* m, size_t k, uint32_t q) {
      return std::string(m) + std::to_string(k) + "_" + std::to_string(q / 32);
    };
    auto mbit = [&](uint32_t q) { return u32(1u << (q % 32)); };
    // status row of block position q: its LDS address and row index
    auto row = [&](uint32_t q) { return "s_w + " + u32(KV_ROW0 + (hbase + q) * KV_RSTRIDE) + ", " + u32(hbase + q); };
    // EState of rule g from its registers (error kind / flags / pattern node in `ekx`)
    auto estate = [&](const RGen* g, const std::string& ekx) {
      std::ostringstream k;
      if (!g) return std::string("EState e_{0u, 0u, 0u, ABSENT, ABSENT, 0u, 0u, 0u, 0u};");
      k << "EState e_{" << ekx << " & 15u, (" << ekx << " >> 4) & 15u, " << ekx << " >> 8, "
        << (g->uses_keyglob ? "ekn" + g->s : std::string("ABSENT")) << ", ABSENT";
      for (uint32_t lv = 0; lv < 4; lv++) k << ", " << (lv <= g->max_level ? "ei" + std::to_string(lv) + g->s : "0u");
      k << "};";
      return k.str();
    };
    // status + error record of rule `ri` (block position q): LDS status byte (copied to the
    // status matrix at the end of the kernel) + the error record, or the ballot histogram
    auto store_st = [&](uint32_t q, const RGen* g, const std::string& st, const std::string& ekx) {
      const uint32_t ri = ch.rules[q];
      std::ostringstream k;
      k << "  { " << estate(g, ekx) << "\n";
      if (hist_lds)
        k << "    kv_final(O, " << ri << "u, n_res, r, valid, " << st << ", e_, " << row(q) << "); }\n";
      else
        k << "    store_result2(O, " << ri << "u, n_res, r, valid, " << st << ", e_, &s_hist[" << (hbase + q)
          << "][0]); }\n";
      return k.str();
    };
    auto store = [&](uint32_t q) {
      const RGen* g = nullptr;
      for (const RGen& x : gs)
        if (x.q == q) g = &x;
      const std::string s = g ? g->s : "_" + std::to_string(ch.rules[q]);
      const std::string st = "rs" + s + " & 0xFFu";
      if (!g) return store_st(q, g, st, "0u");
      // the members alive at a group's end passed: their PASS was staged by the match code
      // (a group ends only at DONE, ST_PASS, or with every member decided, ST_STORED_)
      if (g->grp) return std::string();
      return "  if ((rs" + s + " & 0xFFu) != ST_STORED_" + (hist_lds ? std::string(" && (rs" + s + " & 0xFFu) != ST_NOMATCH") : "") +
             ") {\n" + store_st(q, g, st, "ek" + s) + "  }\n";
    };
    // match / route of rule q (rs = its first pc, or FIN | status); of a group: every member's,
    // the matched ones alive (al), the others stored
    auto match_code = [&](uint32_t q) {
      const RGen* gp = nullptr;
      for (const RGen& x : gs)
        if (x.q == q && x.grp) gp = &x;
      if (gp) {
        // a group's members are consecutive rows, so their match bits are consecutive bits of the
        // block's match words: one extract instead of a branch per member. Statuses are staged
        // here, branch-free: PASS for every member that runs (a failure overwrites its byte where
        // it is raised, so the group's end stores nothing), CPU for the members an anchor-error
        // phrase or a panicking labels / annotations shape routes (rows start as NOMATCH; 0xFF
        // past the batch)
        const RGen& g = *gp;
        std::ostringstream k;
        const uint32_t p0 = mt_kbase * 32u + g.grow, w0 = p0 / 32u, s0 = p0 % 32u;
        const uint32_t mask = g.gn >= 32 ? 0xFFFFFFFFu : (1u << g.gn) - 1u;
        k << "  { uint32_t mt_ = ((mw" << w0 << " >> " << s0 << "u)";
        if (s0 + g.gn > 32u) k << " | (mw" << (w0 + 1) << " << " << (32u - s0) << "u)";
        k << ") & " << hex32(mask) << ";\n";
        for (uint32_t j = 0; j < g.gn; j++)
          if (name_dependent(g.gri[j]))
            k << "    if (((mt_ >> " << j << "u) & 1u) && !g_match_" << g.gri[j] << "(P, B, R, rkind, rflags)) mt_ &= "
              << hex32(~(1u << j)) << ";\n";
        k << "    uint32_t cpu_ = (rflags & RF_MAGIC) ? mt_ : 0u;\n";
        for (uint32_t j = 0; j < g.gn; j++) {
          const RuleRec& rr = ps.rules[g.gri[j]];
          if (rr.flags & RR_META_EXPAND)
            k << "    cpu_ |= (rflags & " << u32(meta_bad_flags(rr.flags)) << ") ? (mt_ & " << u32(1u << j) << ") : 0u;\n";
        }
        for (uint32_t j = 0; j < g.gn; j++)
          k << "    s_w[" << u32(KV_ROW0 + (g.grow + j) * KV_RSTRIDE) << " + threadIdx.x] = valid ? (uint8_t)(((mt_ >> " << j
            << "u) & 1u) ? (((cpu_ >> " << j << "u) & 1u) ? ST_CPU : ST_PASS) : ST_NOMATCH) : (uint8_t)0xFFu;\n";
        k << "    al" << g.s << " = mt_ & ~cpu_; }\n";
        k << "  rs" << g.s << " = al" << g.s << " ? " << u32(g.b) << " : FIN_ | ST_STORED_;\n";
        return k.str();
      }
      const uint32_t ri = ch.rules[q];
      const RuleRec& rr = ps.rules[ri];
      const std::string s = "_" + std::to_string(ri);
      std::ostringstream k;
      k << "  if (" << mt_cond(ri, hbase + q) << ") {\n";
      switch (rr.route) {
        case 1: k << "    rs" << s << " = FIN_ | ST_CPU;\n"; break;
        case 2: k << "    rs" << s << " = FIN_ | ST_NOMATCH;\n"; break;
        case 3: k << "    rs" << s << " = FIN_ | " << u32(rr.const_status) << ";\n"; break;
        default:
          k << "    if (rflags & RF_MAGIC) rs" << s << " = FIN_ | ST_CPU;\n";
          if (rr.flags & RR_META_EXPAND)
            k << "    else if (rflags & " << u32(meta_bad_flags(rr.flags)) << ") rs" << s << " = FIN_ | ST_CPU;\n";
          if (rr.dyn)
            k << "    else if (B.dyn_st[(size_t)" << (rr.dyn - 1) << "u * n_res + r]) rs" << s << " = FIN_ | B.dyn_st[(size_t)"
              << (rr.dyn - 1) << "u * n_res + r];\n";
          k << "    else rs" << s << " = " << u32(rr.prog) << ";\n";
          break;
      }
      k << "  }\n";
      return k.str();
    };
    std::ostringstream body;  // everything after the per-rule declarations
    for (size_t k = 0; k <= K; k++) {
      std::ostringstream seg;  // the stage-k segments of every rule
      for (RGen& g : gs) {
        if (k > g.loops.size()) continue;
        const uint32_t sb = k == 0 ? g.b : g.loops[k - 1].second + 1;
        const uint32_t se = k < g.loops.size() ? g.loops[k].first + 1 : g.e + 1;  // include the LOOP_BEGIN
        Region R;
        R.kind = 0;
        R.rb = sb;
        R.re = se;
        R.jre = se;
        R.se = "R" + std::to_string(g.ri) + "_S" + std::to_string(k);
        std::ostringstream w;
        g.seg_jumps.clear();
        g.seg_err_jumps.clear();
        emit_region(g, R, w);
        if (k == 0) seg << match_code(g.q);  // just before its first segment: rs is born here
        if (k > 0 && g.lean[k - 1]) {  // resume pc of a lean rule from its stage-(k-1) bits
          const uint32_t le = g.loops[k - 1].second;
          seg << "  rs" << g.s << " = (" << mword("am", k - 1, g.q) << " & " << mbit(g.q) << ") ? " << u32(le + 1) << " : ";
          if (g.skip_to[k - 1] != 0xFFFFFFFFu)
            seg << "(" << mword("sk", k - 1, g.q) << " & " << mbit(g.q) << ") ? " << u32(g.skip_to[k - 1]) << " : ";
          seg << "FIN_ | ST_STORED_;\n";
          // the error state of a lane that left the loop clean (no register of the rule lives
          // across the loop)
          seg << "  ek" << g.s << " = 0u;";
          for (uint32_t lv = 0; lv <= g.max_level && lv < 4; lv++) seg << " ei" << lv << g.s << " = 0u;";
          if (g.uses_keyglob) seg << " ekn" << g.s << " = ABSENT;";
          seg << "\n";
        }
        seg << "  // rule " << g.ri << " stage " << k << "\n  switch (rs" << g.s << ") {\n";
        if (k == 0) seg << "    case " << u32(g.b) << ": goto R" << g.ri << "_L" << g.b << ";\n";
        for (uint32_t t : g.resume)
          if (t >= sb && t < se) seg << "    case " << u32(t) << ": goto R" << g.ri << "_L" << t << ";\n";
        seg << "    default: goto " << R.se << ";\n  }\n" << w.str() << R.se << ":;\n";
        if (k == g.loops.size()) {
          seg << store(g.q);  // the rule has finished for every lane
          continue;
        }
        // stage loop k follows: lean when the kernel stages statuses in LDS, the post chain of
        // the loop is pure, and the segment leaves at most one way past the loop, whose chain
        // is pure for any pending error (a lane that jumps there with an error is decided at
        // once; one without resumes there after the loop)
        const uint32_t le = g.loops[k].second;
        const PostChain pcn = post_chain(g, ps.prog[le].c);
        // every way past loop k: this segment's jumps and the targets of earlier stages that lie
        // beyond this segment (they pass through it)
        std::set<uint32_t> okset = g.seg_jumps, errset = g.seg_err_jumps;
        for (uint32_t t : g.carry_ok)
          if (t >= se) okset.insert(t);
        for (uint32_t t : g.carry_err)
          if (t >= se) errset.insert(t);
        bool lean = hist_lds && pcn.pure && okset.size() <= 1;
        std::vector<std::pair<uint32_t, PostChain>> errc;  // chains of the error targets
        for (uint32_t t : errset) {
          errc.push_back({t, post_chain(g, t, true)});
          lean &= errc.back().second.pure;
        }
        bool alt0 = !errc.empty() && errc[0].second.alt;
        for (auto& e : errc) lean &= e.second.alt == alt0;
        g.carry_ok = okset;
        if (lean) {
          g.carry_err.clear();  // errors past the loop are decided at the segment end
        } else {
          g.carry_ok.insert(le + 1);
          g.carry_err = errset;
          g.carry_err.insert(ps.prog[le].c);
        }
        g.lean[k] = lean;
        g.post_flags[k] = pcn.flags;
        g.post_alt[k] = pcn.alt;
        if (!lean) continue;
        const std::string ek = "ek" + g.s;
        seg << "  if (rs" << g.s << " & ACT_) " << mword("am", k, g.q) << " |= " << mbit(g.q) << ";\n";
        if (!okset.empty() || !errc.empty()) {
          // past the loop: with an error the status is decided now, else resume there later
          seg << "  else if (rs" << g.s << " < FIN_) {\n";
          if (!errc.empty()) {
            std::string fl = "0u";
            for (auto it = errc.rbegin(); it != errc.rend(); ++it)
              fl = "(rs" + g.s + " == " + u32(it->first) + " ? " + u32(it->second.flags << 4) + " : " + fl + ")";
            const std::string ekx = "(" + ek + " | " + fl + ")";
            seg << "    if (" << ek << " & 15u) {\n" << store_st(g.q, &g, done_status(g, ekx, alt0), ekx) << "    }\n";
          }
          if (!okset.empty()) {
            g.skip_to[k] = *okset.begin();
            seg << "    " << (errc.empty() ? "" : "else ") << mword("sk", k, g.q) << " |= " << mbit(g.q) << ";\n";
          }
          seg << "  }\n";
        }
        seg << "  else {\n" << store(g.q) << "  }\n";
      }
      if (k < K) {  // stage-k masks of the lean rules
        std::ostringstream mk;
        mk << "  uint32_t";
        for (uint32_t w = 0; w < nw; w++) mk << (w ? "," : "") << " am" << k << "_" << w << " = 0u, sk" << k << "_" << w << " = 0u";
        mk << ";\n";
        body << mk.str();
      }
      body << global.flush() << seg.str();
      if (k == K) break;
      // fused loops of stage k: group rules by the symbolic array cursor
      std::map<std::string, std::vector<RGen*>> groups;
      std::vector<std::string> order;
      for (RGen& g : gs) {
        if (k >= g.loops.size()) continue;
        const uint32_t lb = g.loops[k].first;
        const uint32_t d = (ps.prog[lb].op >> 8) & 0xFF;
        std::string key = g.expr[d].empty() ? "U" + std::to_string(g.ri) : g.expr[d];
        if (!groups.count(key)) order.push_back(key);
        groups[key].push_back(&g);
      }
      uint32_t li = 0;
      for (const std::string& key : order) {
        std::vector<RGen*>& grp = groups[key];
        const std::string tag = std::to_string(k) + "_" + std::to_string(li++);
        const RGen& g0 = *grp[0];
        const uint32_t d0 = (ps.prog[g0.loops[k].first].op >> 8) & 0xFF;
        const std::string arr_node = key[0] == 'U' ? "N[c" + std::to_string(d0) + g0.s + "]" : g0.hv[d0].node;
        HoistTable T;
        T.prefix = "l" + tag + "_";
        const std::string troot = "E" + tag;
        // the elements' lookups from the columns of the array's family (the array must be a
        // column itself: its cell carries the offset of its element rows)
        const uint32_t fam = key[0] == 'R' && fams[0].idx.count(key) ? family(key) : kNoCol;
        if (fam != kNoCol) {
          T.fam = (int)fam;
          T.troot = troot;
          T.cell0 = "ec" + tag;
        }
        std::ostringstream bodies;
        std::vector<uint32_t> gmask(nw, 0);  // lean rules of the group, per mask word
        for (RGen* gp : grp) {
          RGen& g = *gp;
          const uint32_t lb = g.loops[k].first, le = g.loops[k].second;
          const uint32_t d = (ps.prog[lb].op >> 8) & 0xFF;
          g.expr[d + 1] = troot;
          g.hv[d + 1] = HVar{"el" + tag, "eln" + tag};
          Region R;
          R.kind = 1;
          R.rb = lb + 1;
          R.re = le;  // LOOP_END emitted below
          R.jre = le + 1;
          R.li0 = "fli" + tag;
          R.T = &T;
          R.troot = troot;
          std::ostringstream w;
          emit_region(g, R, w);
          const Inst& end = ps.prog[le];
          if (end.c <= le) throw std::runtime_error("kvjit: loop exit target inside the loop");
          const std::string ek = "ek" + g.s;
          if (g.grp) {  // errors were decided where raised: a group with no member left stops
            const std::string act = g.lean[k] ? mword("am", k, g.q) + " & " + mbit(g.q) : "rs" + g.s + " & ACT_";
            if (g.lean[k]) gmask[g.q / 32] |= 1u << (g.q % 32);
            bodies << "    if (" << act << ") {\n      c" << (d + 1) << g.s << " = el" << tag << ";\n"
                   << w.str() << "R" << g.ri << "_L" << le << ":;\n      if (!al" << g.s << ") ";
            if (g.lean[k]) bodies << mword("am", k, g.q) << " &= ~" << mbit(g.q) << ";\n    }\n";
            else bodies << "rs" << g.s << " = FIN_ | ST_STORED_;\n    }\n";
          } else if (g.lean[k]) {
            gmask[g.q / 32] |= 1u << (g.q % 32);
            // element-local error state; an error that leaves the loop decides the status now
            bodies << "    if (" << mword("am", k, g.q) << " & " << mbit(g.q) << ") {\n      " << ek << " = 0u;";
            for (uint32_t lv = 0; lv <= g.max_level && lv < 4; lv++) bodies << " ei" << lv << g.s << " = 0u;";
            if (g.uses_keyglob) bodies << " ekn" << g.s << " = ABSENT;";
            bodies << "\n      c" << (d + 1) << g.s << " = el" << tag << ";\n"
                   << w.str() << "R" << g.ri << "_L" << le << ":;\n"
                   << "      if (" << ek << " & 15u) { if (" << ek << " & " << u32(EF_COND << 4) << ") " << ek
                   << " = 0u; else {\n        " << mword("am", k, g.q) << " &= ~" << mbit(g.q) << ";\n";
            const std::string ekx = g.post_flags[k] ? "(" + ek + " | " + u32(g.post_flags[k] << 4) + ")" : ek;
            bodies << "  " << store_st(g.q, &g, done_status(g, ekx, g.post_alt[k]), ekx) << "      } }\n    }\n";
          } else {
            bodies << "    if (rs" << g.s << " & ACT_) {\n      c" << (d + 1) << g.s << " = el" << tag << ";\n"
                   << w.str() << "R" << g.ri << "_L" << le << ":;\n"
                   << "      if (" << ek << " & 15u) { if (" << ek << " & " << u32(EF_COND << 4) << ") " << ek
                   << " = 0u; else rs" << g.s << " = " << u32(end.c) << "; }\n    }\n";
            g.resume.insert(end.c);
          }
          g.resume.insert(le + 1);
          for (uint32_t x = d + 1; x < g.expr.size(); x++) g.expr[x].clear();  // loop-local exprs end here
        }
        body << "  { // fused loop " << tag << " over " << key << " (" << grp.size() << " rules)\n"
             << "    uint32_t fn" << tag << " = 0u, ff" << tag << " = 0u, fe" << tag << " = 0u;\n    if (((0u";
        for (RGen* gp : grp)
          if (!gp->lean[k]) body << " | rs" << gp->s;
        body << ") & ACT_)";
        for (uint32_t w = 0; w < nw; w++)
          if (gmask[w]) body << " | (am" << k << "_" << w << " & " << u32(gmask[w]) << ")";
        body << ") { const Node an_ = " << arr_node << "; ff" << tag << " = an_.a; fn" << tag << " = an_.b; fe" << tag
             << " = an_.c; }\n";
        body << "    for (uint32_t fli" << tag << " = 0u; fli" << tag << " < fn" << tag << "; fli" << tag << "++) {\n"
             << "      const uint32_t el" << tag << " = ni(ff" << tag << " + fli" << tag << ");\n";
        if (fam != kNoCol)  // the element's column-0 cell: element row fe + i of its family
          body << "      const uint32_t ec" << tag << " = fe" << tag << " + fli" << tag << " * (KVC_J" << fam
               << " * " << u32(KV_LANES) << ") + ln_;\n      const Node eln" << tag << " = kv_ldc(PC, PCB, ec" << tag << ");\n";
        else
          body << "      const Node eln" << tag << " = N[el" << tag << "];\n";
        body << T.flush() << bodies.str() << "    }\n";
        for (RGen* gp : grp)
          if (!gp->lean[k]) body << "    rs" << gp->s << " &= ~ACT_;\n";
        body << "  }\n";
      }
    }
    // every resume pc must lie in a segment (else the rule would never finish)
    for (const RGen& g : gs)
      for (uint32_t t : g.resume) {
        bool ok = false;
        for (size_t k = 0; k <= g.loops.size() && !ok; k++) {
          const uint32_t sb = k == 0 ? g.b : g.loops[k - 1].second + 1;
          const uint32_t se = k < g.loops.size() ? g.loops[k].first + 1 : g.e + 1;
          ok = t >= sb && t < se;
        }
        if (!ok) throw std::runtime_error("kvjit: resume target " + std::to_string(t) + " of rule " +
                                         std::to_string(g.ri) + " is not in a segment");
      }

    std::ostringstream k;
    // per-rule state (rules of other routes only carry rs = FIN | status); a group's: rs and the
    // alive members
    for (uint32_t ri : ch.rules)
      if (!gof.count(ri)) k << "  uint32_t rs_" << ri << " = FIN_ | ST_NOMATCH;\n";
    for (const RGen& g : gs) {
      const std::string& s = g.s;
      if (g.grp) k << "  uint32_t rs" << s << " = FIN_ | ST_STORED_, al" << s << " = 0u;\n";
      k << "  uint32_t ek" << s << " = 0u";
      for (uint32_t lv = 0; lv <= g.max_level && lv < 4; lv++) k << ", ei" << lv << s << " = 0u";
      if (g.uses_keyglob) k << ", kn" << s << " = ABSENT, ekn" << s << " = ABSENT";
      k << ";\n";
      if (g.uses_anchor) k << "  uint64_t areg" << s << " = 0ull, apres" << s << " = 0ull;\n";
      k << "  uint32_t c0" << s << " = root";
      for (uint32_t d = 1; d < g.maxd; d++) k << ", c" << d << s << " = ABSENT";
      k << ";\n";
      k << "  uint32_t";
      for (uint32_t l = 0; l <= g.max_level && l < 4; l++)
        k << (l ? "," : "") << " li" << l << s << " = 0u, lf" << l << s << " = 0u, ll" << l << s << " = 0u";
      k << ";\n";
    }
    // rules of other routes are final after match / route
    for (uint32_t q = 0; q < nr; q++)
      if (ps.rules[ch.rules[q]].route != 0) k << match_code(q) << store(q);
    k << body.str();
    return k.str();
  }

  // One kernel running the fused chunks `chs` one after the other for each
  // resource: a workgroup re-reads its resources' node rows per chunk while they
  // are still cache-resident, instead of one grid-wide pass per chunk.
  // Statuses: one LDS row per rule of the kernel (KV_RSTRIDE bytes: a status byte per lane)
  // after the waves' record counters (KV_ROW0 bytes: a byte per (wave, rule)), prefilled with NOMATCH, flushed once when the kernel ends
  // (kv_end_flush: status matrix, per-rule and per-scope histograms). A per-block flush of
  // wave-private rows (round 4, first build) freed the LDS but cost C5 25 flushes per wave:
  // 3.91 against 3.25 ms per pass.
  static uint32_t kernel_lds(uint32_t nr) { return KV_ROW0 + nr * KV_RSTRIDE; }
  // waves per SIMD a CU's 160 KB LDS admits (workgroups of KV_RWAVES waves): allocations are made
  // in 1280 B granules (C3's 124-rule kernels, 32 240 B, ran at 4 workgroups of 4 waves per CU and
  // 1.3x the time of the 123-rule ones at 31 980 B; round 4, gpurun_out/r4h)
  static int lds_waves(uint32_t nr) {
    const uint32_t g = 1280u, b = (kernel_lds(nr) + g - 1u) / g * g;
    return (int)std::max<uint32_t>(1u, (160u * 1024u) / std::max(b, g) * KV_RWAVES / 4u);
  }
  std::vector<uint32_t> group_kernel(const std::string& name, const std::vector<const JitChunk*>& chs, int waves) {
    std::vector<std::string> blocks;
    std::vector<std::pair<uint32_t, uint32_t>> rows;  // LDS rows [first, first + count) of each block
    std::vector<uint32_t> rules;
    uint32_t nr_all = 0;
    for (const JitChunk* c : chs) nr_all += (uint32_t)c->rules.size();
    hist_lds = true;
    // (the waves' record counters hold a byte per (wave, row): KV_KROWS rows)
    if (nr_all > KV_KROWS) throw std::runtime_error("kvjit: at most KV_KROWS rules per kernel (KVGPU_JIT_CHUNK)");
    block_decls.clear();
    mt_kbase = (uint32_t)(mt_bits.size() / 32u);
    k_gs0 = (uint32_t)(gs_desc.size() / 4u);
    k_gsn = 0;
    for (const JitChunk* c : chs) {
      std::vector<uint32_t> ord;
      rows.push_back({(uint32_t)rules.size(), (uint32_t)c->rules.size()});
      blocks.push_back(fused_block(*c, (uint32_t)rules.size(), &ord));
      rules.insert(rules.end(), ord.begin(), ord.end());
    }
    mt_bits.insert(mt_bits.end(), rules.begin(), rules.end());
    while (mt_bits.size() % 32u) mt_bits.push_back(0xFFFFFFFFu);
    const uint32_t nr = (uint32_t)rules.size();
    // a wave's lane l zeroes / writes the site-record counters of the kernel's group l (groups have
    // 2+ members and a kernel at most KV_KROWS rules: at most 64 groups)
    if (k_gsn > 64u) throw std::runtime_error("kvjit: more than 64 site-record groups in one kernel");
    KernelText kt(*this, name);
    o << block_decls;
    if (getenv("KVGPU_JIT_STAMPS")) o << "__device__ unsigned long long* kvj_stamps;\n";
    o << "__device__ const uint32_t " << name << "_rules[" << nr << "] = {";
    for (uint32_t q = 0; q < nr; q++) o << (q ? ", " : "") << u32(rules[q]);
    o << "};\n";
    // Occupancy over registers: the rule kernels are latency-bound on dependent
    // tree loads, so they ask for 8 waves per SIMD (<= 64 VGPRs) unless the plan
    // relaxes it for a kernel that would spill (jit_plan_spills).
    const std::string lb = waves > 0 ? "KV_RWG, " + std::to_string(waves) : "KV_RWG";
    o << "extern \"C\" __global__ __launch_bounds__(" << lb << ") void " << name
      << "(const DevPS* __restrict__ Pp, const DevBatch* __restrict__ Bp, const Node* __restrict__ N, "
         "const Val* __restrict__ V, const uint8_t* __restrict__ S, DevOut O, uint32_t r0) {\n"
      << "  constexpr uint32_t FIN_ = " << u32(FIN) << ", ACT_ = " << u32(ACT) << ", ST_STORED_ = 0x7Eu;\n"
      << "  __shared__ unsigned long long s_stq[" << kernel_lds(nr) / 8 + (KV_RWAVES * k_gsn + 1u) / 2u
      << "];\n  uint32_t* s_stw = (uint32_t*)s_stq;\n"
      << "  const DevPS& P = *Pp;\n  const DevBatch& B = *Bp;\n  const uint8_t* __restrict__ pstr = P.pstr;\n";
    // Workgroup b runs tile (b % 8) * n/8 + b / 8, so each XCD (blocks b, b+8, ... share one)
    // walks a contiguous resource range and its L2 sees the values those resources share
    // (the value table and ptab lines are numbered by first occurrence): C2 -0.6 %, C3 -1 %
    // per pass, traffic -1 %
    o << "  const uint32_t nb_ = gridDim.x, x_ = blockIdx.x & 7u, per_ = nb_ >> 3, rem_ = nb_ & 7u;\n"
      << "  const uint32_t bx_ = x_ * per_ + (x_ < rem_ ? x_ : rem_) + (blockIdx.x >> 3);\n";
    o << "  const uint32_t r = r0 + bx_ * KV_RWG + threadIdx.x;\n"
      << "  const uint32_t n_res = B.n_res;\n"
      << "  const bool valid = r < n_res;\n"
      << "  const Res* __restrict__ R = B.res + (valid ? r : 0u);\n"
      << "  uint32_t root = ABSENT, rkind = KEY_NONE, rflags = 0u, rtup = 0u;\n"
      << "  if (valid) { root = ni(kv_gld(&R->root, 0)); rkind = kv_gld(&R->kind, 0); rflags = kv_gld(&R->flags, 0); rtup = kv_gld(&R->tup, 0); }\n"
      << "  Node rootn{0u, 0u, 0u, 0u};\n";
    // path columns (kvdevtypes.h): cell offset of this lane's family-0 columns; column 0 = the root
    o << "  const uint32_t* __restrict__ PC = B.pcol;\n  const uint32_t* __restrict__ PCB = B.pcolb;\n"
        << "  const uint32_t ln_ = threadIdx.x & " << u32(KV_LANES - 1) << ", gc_ = (r >> 6) * (KVC_J0 * " << u32(KV_LANES)
        << ") + ln_;\n  if (valid) rootn = kv_ldc(PC, PCB, gc_);\n";
    o
      << "  const uint32_t* __restrict__ mtr_ = P.mtup + rtup;\n  const uint32_t ntup_ = B.n_tup;\n"
      << "  uint8_t* s_w = (uint8_t*)s_stw;\n"
      // every status row starts as NOMATCH (0xFF past the batch): only matched lanes store
      // site-record counters of the kernel's groups, [group][wave] after the rows (zeroed before
      // the prefill's barrier)
      << "  uint32_t* const s_gc_ = s_stw + " << u32(kernel_lds(nr) / 4u) << ";\n"
      << (k_gsn ? "  for (uint32_t t_ = threadIdx.x; t_ < " + u32(KV_RWAVES * k_gsn) + "; t_ += KV_RWG) s_gc_[t_] = 0u;\n"
                : std::string())
      << "  kv_prefill_rows(s_stw, " << nr << "u, r - threadIdx.x, n_res);\n";
    // diagnostics (KVGPU_JIT_STAMPS): a wave's shader clock at the start, after each block and
    // after the flush, into the program's global kvj_stamps ([workgroup][wave][kJitStamps], set by
    // kvapi.cpp)
    const bool stamps = getenv("KVGPU_JIT_STAMPS") != nullptr;
    auto stamp = [&](size_t k) {
      if (stamps && k < kJitStamps)
        o << "  if (kvj_stamps && (threadIdx.x & 63u) == 0u) kvj_stamps[((size_t)blockIdx.x * KV_RWAVES + (threadIdx.x >> 6)) * "
          << kJitStamps << "u + " << k << "u] = __builtin_amdgcn_s_memtime();\n";
    };
    stamp(0);
    for (size_t bi = 0; bi < blocks.size(); bi++) {
      // the block's match words (bits of its rules, kv_mtup_kernel); a wave none of whose resources
      // matches any rule of the block skips it whole (every rule NOMATCH on every lane)
      const uint32_t r0 = rows[bi].first, rn = rows[bi].second;
      const uint32_t p0 = mt_kbase * 32u + r0, p1 = p0 + rn;  // bit positions [p0, p1)
      o << "  {\n";
      std::string any = "0u";
      for (uint32_t w = p0 / 32u; w * 32u < p1; w++) {
        const uint32_t lo = std::max(p0, w * 32u) - w * 32u, hi = std::min(p1, w * 32u + 32u) - w * 32u;
        const uint32_t m = hi - lo == 32u ? 0xFFFFFFFFu : ((1u << (hi - lo)) - 1u) << lo;
        o << "  const uint32_t mw" << w << " = valid ? kv_gld(mtr_, (size_t)" << w << "u * ntup_) : 0u;\n";
        any += " | (mw" + std::to_string(w) + " & " + u32(m) + ")";
      }
      // (the rows of a skipped block keep their NOMATCH prefill)
      o << "  if (__ballot((" << any << ") != 0u) != 0ull) {\n" << blocks[bi] << "  }\n";
      o << "  }\n";
      stamp(bi + 1);
    }
    // statuses to the status matrix, per-rule (and per-scope) histograms
    o << "  const uint32_t wg0_ = r - threadIdx.x;\n";
    // each wave's site-record counts (lane l: the kernel's group l)
    if (k_gsn)
      o << "#ifndef KVEMU\n  if ((KV_OFULL(O) & 2u) && !(KV_OFULL(O) & 4u) && (threadIdx.x & 63u) < " << u32(k_gsn)
        << " && r - (threadIdx.x & 63u) < n_res)\n    O.gcnt[(size_t)(" << u32(k_gs0)
        << " + (threadIdx.x & 63u)) * ((n_res + 63u) >> 6) + (r >> 6)] = s_gc_[(threadIdx.x & 63u) * KV_RWAVES + (threadIdx.x >> 6)];\n#endif\n";
    o << "  kv_end_flush(O, s_stw, " << nr << "u, " << name << "_rules, n_res, r, valid, "
         "(KV_OFULL(O) & 8u) && valid ? O.scope[r] : 0xFFFFFFFFu, (KV_OFULL(O) & 8u) && wg0_ < n_res ? O.scope[wg0_] : 0xFFFFFFFFu, "
         "P.n_rules);\n";
    stamp(std::min<size_t>(blocks.size() + 1, kJitStamps - 1));
    o << "}\n\n";
    hist_lds = false;
    return rules;
  }

  // Factored match descriptors (DevPS::fac_*, kv_mfac / kv_mtup in kvkernel.hip) for the
  // match bits of every rule in kernel order. A rule's match is an OR of planes minus an OR
  // of exclude planes (rule_matches, kvdevfn.h): `any` blocks give one plane per filter,
  // `all` blocks one plane of all their filters, a legacy block one plane of its filter. A
  // word takes as many match / exclude planes as its widest rule; rules with name filters
  // keep their per-resource bit, rules with more than KV_FAC_MAXP planes run rule_matches per
  // tuple.
  void build_fac(JitImage* out) const {
    const uint32_t W = (uint32_t)(mt_bits.size() / 32u);
    out->fac_word.assign(4u * W, 0u);
    out->fac_bit.clear();
    out->fac_flist.clear();
    out->fac_rule = mt_bits;
    auto planes = [&](uint32_t mode, uint32_t first, uint32_t count) {
      std::vector<std::vector<uint32_t>> p;
      if (mode == 1) {
        for (uint32_t f = first; f < first + count; f++) p.push_back({f});
      } else if (mode == 2) {
        std::vector<uint32_t> all;
        for (uint32_t f = first; f < first + count; f++) all.push_back(f);
        p.push_back(all);
      } else {
        p.push_back({first});
      }
      return p;
    };
    uint32_t slot = 0;
    for (uint32_t w = 0; w < W; w++) {
      std::vector<std::vector<std::vector<uint32_t>>> mp(32), xp(32);
      uint32_t nm = 0, nx = 0, named = 0, cx = 0;
      for (uint32_t b = 0; b < 32u; b++) {
        const uint32_t ri = mt_bits[w * 32u + b];
        if (ri == 0xFFFFFFFFu) continue;
        if (name_dependent(ri)) {
          named |= 1u << b;
          continue;
        }
        const RuleRec& rr = ps.rules[ri];
        auto m = planes(rr.m_mode, rr.m_first, rr.m_count), x = planes(rr.x_mode, rr.x_first, rr.x_count);
        if (m.size() > KV_FAC_MAXP || x.size() > KV_FAC_MAXP) {
          cx |= 1u << b;
          continue;
        }
        nm = std::max<uint32_t>(nm, (uint32_t)m.size());
        nx = std::max<uint32_t>(nx, (uint32_t)x.size());
        mp[b] = std::move(m);
        xp[b] = std::move(x);
      }
      out->fac_word[4u * w] = slot;
      out->fac_word[4u * w + 1] = nm | nx << 8;
      out->fac_word[4u * w + 2] = named;
      out->fac_word[4u * w + 3] = cx;
      for (uint32_t p = 0; p < nm + nx; p++, slot++)
        for (uint32_t b = 0; b < 32u; b++) {
          const auto& pl = p < nm ? mp[b] : xp[b];
          const uint32_t k = p < nm ? p : p - nm;
          if (k < pl.size()) {
            out->fac_bit.push_back((uint32_t)out->fac_flist.size());
            out->fac_bit.push_back((uint32_t)pl[k].size() | KV_FAC_PRESENT);
            out->fac_flist.insert(out->fac_flist.end(), pl[k].begin(), pl[k].end());
          } else {
            out->fac_bit.push_back(0u);
            out->fac_bit.push_back(0u);
          }
        }
    }
    out->fac_slots = slot;
    if (out->fac_flist.empty()) out->fac_flist.push_back(0u);
    if (out->fac_bit.empty()) out->fac_bit.assign(2, 0u);
  }

  // Register weight of rule ri in a fused block: the state it keeps across the block (status
  // / resume pc, error kind, cursors per depth, loop counters and error indices per loop
  // level, anchor bitsets, wildcard-key node); 0 for rules of other routes.
  uint32_t rule_weight(uint32_t ri) {
    if (ps.rules[ri].route != 0) return 0;
    const RGen g = analyze(ri);
    uint32_t w = 2 + g.maxd;
    if (!g.loops.empty()) w += 4 * (g.max_level + 1);
    if (g.uses_anchor) w += 4;
    if (g.uses_keyglob) w += 3;
    return w;
  }

  // First block sizes of the kernel of sorted rules [a, e): greedy runs whose weight stays
  // within a budget (KVGPU_JIT_BLOCK_W, default 160, see below); a rule of the same structural
  // form as an earlier rule of the run joins it for free (rule groups run its program once).
  // A kernel the default budget cuts into many blocks is cut again with 1.5x the budget: it
  // re-walks its resources once per block, and the block probes still split whatever does not
  // fit its registers (round 4, gpurun_out/ab9 / ab8, ms per pass: C5 3.45 -> 3.25, C4 1.00 ->
  // 0.99; C2, three blocks, keeps the default: with 1.5x 0.694 -> 0.712).
  std::vector<uint32_t> initial_blocks(const std::vector<uint32_t>& sorted, uint32_t a, uint32_t e) {
    const char* bw = getenv("KVGPU_JIT_BLOCK_W");
    if (bw && atoi(bw) > 0) return initial_blocks_w(sorted, a, e, (uint32_t)atoi(bw));
    std::vector<uint32_t> out = initial_blocks_w(sorted, a, e, 160u);
    if (out.size() >= 6) out = initial_blocks_w(sorted, a, e, 240u);
    return out;
  }
  std::vector<uint32_t> initial_blocks_w(const std::vector<uint32_t>& sorted, uint32_t a, uint32_t e, uint32_t budget) {
    std::vector<uint32_t> out;
    std::set<std::string> forms;
    uint32_t cur = 0, w = 0;
    for (uint32_t q = a; q < e; q++) {
      const uint32_t ri = sorted[q];
      std::vector<uint32_t> pr, pn, lp;
      const std::string f = group_form(ri, &pr, &pn, &lp);
      const uint32_t rw = !f.empty() && forms.count(f) ? 0u : rule_weight(ri);
      if (cur > 0 && w + rw > budget) {
        out.push_back(cur);
        cur = 0;
        w = 0;
        forms.clear();
      }
      cur++;
      w += !f.empty() && forms.count(f) ? 0u : rule_weight(ri);
      if (!f.empty()) forms.insert(f);
    }
    if (cur) out.push_back(cur);
    return out;
  }
};

// Sort key grouping rules with the same walk: the symbolic path of the first
// top-level array loop, then the sorted paths of the leaves it tests.
std::string rule_signature(const PolicySet& ps, uint32_t ri) {
  std::vector<std::string> expr(64);
  expr[0] = "R";
  std::string arr;
  std::vector<std::string> leaves;
  int nest = 0;
  for (uint32_t pc = ps.rules[ri].prog;; pc++) {
    const Inst& in = ps.prog[pc];
    const uint32_t op = in.op & 0xFF, d = (in.op >> 8) & 0xFF, aux = (in.op >> 16) & 0xFF;
    if (op == OP_DONE || d + 1 >= expr.size()) break;
    switch (op) {
      case OP_KEY:
      case OP_KEYV:
        expr[d + 1] = expr[d].empty() ? "" : expr[d] + ((aux & AUX_SCAN) ? "/k" : "/s") + std::to_string(in.a);
        break;
      case OP_LEAF:
        leaves.push_back(expr[d]);
        break;
      case OP_LOOP_BEGIN:
      case OP_EXIST_BEGIN:
        if (op == OP_LOOP_BEGIN && nest == 0 && arr.empty()) {
          arr = expr[d].empty() ? "?" : expr[d];
          expr[d + 1] = "E";
        } else {
          expr[d + 1].clear();
        }
        nest++;
        break;
      case OP_LOOP_END:
      case OP_EXIST_END:
        nest--;
        break;
      case OP_KEYGLOB:
      case OP_INDEX:
        expr[d + 1].clear();
        break;
      default:
        break;
    }
  }
  std::sort(leaves.begin(), leaves.end());
  std::string sig = (arr.empty() ? "~" : arr) + "|";
  for (auto& l : leaves) sig += l + ",";
  return sig;
}

// The kinds rule ri's match blocks admit ("*" when any block admits every kind): rules of
// one kind set then share blocks, which the kind-grouped store order lets whole waves skip
std::string rule_kind_key(const PolicySet& ps, uint32_t ri) {
  const RuleRec& rr = ps.rules[ri];
  std::vector<std::string> ks;
  for (uint32_t f = rr.m_first; f < rr.m_first + rr.m_count; f++) {
    const MFilter& F = ps.filters[f];
    if (!(F.flags & MF_KINDS)) return "*";
    for (uint32_t i = F.kinds_first; i < F.kinds_first + F.kinds_count; i++) {
      const KindSpec& k = ps.kinds[i];
      if (k.form == 3) return "*";
      ks.push_back(std::to_string(k.kind));
    }
  }
  std::sort(ks.begin(), ks.end());
  ks.erase(std::unique(ks.begin(), ks.end()), ks.end());
  std::string key;
  for (auto& k : ks) key += k + ",";
  return key;
}

}  // namespace

uint32_t jit_chunk_rules() {
  const char* ch = getenv("KVGPU_JIT_CHUNK");
  // (at most KV_KROWS: the kernels' record counters have a byte per (wave, rule))
  return ch && atoi(ch) > 0 ? std::min<uint32_t>((uint32_t)atoi(ch), KV_KROWS) : KV_KROWS;
}

void jit_generate(const PolicySet& ps, uint32_t chunk_rules, JitImage* out) {
  auto t0 = std::chrono::steady_clock::now();
  Gen g(ps);
  // KVGPU_JIT_DIAG=A,B: diagnostics-only kernel variants (#define KV_DIAG_A ... ahead of the
  // prelude; their results are wrong)
  std::string diag;
  if (const char* dg = getenv("KVGPU_JIT_DIAG")) {
    const std::string d = dg;
    for (size_t at = 0; at <= d.size();) {
      const size_t nx = d.find(',', at);
      const std::string t = d.substr(at, nx == std::string::npos ? std::string::npos : nx - at);
      if (!t.empty()) diag += "#define KV_DIAG_" + t + " 1\n";
      if (nx == std::string::npos) break;
      at = nx + 1;
    }
  }
  const std::string prelude =
      diag + kPrelude + std::string("\nusing namespace kv;\n\n") +
      "__device__ __noinline__ bool kv_dleaf_impl(const DevBatch& B, const Node* __restrict__ N, uint32_t dp, Node vn);\n\n";
  for (uint32_t ri = 0; ri < ps.rules.size(); ri++)
    if (ps.rules[ri].route == 0) g.leaf_classes(ri);
  for (uint32_t ri = 0; ri < ps.rules.size(); ri++) g.match_fn(ri);
  out->chunks.clear();
  const uint32_t n = (uint32_t)ps.rules.size();
  if (chunk_rules == 0 || chunk_rules > KV_KROWS) chunk_rules = KV_KROWS;
  {
    // rules that walk the same arrays and leaves share a kernel (and its hoisted lookups)
    std::vector<std::pair<std::string, uint32_t>> order;
    // rules grouped by the kinds they match first, walk signature second (round 3: C5 4.07 ->
    // 3.72 ms against signature only, C3 10.19 -> 10.32)
    for (uint32_t ri = 0; ri < n; ri++)
      order.push_back({ps.rules[ri].route == 0 ? "0" + rule_kind_key(ps, ri) + "#" + rule_signature(ps, ri) : "1", ri});
    std::stable_sort(order.begin(), order.end());
    // One kernel per range of the signature order: its rules run as one fused block (every
    // array they walk is walked once per resource, all rules of the range in one loop over
    // it). Default: ceil(n / chunk_rules) ranges of near-equal size.
    // KVGPU_JIT_WAVES: launch bound in waves per SIMD (default 8, 0: none)
    if (out->plan.empty() && n) {
      // first bound: about 160 KB / (256 B x rules) waves, at most 8 and at most what the
      // kernel's LDS (kernel_lds) leaves of a CU's 160 KB (one workgroup = one wave per SIMD);
      // the spill plan splits blocks (or lowers the bound) until the compiler meets it. A kernel
      // of many rules keeps more state live across its fused blocks, and trading occupancy for
      // fewer, larger blocks (fewer walks of the resource tree) wins there: C2 (100 rules, one
      // kernel) 6 waves 4 blocks 0.697 ms, 7 waves 16 blocks 0.902 ms, 8 waves 35 blocks
      // 1.224 ms per pass (round 4, gpurun_out/r4b/ab); C4's ~70-rule kernels run at 8.
      const char* wz = getenv("KVGPU_JIT_WAVES");
      uint32_t parts = (n + chunk_rules - 1) / chunk_rules;
      // one more range while the longest ranges would get fewer workgroups per CU than the
      // shortest (C3: 1 973 rules in 16 ranges of 123/124 -> 17 of 116/117)
      while (parts < n && Gen::lds_waves((n + parts - 1) / parts) < Gen::lds_waves(n / parts)) parts++;
      std::vector<uint32_t> sorted;
      for (auto& o : order) sorted.push_back(o.second);
      for (uint32_t k = 0; k < parts; k++) {
        const uint32_t a = (uint32_t)((uint64_t)n * k / parts), e = (uint32_t)((uint64_t)n * (k + 1) / parts);
        std::vector<uint32_t> bl = g.initial_blocks(sorted, a, e);
        // workgroups of 4 waves: waves per SIMD = workgroups per CU the LDS admits
        const int lds_waves = Gen::lds_waves(e - a);
        const int rule_waves = (int)std::max<uint32_t>(1u, (160u * 1024u) / std::max<uint32_t>(1u, (e - a) * 256u));
        out->plan.push_back({a, e - a, wz ? atoi(wz) : std::min({8, lds_waves, rule_waves}), bl});
      }
    }
    for (const JitKernelPlan& kp : out->plan) {
      JitChunk kc;
      // named by its rule range and block count: stable when other ranges are re-planned
      kc.name = "kvj_r" + std::to_string(kp.first) + "_" + std::to_string(kp.count) +
                (kp.blocks.size() > 1 ? "_b" + std::to_string(kp.blocks.size()) : "") + (kp.waves ? "" : "u");
      for (uint32_t q = kp.first; q < kp.first + kp.count; q++) kc.rules.push_back(order.at(q).second);
      std::vector<JitChunk> bl;
      uint32_t at = 0;
      for (uint32_t c : kp.blocks) {
        JitChunk b;
        b.rules.assign(kc.rules.begin() + at, kc.rules.begin() + at + c);
        at += c;
        bl.push_back(std::move(b));
      }
      if (at != kp.count) throw std::runtime_error("kvjit: kernel plan blocks do not cover its rules");
      std::vector<const JitChunk*> bp;
      for (auto& b : bl) bp.push_back(&b);
      // the kernel's rules in LDS-row order (blocks reorder rule-group members)
      kc.rules = g.group_kernel(kc.name, bp, kp.waves);
      out->chunks.push_back(kc);
    }
  }
  out->mtup_words = (uint32_t)(g.mt_bits.size() / 32u);
  if (out->mtup_words && !out->probe) g.build_fac(out);
  out->rec_compact.assign(n, 1);
  for (uint32_t ri = 0; ri < n; ri++) out->rec_compact[ri] = g.rec_slot[ri] ? 0 : 1;
  out->gs_desc = g.gs_desc;
  out->gs_mem = g.gs_mem;
  out->gs_members = g.gs_members;
  std::string cdefs;  // the column count of every path-column family (KVC_J<f>)
  g.col_plan(out, &cdefs);

  out->memo_preds.clear();
  out->memo_words = 0;
  if (!g.mpreds.empty() && !out->probe) {
    g.ptab_kernel();
    out->memo_preds = g.mpreds;
    out->memo_words = (uint32_t)((g.mpreds.size() + 31) / 32);
    out->ptab_row = g.ptab_row_out();
  }
  // Each kernel program = prelude + the helper functions it reaches + the kernel:
  // helpers (g_glob_/g_atom_/g_pred_/m_pred_/g_blk_/g_match_/g_rule_) are split at
  // their definitions and selected by a transitive scan of the identifiers they
  // use, in generation order (which is dependency order).
  const std::string helpers = g.o.str();
  std::vector<std::pair<std::string, std::string>> defs;  // (name, text)
  {
    const std::string mark = "__device__ __forceinline__ ";
    size_t at = helpers.find(mark);
    while (at != std::string::npos) {
      size_t next = helpers.find("\n" + mark, at + 1);
      const size_t end = next == std::string::npos ? helpers.size() : next + 1;
      const std::string text = helpers.substr(at, end - at);
      const size_t nb = text.find(' ', mark.size() + 1) + 1;  // after the return type
      const size_t ne = text.find('(', nb);
      defs.push_back({text.substr(nb, ne - nb), text});
      at = next == std::string::npos ? std::string::npos : next + 1;
    }
  }
  std::unordered_map<std::string, size_t> def_index;
  for (size_t i = 0; i < defs.size(); i++) def_index[defs[i].first] = i;
  auto refs = [&](const std::string& text, std::vector<size_t>* out_ids) {
    static const char* prefixes[] = {"g_glob_", "g_atom_", "g_pred_", "g_blk_", "g_match_",
                                     "g_dleaf_", "q_glob_", "q_atom_", "q_pred_", "r_glob_", "r_atom_", "r_pred_"};
    for (const char* pf : prefixes) {
      const size_t pl = strlen(pf);
      for (size_t q = text.find(pf); q != std::string::npos; q = text.find(pf, q + pl)) {
        size_t e = q + pl;
        while (e < text.size() && isdigit((unsigned char)text[e])) e++;
        auto it = def_index.find(text.substr(q, e - q));
        if (it != def_index.end()) out_ids->push_back(it->second);
      }
    }
  };
  out->common = prelude;
  out->kernel_name.clear();
  out->kernel_src.clear();
  out->source = prelude + cdefs + helpers;
  for (auto& k : g.kernels) {
    std::vector<char> used(defs.size(), 0);
    std::vector<size_t> stack;
    refs(k.second, &stack);
    while (!stack.empty()) {
      const size_t d = stack.back();
      stack.pop_back();
      if (used[d]) continue;
      used[d] = 1;
      refs(defs[d].second, &stack);
    }
    std::string prog;
    for (size_t d = 0; d < defs.size(); d++)
      if (used[d]) prog += defs[d].second;
    out->kernel_name.push_back(k.first);
    out->kernel_src.push_back(cdefs + prog + k.second);
    out->source += k.second;
  }
  out->gen_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

namespace {

uint64_t fnv1a64(const std::string& a, uint64_t h = 1469598103934665603ull) {
  for (unsigned char c : a) h = (h ^ c) * 1099511628211ull;
  return h;
}

std::string cache_dir() {
  const char* e = getenv("KVGPU_JIT_CACHE");
  if (e && std::string(e) == "0") return "";
  if (e && *e) return e;
  if (const char* x = getenv("XDG_CACHE_HOME"); x && *x) return std::string(x) + "/kvgpu";
  if (const char* h = getenv("HOME"); h && *h) return std::string(h) + "/.cache/kvgpu";
  return "";
}

bool read_file(const std::string& path, std::vector<char>* out) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  out->resize(n > 0 ? (size_t)n : 0);
  const bool ok = n > 0 && fread(out->data(), 1, (size_t)n, f) == (size_t)n;
  fclose(f);
  return ok;
}

void write_file_atomic(const std::string& dir, const std::string& path, const std::vector<char>& data) {
  std::string cmd = dir;  // create the directory (one level under an existing parent is enough here)
  for (size_t i = 1; i <= cmd.size(); i++)
    if (i == cmd.size() || cmd[i] == '/') mkdir(cmd.substr(0, i).c_str(), 0755);
  const std::string tmp = path + ".tmp." + std::to_string((unsigned long long)getpid()) + "." +
                          std::to_string(std::hash<std::thread::id>()(std::this_thread::get_id()));
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) return;
  const bool ok = fwrite(data.data(), 1, data.size(), f) == data.size();
  fclose(f);
  if (!ok || rename(tmp.c_str(), path.c_str()) != 0) unlink(tmp.c_str());
}

const char* const kOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-unused-label", "-Wno-unused-variable"};

std::vector<char> compile_one(const std::string& src, const std::string& name) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), (name + ".hip").c_str(), 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    throw std::runtime_error("hiprtcCreateProgram failed");
  hiprtcResult rc = hiprtcCompileProgram(prog, (int)(sizeof kOpts / sizeof kOpts[0]), kOpts);
  if (rc != HIPRTC_SUCCESS) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls, '\0');
    if (ls) hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    throw std::runtime_error("hiprtc compile of " + name + " failed: " + log.substr(0, 4000));
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  std::vector<char> code(cs);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  return code;
}

// kvjitc next to libkvgpu.so (KVGPU_JITC overrides): compiles one program per process
std::string jitc_path() {
  if (const char* e = getenv("KVGPU_JITC")) return e;
  Dl_info info{};
  if (!dladdr((void*)&jitc_path, &info) || !info.dli_fname) return "";
  std::string p = info.dli_fname;
  const size_t slash = p.rfind('/');
  p = (slash == std::string::npos ? std::string(".") : p.substr(0, slash)) + "/kvjitc";
  return access(p.c_str(), X_OK) == 0 ? p : "";
}

// cores this process may use: affinity, capped by a cgroup v2 CPU quota
unsigned host_threads() {
  unsigned n = std::thread::hardware_concurrency();
  cpu_set_t cs;
  if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = (unsigned)CPU_COUNT(&cs);
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    unsigned long long per = 0;
    if (fscanf(f, "%31s %llu", q, &per) == 2 && strcmp(q, "max") != 0 && per)
      n = std::min<unsigned>(n, (unsigned)std::max(1ull, strtoull(q, nullptr, 10) / per));
    fclose(f);
  }
  return std::max(1u, n);
}

// compile programs `todo` of img in child processes (kvjitc), `T` at a time
void compile_in_children(JitImage* img, const std::vector<size_t>& todo, const std::string& jitc, unsigned T) {
  const char* td = getenv("TMPDIR");
  std::string tmpl = std::string(td && *td ? td : "/tmp") + "/kvjit.XXXXXX";
  std::vector<char> tbuf(tmpl.begin(), tmpl.end());
  tbuf.push_back('\0');
  if (!mkdtemp(tbuf.data())) throw std::runtime_error("kvjit: mkdtemp failed");
  const std::string dir(tbuf.data());
  std::atomic<size_t> next{0}, done{0};
  std::vector<std::string> errs(T);
  // KVGPU_PROGRESS=1: a line on stderr at most every 15 s (long compiles stay visibly alive)
  const bool progress = getenv("KVGPU_PROGRESS") && getenv("KVGPU_PROGRESS")[0] == '1';
  const auto t0 = std::chrono::steady_clock::now();
  std::atomic<int64_t> last_ms{0};
  std::vector<std::thread> th;
  for (unsigned t = 0; t < T; t++)
    th.emplace_back([&, t]() {
      for (size_t j; (j = next++) < todo.size();) {
        const size_t i = todo[j];
        const std::string src = dir + "/" + std::to_string(i) + ".hip", out = dir + "/" + std::to_string(i) + ".co";
        {
          FILE* f = fopen(src.c_str(), "wb");
          const std::string prog = img->common + img->kernel_src[i];
          if (!f || fwrite(prog.data(), 1, prog.size(), f) != prog.size()) {
            errs[t] = "kvjit: cannot write " + src;
            if (f) fclose(f);
            return;
          }
          fclose(f);
        }
        std::vector<std::string> av = {jitc, src, out, img->kernel_name[i]};
        std::vector<char*> argv;
        for (auto& a : av) argv.push_back(&a[0]);
        argv.push_back(nullptr);
        pid_t pid = 0;
        if (posix_spawn(&pid, jitc.c_str(), nullptr, nullptr, argv.data(), environ) != 0) {
          errs[t] = "kvjit: cannot start " + jitc;
          return;
        }
        int status = 0;
        while (waitpid(pid, &status, 0) < 0 && errno == EINTR) {
        }
        std::vector<char> code;
        if (!WIFEXITED(status) || WEXITSTATUS(status) != 0 || !read_file(out, &code)) {
          errs[t] = "kvjit: compiling " + img->kernel_name[i] + " failed (kvjitc status " + std::to_string(status) + ")";
          return;
        }
        img->codes[i] = std::move(code);
        unlink(src.c_str());
        unlink(out.c_str());
        const size_t d = ++done;
        if (progress) {
          const int64_t now =
              (int64_t)std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
          int64_t prev = last_ms.load();
          if (now - prev >= 15000 && last_ms.compare_exchange_strong(prev, now))
            fprintf(stderr, "[kvgpu] hiprtc: %zu/%zu kernel programs compiled (%.0f s)\n", d, todo.size(), now / 1e3);
        }
      }
    });
  for (auto& x : th) x.join();
  rmdir(dir.c_str());
  for (auto& e : errs)
    if (!e.empty()) throw std::runtime_error(e);
}

}  // namespace

// Private (scratch) segment size and code size of kernel `name` in a gfx950 code
// object: the kernel descriptor `<name>.kd` (offset 4: private_segment_fixed_size)
// and the size of the function symbol. A non-zero private segment in these
// kernels means register spills (they keep no arrays on the stack).
bool co_kernel_info(const std::vector<char>& co, const std::string& name, uint32_t* private_seg, uint64_t* code,
                    uint32_t* vgprs) {
  auto rd = [&](size_t off, size_t n, void* out) {
    if (off + n > co.size()) return false;
    memcpy(out, co.data() + off, n);
    return true;
  };
  if (co.size() < 64 || memcmp(co.data(), "\x7f" "ELF", 4) != 0 || co[4] != 2) return false;
  uint64_t shoff = 0;
  uint16_t shentsize = 0, shnum = 0;
  rd(0x28, 8, &shoff);
  rd(0x3A, 2, &shentsize);
  rd(0x3C, 2, &shnum);
  struct Sh { uint32_t name, type; uint64_t flags, addr, off, size; uint32_t link, info; uint64_t align, entsize; };
  std::vector<Sh> sh(shnum);
  for (uint16_t i = 0; i < shnum; i++)
    if (!rd(shoff + (uint64_t)i * shentsize, sizeof(Sh), &sh[i])) return false;
  bool kd = false, fn = false;
  for (const Sh& t : sh) {
    if (t.type != 2 /* SHT_SYMTAB */ || t.link >= shnum) continue;
    const Sh& strtab = sh[t.link];
    for (uint64_t o = t.off; o + 24 <= t.off + t.size; o += 24) {
      uint32_t nm = 0;
      uint16_t shndx = 0;
      uint64_t value = 0, size = 0;
      rd(o, 4, &nm);
      rd(o + 6, 2, &shndx);
      rd(o + 8, 8, &value);
      rd(o + 16, 8, &size);
      if (strtab.off + nm >= co.size()) continue;
      const char* sn = co.data() + strtab.off + nm;
      const size_t maxlen = co.size() - (strtab.off + nm);
      const std::string sym(sn, strnlen(sn, maxlen));
      if (sym == name + ".kd" && shndx < shnum) {
        const Sh& sec = sh[shndx];
        kd = rd(sec.off + (value - sec.addr) + 4, 4, private_seg);
        // compute_pgm_rsrc1 (descriptor offset 48): granulated VGPR count, 8-register granules
        // of the unified (arch + acc) file on gfx950
        uint32_t rsrc1 = 0;
        if (kd && vgprs && rd(sec.off + (value - sec.addr) + 48, 4, &rsrc1)) *vgprs = ((rsrc1 & 0x3Fu) + 1u) * 8u;
      } else if (sym == name) {
        *code = size;
        fn = true;
      }
    }
  }
  return kd && fn;
}

// SGPR spill count of a code object's kernel from its AMDGPU metadata note (msgpack:
// ".sgpr_spill_count" then a positive fixint / uint8 / uint16 / uint32; one kernel per object).
// SGPRs spill into VGPR lanes (v_writelane / v_readlane), not into the private segment.
uint32_t co_sgpr_spills(const std::vector<char>& co) {
  static const char key[] = "\xb1.sgpr_spill_count";
  const auto it = std::search(co.begin(), co.end(), key, key + sizeof key - 1);
  if (it == co.end()) return 0;
  const size_t at = (size_t)(it - co.begin()) + sizeof key - 1;
  if (at >= co.size()) return 0;
  const uint8_t t = (uint8_t)co[at];
  auto be = [&](size_t n) {
    uint32_t v = 0;
    for (size_t i = 0; i < n && at + 1 + i < co.size(); i++) v = v << 8 | (uint8_t)co[at + 1 + i];
    return v;
  };
  if (t < 0x80) return t;
  if (t == 0xcc) return be(1);
  if (t == 0xcd) return be(2);
  if (t == 0xce) return be(4);
  return 0;
}

bool jit_plan_spills(JitImage* img) {
  // No rule kernel ships with a private (scratch) segment, bounded or not (DESIGN.md §4
  // *Register plan*: every faulting round-1 build had one), and a bound is only kept when the
  // compiler met it. A kernel that spills under its bound of w waves per SIMD, or that takes
  // more than 512 / w registers, is recompiled at w - 1 (w = 1: without a bound); an unbounded
  // kernel that still spills is split in two; a single rule range that does is an error.
  std::vector<JitKernelPlan> next;
  bool changed = false;
  img->kernel_scratch.assign(img->plan.size(), 0);
  for (size_t k = 0; k < img->plan.size(); k++) {
    const JitKernelPlan& kp = img->plan[k];
    const std::string& name = img->chunks[k].name;
    uint32_t priv = 0, vgprs = 0;
    uint64_t code = 0;
    size_t ci = 0;
    while (ci < img->kernel_name.size() && img->kernel_name[ci] != name) ci++;
    if (ci == img->kernel_name.size() || !co_kernel_info(img->codes[ci], name, &priv, &code, &vgprs))
      throw std::runtime_error("kvjit: no kernel descriptor for " + name);
    img->kernel_scratch[k] = priv;
    const bool met = kp.waves == 0 || vgprs <= 512u / (uint32_t)kp.waves;
    // the out-of-line dynamic-leaf evaluator (pattern variables) keeps a call frame in
    // scratch: allowed in a kernel without a launch bound (the round-1 fault was spill code
    // under a bound), so such a kernel drops its bound instead of splitting blocks
    const bool calls = img->kernel_src[ci].find("kv_dleaf_impl") != std::string::npos;
    if ((priv == 0 || (calls && kp.waves == 0)) && met) {
      next.push_back(kp);
      continue;
    }
    changed = true;
    JitKernelPlan np = kp;
    if (calls && met && priv != 0) {
      np.waves = 0;
      next.push_back(np);
      continue;
    }
    size_t big = 0;
    for (size_t b = 1; b < np.blocks.size(); b++)
      if (np.blocks[b] > np.blocks[big]) big = b;
    if (kp.waves > 6 && np.blocks.size() > 1) {
      // the blocks met the bound alone (jit_refine_blocks) and the kernel still does not: the
      // pressure crosses blocks, which splitting one block at a time fixes only slowly (C4:
      // 20+ recompiles); a kernel of multi-block form gives up a wave first (down to 6)
      np.waves = kp.waves - 1;
    } else if (!np.blocks.empty() && np.blocks[big] > 1) {  // the largest block in two halves
      const uint32_t c = np.blocks[big], h = c / 2;
      np.blocks[big] = h;
      np.blocks.insert(np.blocks.begin() + big + 1, c - h);
    } else if (kp.waves > 1) {
      np.waves = kp.waves - 1;
    } else if (kp.waves == 1) {
      np.waves = 0;
    } else if (kp.count > 1) {
      const uint32_t h = kp.count / 2;
      next.push_back({kp.first, h, 0, std::vector<uint32_t>(h, 1u)});
      next.push_back({kp.first + h, kp.count - h, 0, std::vector<uint32_t>(kp.count - h, 1u)});
      continue;
    } else {
      throw std::runtime_error("kvjit: kernel " + name + " needs " + std::to_string(priv) +
                               " B of scratch per lane even without a launch bound");
    }
    next.push_back(np);
  }
  if (changed) img->plan = next;
  return changed;
}

void jit_compile_variants(JitImage* img) {
  img->variants.clear();
  for (uint32_t full : {3u, 8u}) {
    JitImage v;
    v.common = "#define KVJ_FULL " + std::to_string(full) + "u\n" + img->common;
    std::vector<size_t> at;  // program of each variant program
    for (size_t i = 0; i < img->kernel_name.size(); i++)
      if (img->kernel_name[i].rfind("kvj_r", 0) == 0) {
        v.kernel_name.push_back(img->kernel_name[i]);
        v.kernel_src.push_back(img->kernel_src[i]);
        at.push_back(i);
      }
    if (at.empty()) return;
    jit_compile(&v);
    img->compile_ms += v.compile_ms;
    JitImage::Variant out;
    out.full = full;
    out.codes.resize(img->kernel_name.size());
    for (size_t j = 0; j < at.size(); j++) {
      // the plan's bound of this kernel; the variant ships only where it meets the same register
      // rules as the generic kernel (no scratch, within the bound's registers)
      int waves = 0;
      for (size_t k = 0; k < img->chunks.size() && k < img->plan.size(); k++)
        if (img->chunks[k].name == v.kernel_name[j]) waves = img->plan[k].waves;
      uint32_t priv = 0, vgprs = 0;
      uint64_t code = 0;
      if (!co_kernel_info(v.codes[j], v.kernel_name[j], &priv, &code, &vgprs)) continue;
      const bool calls = v.kernel_src[j].find("kv_dleaf_impl") != std::string::npos;
      if ((priv != 0 && !(calls && waves == 0)) || (waves > 0 && vgprs > 512u / (uint32_t)waves)) continue;
      out.codes[at[j]] = std::move(v.codes[j]);
    }
    img->variants.push_back(std::move(out));
  }
}

void jit_refine_blocks(const PolicySet& ps, uint32_t chunk_rules, JitImage* img) {
  // Each block of the plan compiled alone as a probe kernel under its kernel's bound (small
  // programs, compiled in parallel); a block whose probe spills or exceeds the bound's
  // registers is split in two, and its halves are probed in the next round.
  for (int round = 0; round < 12; round++) {
    JitImage probe;
    probe.probe = true;
    std::vector<std::pair<size_t, size_t>> at;  // (kernel, block) of each probe
    for (size_t k = 0; k < img->plan.size(); k++) {
      const JitKernelPlan& kp = img->plan[k];
      if (kp.blocks.size() < 2 || kp.waves == 0) continue;
      uint32_t first = kp.first;
      for (size_t b = 0; b < kp.blocks.size(); b++) {
        if (kp.blocks[b] > 1) {
          probe.plan.push_back({first, kp.blocks[b], kp.waves, {kp.blocks[b]}});
          at.push_back({k, b});
        }
        first += kp.blocks[b];
      }
    }
    if (probe.plan.empty()) return;
    jit_generate(ps, chunk_rules, &probe);
    jit_compile(&probe);
    img->compile_ms += probe.compile_ms;
    std::vector<std::vector<char>> split(img->plan.size());
    bool any = false;
    for (size_t i = 0; i < probe.plan.size(); i++) {
      const std::string& name = probe.chunks[i].name;
      size_t ci = 0;
      while (ci < probe.kernel_name.size() && probe.kernel_name[ci] != name) ci++;
      uint32_t priv = 0, vgprs = 0;
      uint64_t code = 0;
      if (ci == probe.kernel_name.size() || !co_kernel_info(probe.codes[ci], name, &priv, &code, &vgprs))
        throw std::runtime_error("kvjit: no kernel descriptor for probe " + name);
      const bool calls = probe.kernel_src[ci].find("kv_dleaf_impl") != std::string::npos;
      if ((priv != 0 && !calls) || vgprs > 512u / (uint32_t)probe.plan[i].waves) {
        split[at[i].first].resize(img->plan[at[i].first].blocks.size(), 0);
        split[at[i].first][at[i].second] = 1;
        any = true;
      }
    }
    if (!any) return;
    for (size_t k = 0; k < img->plan.size(); k++) {
      if (split[k].empty()) continue;
      std::vector<uint32_t> nb;
      for (size_t b = 0; b < img->plan[k].blocks.size(); b++) {
        const uint32_t c = img->plan[k].blocks[b];
        if (split[k][b]) {
          nb.push_back(c / 2);
          nb.push_back(c - c / 2);
        } else {
          nb.push_back(c);
        }
      }
      img->plan[k].blocks = nb;
    }
  }
}

uint64_t code_bytes(const JitImage& img) {
  uint64_t n = 0;
  for (auto& c : img.codes) n += c.size();
  return n;
}

namespace {

// hash of the compiler options, hiprtc version and the common prelude of img's programs
uint64_t common_hash(const JitImage& img) {
  std::string opt_key;
  for (const char* o : kOpts) opt_key += std::string(o) + "\n";
  int hv = 0;
  (void)hiprtcVersion(&hv, &hv);
  opt_key += "hiprtc " + std::to_string(hv) + "\n";
  return fnv1a64(img.common, fnv1a64(opt_key));
}

// code-object cache file of kernel program i: <name>-<hash of options + program text>.co
std::string cache_file(const JitImage& img, size_t i, uint64_t hcommon) {
  char key[40];
  snprintf(key, sizeof key, "%016llx", (unsigned long long)fnv1a64(img.kernel_src[i], hcommon));
  return img.kernel_name[i] + "-" + key + ".co";
}

}  // namespace

std::string jit_plan_key(const JitImage& img) {
  uint64_t h = common_hash(img);
  for (size_t i = 0; i < img.kernel_src.size(); i++) h = fnv1a64(img.kernel_src[i], fnv1a64(img.kernel_name[i], h));
  char key[40];
  snprintf(key, sizeof key, "%016llx", (unsigned long long)h);
  return key;
}

bool jit_load_plan(const std::string& key, JitImage* img) {
  const std::string dir = cache_dir();
  std::vector<char> text;
  if (dir.empty() || !read_file(dir + "/plan-" + key + ".txt", &text)) return false;
  std::vector<JitKernelPlan> plan;
  std::string line;
  for (size_t i = 0; i <= text.size(); i++) {
    if (i < text.size() && text[i] != '\n') {
      line.push_back(text[i]);
      continue;
    }
    if (line.rfind("kernel ", 0) == 0) {  // kernel <first> <count> <waves> <block sizes...>
      JitKernelPlan kp{0, 0, 0, {}};
      const char* c = line.c_str() + 7;
      char* e = nullptr;
      kp.first = (uint32_t)strtoul(c, &e, 10);
      kp.count = (uint32_t)strtoul(e, &e, 10);
      kp.waves = (int)strtol(e, &e, 10);
      uint32_t sum = 0;
      while (*e) {
        char* f = nullptr;
        const unsigned long b = strtoul(e, &f, 10);
        if (f == e) break;
        kp.blocks.push_back((uint32_t)b);
        sum += (uint32_t)b;
        e = f;
      }
      if (sum != kp.count || kp.blocks.empty()) return false;
      plan.push_back(kp);
    }
    line.clear();
  }
  if (plan.empty()) return false;
  img->plan = plan;
  return true;
}

void jit_save_plan(const std::string& key, const JitImage& img) {
  const std::string dir = cache_dir();
  if (dir.empty()) return;
  std::string t;
  for (const JitKernelPlan& kp : img.plan) {
    t += "kernel " + std::to_string(kp.first) + " " + std::to_string(kp.count) + " " + std::to_string(kp.waves);
    for (uint32_t b : kp.blocks) t += " " + std::to_string(b);
    t += "\n";
  }
  // the code objects of the final kernels (tools/jit_warm.sh keeps these, drops the
  // intermediate probes and re-plans)
  const uint64_t hc = common_hash(img);
  for (size_t i = 0; i < img.kernel_src.size(); i++) t += "co " + cache_file(img, i, hc) + "\n";
  for (const JitImage::Variant& v : img.variants) {  // (the output-mode variants' code objects)
    JitImage w;
    w.common = "#define KVJ_FULL " + std::to_string(v.full) + "u\n" + img.common;
    w.kernel_src = img.kernel_src;
    w.kernel_name = img.kernel_name;
    const uint64_t hv = common_hash(w);
    for (size_t i = 0; i < img.kernel_src.size(); i++)
      if (i < v.codes.size() && !v.codes[i].empty()) t += "co " + cache_file(w, i, hv) + "\n";
  }
  write_file_atomic(dir, dir + "/plan-" + key + ".txt", std::vector<char>(t.begin(), t.end()));
}

void jit_compile(JitImage* img) {
  auto t0 = std::chrono::steady_clock::now();
  const size_t K = img->kernel_src.size();
  img->codes.assign(K, {});
  img->cache_hits = 0;
  const std::string dir = cache_dir();
  const uint64_t hcommon = common_hash(*img);
  // cache lookups; the misses compile in child processes (hiprtc serialises the
  // compilations of one process), or in this process when kvjitc is unavailable
  // (KVGPU_JIT_PROCS=0 forces that)
  std::vector<std::string> paths(K);
  std::vector<size_t> todo;
  uint32_t hits = 0;
  for (size_t i = 0; i < K; i++) {
    paths[i] = dir.empty() ? "" : dir + "/" + cache_file(*img, i, hcommon);
    if (!paths[i].empty() && read_file(paths[i], &img->codes[i])) hits++;
    else todo.push_back(i);
  }
  unsigned T = std::min(16u, host_threads());
  if (const char* e = getenv("KVGPU_JIT_THREADS")) T = (unsigned)std::max(1, atoi(e));
  T = std::max(1u, std::min<unsigned>(T, (unsigned)todo.size()));
  const std::string jitc = jitc_path();
  const bool procs = !(getenv("KVGPU_JIT_PROCS") && getenv("KVGPU_JIT_PROCS")[0] == '0');
  if (!todo.empty() && procs && !jitc.empty() && todo.size() > 1) {
    compile_in_children(img, todo, jitc, T);
  } else {
    for (size_t i : todo) img->codes[i] = compile_one(img->common + img->kernel_src[i], img->kernel_name[i]);
  }
  if (!dir.empty())
    for (size_t i : todo) write_file_atomic(dir, paths[i], img->codes[i]);
  img->cache_hits = hits;
  img->compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace kvh
