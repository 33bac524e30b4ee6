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

#include <chrono>
#include <cstdio>
#include <cstring>
#include <set>
#include <sstream>
#include <stdexcept>

#include "kvjit.hpp"

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

struct Gen {
  const PolicySet& ps;
  std::ostringstream o;
  std::set<uint32_t> preds_done, atoms_done;
  explicit Gen(const PolicySet& p) : ps(p) {}

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
      o << "  { bool found = false;\n"
        << "    for (uint32_t k = pos; k + " << u32(sg.len) << " <= end; k++)\n"
        << "      if (" << seg_expr(sg, "k", false) << ") { pos = k + " << u32(sg.len) << "; found = true; break; }\n"
        << "    if (!found) return false; }\n";
    }
    o << "  (void)pos; (void)end;\n  return true;\n}\n";
  }

  // ---------------------------------------------------------------- atoms / predicates
  void atom_fn(uint32_t ai) {
    if (!atoms_done.insert(ai).second) return;
    const Atom& A = ps.atoms[ai];
    if (A.kind == AT_GLOB_E || A.kind == AT_GLOB_N) glob_fn(ai);
    o << "__device__ __forceinline__ bool g_atom_" << ai
      << "(const Val* __restrict__ V, const uint8_t* __restrict__ S, const uint8_t* __restrict__ pstr, uint32_t type, "
         "const Node& n) {\n";
    switch (A.kind) {
      case AT_FALSE: o << "  return false;\n"; break;
      case AT_GLOB_E:
        o << "  if (type == NT_MAP || type == NT_ARR || type == NT_NULL) return false;\n"
          << "  const bool r = g_glob_" << ai << "(S + n.b, n.c & NC_LEN_MASK, (n.c & NC_ASCII_E) != 0u, pstr);\n"
          << "  return " << (A.op == CO_NE ? "!r" : "r") << ";\n";
        break;
      case AT_GLOB_N:
        o << "  if (type == NT_MAP || type == NT_ARR || type == NT_BOOL) return false;\n"
          << "  if (type == NT_NULL) return g_glob_" << ai << "(S, 1u, true, pstr);\n"
          << "  if (type != NT_FLOAT) return g_glob_" << ai << "(S + n.b, n.c & NC_LEN_MASK, (n.c & NC_ASCII_E) != 0u, pstr);\n"
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
    o << "__device__ __forceinline__ bool g_pred_" << pi
      << "(const Val* __restrict__ V, const uint8_t* __restrict__ S, const uint8_t* __restrict__ pstr, uint32_t type, "
         "const Node& n) {\n";
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
            auto call = [&](uint32_t at) { return "g_atom_" + std::to_string(at) + "(V, S, pstr, type, n)"; };
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

  // ---------------------------------------------------------------- match / exclude
  // blk_ok(f) == !(MF_EMPTY) && doesResourceMatchConditionBlock(f) has no errors
  // (pkg/engine/utils.go:265-336); MF_EMPTY / MF_UI_FAIL are folded per launch
  // (user info), so they are read from P.fflags; every other criterion is static.
  std::set<uint32_t> blks_done;
  void blk_fn(uint32_t f) {
    if (!blks_done.insert(f).second) return;
    const MFilter& F = ps.filters[f];
    o << "__device__ __forceinline__ bool g_blk_" << f
      << "(const DevPS& P, const DevBatch& B, const Res* __restrict__ R, uint32_t rkind, uint32_t rflags) {\n"
      << "  if (uni(P.fflags[" << f << "]) & (MF_EMPTY | MF_UI_FAIL)) return false;\n";
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
    auto glob_any = [&](uint32_t first, uint32_t count, const char* off, const char* len) {
      o << "  if (!(false";
      for (uint32_t i = first; i < first + count; i++)
        o << " || kv_glob(P.pstr + " << u32(ps.strrefs[i].off) << ", " << u32(ps.strrefs[i].len) << ", B.bstr + R->" << off
          << ", R->" << len << ")";
      o << ")) return false;\n";
    };
    if (F.flags & MF_NAME)
      o << "  if (!kv_glob(P.pstr + " << u32(F.name_off) << ", " << u32(F.name_len)
        << ", B.bstr + R->name_off, R->name_len)) return false;\n";
    if (F.flags & MF_NAMES) glob_any(F.names_first, F.names_count, "name_off", "name_len");
    if (F.flags & MF_NSS) glob_any(F.nss_first, F.nss_count, "ns_off", "ns_len");
    if (F.flags & (MF_ANN | MF_SEL))  // rarer criteria: the generic evaluator, restricted to them
      o << "  if (block_errs_masked(P, B, R, rkind, rflags, " << f << "u, MF_ANN | MF_SEL) != 0u) return false;\n";
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

  void rule_fn(uint32_t ri) {
    const RuleRec& rr = ps.rules[ri];
    const uint32_t b = rr.prog, e = prog_end(ps, rr.prog);
    uint32_t maxd = 1;
    for (uint32_t pc = b; pc <= e; pc++) {
      const Inst& in = ps.prog[pc];
      const uint32_t op = in.op & 0xFF, d = (in.op >> 8) & 0xFF;
      maxd = std::max(maxd, d + 2);
      if (op == OP_LEAF) pred_fn(in.a);
    }
    o << "__device__ __forceinline__ uint32_t g_rule_" << ri
      << "(const DevPS& P, const DevBatch& B, const Node* __restrict__ N, const Val* __restrict__ V, "
         "const uint8_t* __restrict__ S, uint32_t root, EState& e) {\n";
    o << "  uint32_t c0 = root";
    for (uint32_t d = 1; d < maxd; d++) o << ", c" << d << " = ABSENT";
    o << ";\n  uint32_t lf0 = 0u, lf1 = 0u, lf2 = 0u, lf3 = 0u, ll0 = 0u, ll1 = 0u, ll2 = 0u, ll3 = 0u;\n"
      << "  uint32_t li0 = 0u, li1 = 0u, li2 = 0u, li3 = 0u, keynode = ABSENT;\n"
      << "  uint64_t areg = 0ull, apres = 0ull;\n"
      << "  const uint8_t* __restrict__ pstr = P.pstr;\n"
      << "  (void)P; (void)B; (void)pstr; (void)lf0; (void)lf1; (void)lf2; (void)lf3; (void)ll0; (void)ll1; (void)ll2; "
         "(void)ll3; (void)keynode;\n";
    auto C = [](uint32_t d) { return "c" + std::to_string(d); };
    auto L = [](uint32_t pc) { return "L" + std::to_string(pc); };
    auto raise = [&](const std::string& kind, uint32_t pn, const std::string& res, uint32_t catch_pc) {
      if (catch_pc < b || catch_pc > e) throw std::runtime_error("kvjit: raising op without a catch target");
      std::ostringstream r;
      r << "{ e.kind = " << kind << "; e.flags = 0u; e.pn = " << u32(pn) << "; e.res = " << res
        << "; e.key = keynode; e.i0 = li0; e.i1 = li1; e.i2 = li2; e.i3 = li3; goto " << L(catch_pc) << "; }";
      return r.str();
    };
    for (uint32_t pc = b; pc <= e; pc++) {
      const Inst& in = ps.prog[pc];
      const uint32_t op = in.op & 0xFF, d = (in.op >> 8) & 0xFF, aux = (in.op >> 16) & 0xFF;
      const std::string cd = C(d), cn = C(d + 1);
      const std::string lv = std::to_string(aux & 3);
      o << L(pc) << ":;\n";
      switch (op) {
        case OP_MAPCHK:
        case OP_ARRCHK:
          o << "  if (" << cd << " == ABSENT || node_type(N[" << cd << "].kt) != " << (op == OP_MAPCHK ? "NT_MAP" : "NT_ARR")
            << ") " << raise(op == OP_MAPCHK ? "E_TYPE_MAP" : "E_TYPE_ARR", in.a, cd, in.c) << "\n";
          break;
        case OP_AREG: {
          const std::string bit = "(1ull << " + std::to_string(aux & 63) + ")";
          o << "  areg |= " << bit << "; if (lookup_op(N, " << cd << ", " << u32(in.a) << ", " << u32(aux)
            << ") != ABSENT) apres |= " << bit << ";\n";
          break;
        }
        case OP_KEY:
          o << "  " << cn << " = lookup_op(N, " << cd << ", " << u32(in.a) << ", " << u32(aux) << "); if (" << cn
            << " == ABSENT) goto " << L(in.b) << ";\n";
          break;
        case OP_KEYV:
          o << "  " << cn << " = lookup_op(N, " << cd << ", " << u32(in.a) << ", " << u32(aux) << ");\n";
          break;
        case OP_KEYGLOB:
          o << "  { uint32_t nd_; if (!keyglob_op(P, B, N, " << cd << ", " << u32(in.op) << ", " << u32(in.a) << ", "
            << u32(in.c) << ", &nd_, &keynode)) goto " << L(in.b) << "; " << cn << " = nd_; }\n";
          break;
        case OP_SCOPE_END:
          // c == 0: no wake-up target (interpreter: the lane keeps running)
          if (in.c == 0) o << "  if (e.kind) e.flags |= " << u32(aux) << ";\n";
          else o << "  if (e.kind) { e.flags |= " << u32(aux) << "; goto " << L(in.c) << "; }\n";
          break;
        case OP_POS_END:
          o << "  if (e.kind) { if (e.flags & EF_COND) e.kind = 0u; else goto " << L(in.c) << "; }\n";
          break;
        case OP_NEG:
          o << "  if (lookup_op(N, " << cd << ", " << u32(in.a) << ", " << u32(aux) << ") != ABSENT) "
            << raise("E_NEG", in.b, "ABSENT", in.c) << "\n";
          break;
        case OP_STAR:
          o << "  if (" << cn << " == ABSENT || node_type(N[" << cn << "].kt) == NT_NULL) "
            << raise("E_STAR", in.b, "ABSENT", in.c) << "\n";
          break;
        case OP_LEAF:
          o << "  { Node vn_{0u, 0u, 0u, 0u}; if (" << cd << " != ABSENT) vn_ = N[" << cd << "];\n"
            << "    const uint32_t vt_ = node_type(vn_.kt); bool ok_;\n"
            << "    if (vt_ == NT_ARR) { ok_ = true; for (uint32_t k_ = 0; k_ < vn_.b && ok_; k_++) { const Node en_ = N[ni(vn_.a + k_)]; "
            << "ok_ = g_pred_" << in.a << "(V, S, pstr, node_type(en_.kt), en_); } }\n"
            << "    else ok_ = g_pred_" << in.a << "(V, S, pstr, vt_, vn_);\n"
            << "    if (!ok_) " << raise("E_VALUE", in.b, cd, in.c) << " }\n";
          break;
        case OP_RAISE:
          o << "  " << raise(u32(in.b), in.a, cd, in.c) << "\n";
          break;
        case OP_EXISTCHK:
          o << "  if (" << cd << " == ABSENT || node_type(N[" << cd << "].kt) != NT_ARR) "
            << raise("E_EXIST_RESTYPE", in.a, cd, in.c) << "\n";
          break;
        case OP_LENCHK:
          o << "  if (N[" << cd << "].b < " << u32(in.a) << ") " << raise("E_LEN", in.b, cd, in.c) << "\n";
          break;
        case OP_INDEX:
          o << "  " << cn << " = ni(N[" << cd << "].a + " << u32(in.a) << ");\n";
          break;
        case OP_LOOP_BEGIN:
        case OP_EXIST_BEGIN:
          o << "  { const Node an_ = N[" << cd << "]; lf" << lv << " = an_.a; ll" << lv << " = an_.b; li" << lv
            << " = 0u;\n    if (an_.b == 0u) ";
          if (op == OP_LOOP_BEGIN) o << "goto " << L(in.a + 1) << ";";
          else o << raise("E_EXIST_FAIL", in.b, cd, in.c);
          o << "\n    " << cn << " = ni(an_.a); }\n";
          break;
        case OP_LOOP_END:
          o << "  if (e.kind) { if (e.flags & EF_COND) e.kind = 0u; else goto " << L(in.c) << "; }\n"
            << "  if (li" << lv << " + 1u < ll" << lv << ") { li" << lv << "++; " << cn << " = ni(lf" << lv << " + li" << lv
            << "); goto " << L(in.a + 1) << "; }\n";
          break;
        case OP_EXIST_END:
          o << "  if (!e.kind) goto " << L(pc + 1) << ";\n  e.kind = 0u;\n"
            << "  if (li" << lv << " + 1u < ll" << lv << ") { li" << lv << "++; " << cn << " = ni(lf" << lv << " + li" << lv
            << "); goto " << L(in.a + 1) << "; }\n"
            << "  " << raise("E_EXIST_FAIL", in.b, cd, in.c) << "\n";
          break;
        case OP_ALT_BEGIN:
          o << "  e.kind = 0u; e.flags = 0u; areg = 0ull; apres = 0ull;\n";
          break;
        case OP_ALT_END:
          o << "  if (e.kind == 0u) return ST_PASS;\n  if (e.kind == E_CPU) return ST_CPU;\n";
          if (in.b) o << "  return ST_FAIL;\n";
          else o << "  e.kind = 0u; e.flags = 0u; areg = 0ull; apres = 0ull;\n";
          break;
        case OP_DONE:
          o << "  if (e.kind == 0u) return ST_PASS;\n"
            << "  if (e.kind == E_CPU) return ST_CPU;\n"
            << "  if (e.flags & (EF_COND | EF_GLOBAL)) return ST_SKIP;\n"
            << "  if (areg & ~apres) return ST_ERROR;\n"
            << "  if (e.kind == E_LEN) return ST_ERROR;\n"
            << "  return ST_FAIL;\n";
          break;
        default:  // OP_NOP, OP_METACHK (handled per resource by RF_BAD_META)
          break;
      }
    }
    o << "}\n\n";
  }

  void chunk_kernel(const JitChunk& ch) {
    const uint32_t nr = ch.rule_end - ch.rule_begin;
    o << "extern \"C\" __global__ __launch_bounds__(KV_WG) void " << ch.name
      << "(const DevPS* __restrict__ Pp, const DevBatch* __restrict__ Bp, const Node* __restrict__ N, "
         "const Val* __restrict__ V, const uint8_t* __restrict__ S, DevOut O) {\n"
      << "  __shared__ uint32_t s_hist[" << nr << "][KV_HIST];\n"
      << "  const DevPS& P = *Pp;\n  const DevBatch& B = *Bp;\n"
      << "  for (uint32_t q = threadIdx.x; q < " << nr << "u * KV_HIST; q += KV_WG) (&s_hist[0][0])[q] = 0u;\n"
      << "  __syncthreads();\n"
      << "  const uint32_t r = blockIdx.x * KV_WG + threadIdx.x;\n"
      << "  const uint32_t n_res = B.n_res;\n"
      << "  const bool valid = r < n_res;\n"
      << "  const Res* __restrict__ R = B.res + (valid ? r : 0u);\n"
      << "  uint32_t root = ABSENT, rkind = KEY_NONE, rflags = 0u;\n"
      << "  if (valid) { root = ni(R->root); rkind = R->kind; rflags = R->flags; }\n";
    for (uint32_t ri = ch.rule_begin; ri < ch.rule_end; ri++) {
      const RuleRec& rr = ps.rules[ri];
      o << "  { // rule " << ri << "\n"
        << "    uint32_t st = ST_NOMATCH;\n"
        << "    EState e{0u, 0u, 0u, ABSENT, ABSENT, 0u, 0u, 0u, 0u};\n"
        << "    if (valid && g_match_" << ri << "(P, B, R, rkind, rflags)) {\n";
      switch (rr.route) {
        case 1: o << "      st = ST_CPU;\n"; break;
        case 2: o << "      st = ST_NOMATCH;\n"; break;
        case 3: o << "      st = " << u32(rr.const_status) << ";\n"; break;
        default:
          o << "      if (rflags & RF_MAGIC) st = ST_CPU;\n";
          if (rr.flags & RR_META_EXPAND) o << "      else if (rflags & RF_BAD_META) st = ST_CPU;\n";
          o << "      else st = g_rule_" << ri << "(P, B, N, V, S, root, e);\n";
          break;
      }
      o << "    }\n"
        << "    store_result(O, " << ri << "u, n_res, r, valid, st, e, &s_hist[" << (ri - ch.rule_begin) << "][0]);\n"
        << "  }\n";
    }
    o << "  __syncthreads();\n"
      << "  for (uint32_t q = threadIdx.x; q < " << nr << "u * KV_HIST; q += KV_WG) {\n"
      << "    const uint32_t v = (&s_hist[0][0])[q];\n"
      << "    if (v) atomicAdd(&O.counts[(size_t)" << ch.rule_begin << "u * KV_HIST + q], (unsigned long long)v);\n"
      << "  }\n}\n\n";
  }
};

}  // namespace

void jit_generate(const PolicySet& ps, uint32_t chunk_rules, JitImage* out) {
  auto t0 = std::chrono::steady_clock::now();
  Gen g(ps);
  g.o << kPrelude << "\nusing namespace kv;\n\n";
  for (uint32_t ri = 0; ri < ps.rules.size(); ri++) {
    g.match_fn(ri);
    if (ps.rules[ri].route == 0) g.rule_fn(ri);
  }
  out->chunks.clear();
  const uint32_t n = (uint32_t)ps.rules.size();
  if (chunk_rules == 0) chunk_rules = 32;
  for (uint32_t b = 0; b < n; b += chunk_rules) {
    JitChunk ch;
    ch.rule_begin = b;
    ch.rule_end = std::min(n, b + chunk_rules);
    ch.name = "kvj_chunk_" + std::to_string(out->chunks.size());
    g.chunk_kernel(ch);
    out->chunks.push_back(ch);
  }
  out->source = g.o.str();
  out->gen_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void jit_compile(JitImage* img) {
  auto t0 = std::chrono::steady_clock::now();
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, img->source.c_str(), "kvjit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    throw std::runtime_error("hiprtcCreateProgram failed");
  const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-unused-label", "-Wno-unused-variable"};
  hiprtcResult rc = hiprtcCompileProgram(prog, (int)(sizeof opts / sizeof opts[0]), opts);
  if (rc != HIPRTC_SUCCESS) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls, '\0');
    if (ls) hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    throw std::runtime_error("hiprtc compile failed: " + log.substr(0, 4000));
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  img->code.resize(cs);
  hiprtcGetCode(prog, img->code.data());
  hiprtcDestroyProgram(&prog);
  img->compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace kvh
