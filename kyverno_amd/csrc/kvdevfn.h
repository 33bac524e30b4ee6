// Device helpers shared by the bytecode interpreter (kvkernel.hip) and the
// specialized per-policy-set kernels generated at run time (kvjit.cpp, which
// embeds this file in its hiprtc prelude). Plain HIP device code: no includes.
#pragma once

#define KV_SENT 0xFFFFFFFFu


// Linkage of the shared helpers: the bytecode VM (kvkernel.hip) keeps the
// generic ones out of line; the specialized kernels' prelude (kvjit.cpp)
// defines KV_JIT_PRELUDE so everything is inlined and the rule kernels make no
// calls (calls under the 8-wave register bound spill caller-saved registers).
#ifdef KV_JIT_PRELUDE
#define KV_FN __device__ __forceinline__
#define KV_GLOB_FN __device__ __forceinline__
#else
#define KV_FN __device__
#define KV_GLOB_FN __device__ __noinline__
#endif

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Wave-uniform read of the read-only policy tables through the scalar data cache
// (s_load into SGPRs, batched, no vector-memory round trip per criterion). The
// device pointers in DevPS are generic; the cast names the constant address
// space. A divergent address still compiles (to a vector load).
#ifndef KV_SCONST
#define KV_SCONST __attribute__((address_space(4)))
#endif
template <class T>
__device__ __forceinline__ T sld(const T* p) {
  static_assert(sizeof(T) % 4 == 0, "sld: whole words");
  const KV_SCONST uint32_t* q = (const KV_SCONST uint32_t*)p;
  uint32_t w[sizeof(T) / 4];
#pragma unroll
  for (uint32_t i = 0; i < sizeof(T) / 4; i++) w[i] = q[i];
  T r;
  __builtin_memcpy(&r, w, sizeof(T));
  return r;
}

// Load through a global-address-space pointer: the tables reached through DevPS /
// DevBatch members are generic pointers, which the compiler lowers to flat loads
// (waiting on both the vector-memory and the LDS/scalar counters).
template <class T>
__device__ __forceinline__ T kv_gld(const T* p, size_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
  return ((const __attribute__((address_space(1))) T*)p)[i];
#else
  return p[i];
#endif
}

// Output mode of the launch (DevOut::full): a rule-kernel program compiled for one mode
// (kvjit.cpp output-mode variants, KVJ_FULL) has it as a constant, so the code of outputs its
// launches never write (records in SCOPES mode, the status copy in COUNTS mode) is not there
#ifdef KVJ_FULL
#define KV_OFULL(O) ((uint32_t)(KVJ_FULL))
#else
#define KV_OFULL(O) ((O).full)
#endif

// A node through a global-address-space pointer (kv_gld for a struct: the copy goes through a
// native vector, the fields the caller reads are the ones loaded). The path columns (DevBatch::
// pcol) are read this way: through the generic pointer they compiled to flat loads (C2: 100 of
// 305 loads), whose waits also drain the LDS / scalar counter.
__device__ __forceinline__ Node kv_ldn(const Node* p, size_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t u32x4_ __attribute__((ext_vector_type(4)));
  const u32x4_ v = ((const __attribute__((address_space(1))) u32x4_*)p)[i];
  return Node{v.x, v.y, v.z, v.w};
#else
  return p[i];
#endif
}

// path-column cell i (DevBatch::pcol / pcolb planes): its (kt, a, c) words as one 12-byte
// global-address-space load and its b word (an array's element count) as a 4-byte one, which
// only array cells need (a caller that never reads .b leaves it dead)
__device__ __forceinline__ Node kv_ldc(const uint32_t* pa, const uint32_t* pb, size_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
  // (a 12-byte cell is 4-byte aligned: the type says so, gfx950 loads it as one dwordx3)
  typedef uint32_t u32x3_ __attribute__((ext_vector_type(3), aligned(4)));
  const u32x3_ x = *(const __attribute__((address_space(1))) u32x3_*)((const __attribute__((address_space(1))) char*)pa + 12u * i);
  const uint32_t y = ((const __attribute__((address_space(1))) uint32_t*)pb)[i];
  return Node{x.x, x.y, y, x.z};
#else
  return Node{pa[3 * i], pa[3 * i + 1], pb[i], pa[3 * i + 2]};
#endif
}

// node index of this lane's cell in a row (wave-group layout, kv_layout.h)
__device__ __forceinline__ uint32_t ni(uint32_t row) { return row * KV_LANES + (threadIdx.x & (KV_LANES - 1)); }

__device__ __forceinline__ uint32_t rune_len(uint8_t c) {
  return c < 0x80 ? 1u : c >= 0xF0 ? 4u : c >= 0xE0 ? 3u : c >= 0xC0 ? 2u : 1u;
}

// minio/pkg v1.1.3 wildcard.Match over valid UTF-8: '*' any run of runes,
// '?' exactly one rune; star backtracking advances by whole runes.
// General path (non-ASCII value with '?' in the pattern, selector/label globs).
KV_GLOB_FN bool kv_glob(const uint8_t* p, uint32_t pl, const uint8_t* s, uint32_t sl) {
  if (pl == 0) return sl == 0;
  if (pl == 1 && p[0] == '*') return true;
  uint32_t si = 0, pi = 0, star = KV_SENT, mark = 0;
  while (si < sl) {
    if (pi < pl) {
      uint8_t pc = p[pi];
      if (pc == '*') { star = pi++; mark = si; continue; }
      if (pc == '?') { si += rune_len(s[si]); pi++; continue; }
      uint32_t w = rune_len(pc);
      bool eq = si + w <= sl && pi + w <= pl;
      for (uint32_t k = 0; eq && k < w; k++) eq = p[pi + k] == s[si + k];
      if (eq) { pi += w; si += w; continue; }
    }
    if (star != KV_SENT) {
      pi = star + 1;
      mark += rune_len(s[mark]);
      si = mark;
      continue;
    }
    return false;
  }
  while (pi < pl && p[pi] == '*') pi++;
  return pi == pl && si == sl;
}

// 64-bit mask of the byte positions p < 64 of the 16 words `w` whose byte may equal
// the byte replicated in c4 (SWAR zero-byte test of w ^ c4: every equal byte is
// flagged; a byte c4 ^ 1 right after an equal one can be flagged too, so callers
// verify each candidate). Straight-line: no per-lane loop.
__device__ __forceinline__ uint64_t kv_bmask(const uint32_t* w, uint32_t c4) {
  uint32_t lo = 0u, hi = 0u;
#pragma unroll
  for (uint32_t i = 0; i < 8; i++) {
    const uint32_t x = w[i] ^ c4, y = w[i + 8] ^ c4;
    // bits 7, 15, 23, 31 of m -> bits 28..31 of m * 0x00204081 (no carries between them)
    const uint32_t mx = (x - 0x01010101u) & ~x & 0x80808080u, my = (y - 0x01010101u) & ~y & 0x80808080u;
    lo |= ((mx * 0x00204081u) >> 28) << (4u * i);
    hi |= ((my * 0x00204081u) >> 28) << (4u * i);
  }
  return ((uint64_t)hi << 32) | lo;
}

// kv_bmask over the first nw words only (nw wave-uniform, a multiple of 4): the mask bits
// of later words are never read (candidates lie below the value length)
__device__ __forceinline__ uint32_t kv_bmask_q(const uint32_t* w, uint32_t c4, uint32_t q) {
  uint32_t r = 0u;  // words 4q .. 4q+3 -> mask bits 16q' .. (nibbles at 4 * (i % 8))
#pragma unroll
  for (uint32_t i = 0; i < 4; i++) {
    const uint32_t x = w[4 * q + i] ^ c4;
    const uint32_t m = (x - 0x01010101u) & ~x & 0x80808080u;
    r |= ((m * 0x00204081u) >> 28) << (4u * ((4 * q + i) & 7u));
  }
  return r;
}
__device__ __forceinline__ uint64_t kv_bmask_n(const uint32_t* w, uint32_t c4, uint32_t nw) {
  uint32_t lo = kv_bmask_q(w, c4, 0), hi = 0u;
  if (nw > 4u) lo |= kv_bmask_q(w, c4, 1);
  if (nw > 8u) hi = kv_bmask_q(w, c4, 2);
  if (nw > 12u) hi |= kv_bmask_q(w, c4, 3);
  return ((uint64_t)hi << 32) | lo;
}
// the smallest multiple of 4 words (<= W) covering the value of every active lane
__device__ __forceinline__ uint32_t kv_wave_words(uint32_t lastw, uint32_t W) {
  uint32_t n = W;
  while (n > 4u && __ballot(lastw > n - 4u) == 0ull) n -= 4u;
  return n;
}

// byte-position masks of values of <= 128 bytes (32 words): positions 0-63 in lo, 64-127 in hi
struct KvM2 {
  uint64_t lo, hi;
};
__device__ __forceinline__ KvM2 kv_bmask2(const uint32_t* w, uint32_t c4) { return {kv_bmask(w, c4), kv_bmask(w + 16, c4)}; }
__device__ __forceinline__ uint64_t kv_bmask_n(const uint32_t* w, uint32_t c4, uint32_t nw);
__device__ __forceinline__ KvM2 kv_bmask2_n(const uint32_t* w, uint32_t c4, uint32_t nw) {
  return {kv_bmask_n(w, c4, nw < 16u ? nw : 16u), nw > 16u ? kv_bmask_n(w + 16, c4, nw - 16u) : 0ull};
}

// candidate-mask helpers of the kvj_ptab register globs, on both mask types: the bits of m
// in [plo, phi] (none when !ok; plo <= phi < mask width when ok), non-empty test, lowest
// set position, lowest bit cleared
__device__ __forceinline__ uint64_t kv_mrange(uint64_t m, uint32_t plo, uint32_t phi, bool ok) {
  return ok ? m & (~0ull << plo) & (~0ull >> (63u - phi)) : 0ull;
}
__device__ __forceinline__ bool kv_mnz(uint64_t m) { return m != 0ull; }
__device__ __forceinline__ uint32_t kv_mctz(uint64_t m) { return (uint32_t)__builtin_ctzll(m); }
__device__ __forceinline__ uint64_t kv_mpop(uint64_t m) { return m & (m - 1ull); }
__device__ __forceinline__ KvM2 kv_mrange(KvM2 m, uint32_t plo, uint32_t phi, bool ok) {
  if (!ok) return {0ull, 0ull};
  const uint64_t lo_lo = plo < 64u ? ~0ull << plo : 0ull, lo_hi = phi < 64u ? ~0ull >> (63u - phi) : ~0ull;
  const uint64_t hi_lo = plo <= 64u ? ~0ull : ~0ull << (plo - 64u), hi_hi = phi >= 64u ? ~0ull >> (127u - phi) : 0ull;
  return {m.lo & lo_lo & lo_hi, m.hi & hi_lo & hi_hi};
}
__device__ __forceinline__ bool kv_mnz(KvM2 m) { return (m.lo | m.hi) != 0ull; }
__device__ __forceinline__ uint32_t kv_mctz(KvM2 m) {
  return m.lo ? (uint32_t)__builtin_ctzll(m.lo) : 64u + (uint32_t)__builtin_ctzll(m.hi);
}
__device__ __forceinline__ KvM2 kv_mpop(KvM2 m) {
  if (m.lo) return {m.lo & (m.lo - 1ull), m.hi};
  return {0ull, m.hi & (m.hi - 1ull)};
}

// segment (uniform words) == value bytes [k, k+len) ; value base 4-byte aligned
__device__ __forceinline__ bool seg_at(const GWord* __restrict__ wd, uint32_t len, const uint32_t* __restrict__ base,
                                       uint32_t k) {
  const uint32_t nw = (len + 3) >> 2;
  const uint32_t a = k >> 2, sh = k & 3;
  uint32_t lo = base[a];
  for (uint32_t i = 0; i < nw; i++) {
    uint32_t hi = base[a + i + 1];
    uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, sh);
    const GWord g = sld(wd + i);
    if ((v ^ g.w) & g.mask) return false;
    lo = hi;
  }
  return true;
}

// compiled glob over a 4-byte aligned value string (see kv_layout.h GlobFlags)
KV_FN bool glob_fast(const DevPS& P, const Atom& A, const uint8_t* s, uint32_t sl) {
  const uint32_t fl = sld(&A.gflags);
  if (fl & G_ALL) return true;
  if (fl & G_EMPTY) return sl == 0;
  if (sl < sld(&A.gmin)) return false;
  const uint32_t* base = (const uint32_t*)s;
  const GSeg* segs = P.gsegs + sld(&A.gfirst);
  const uint32_t n = sld(&A.gcount);
  uint32_t pos = 0, end = sl, i0 = 0, i1 = n;
  if (!(fl & G_LEAD)) {
    const GSeg s0 = sld(segs);
    if (n == 1 && !(fl & G_TRAIL)) return sl == s0.len && seg_at(P.gwords + s0.wfirst, s0.len, base, 0);
    if (!seg_at(P.gwords + s0.wfirst, s0.len, base, 0)) return false;
    pos = s0.len;
    i0 = 1;
  }
  if (!(fl & G_TRAIL)) {
    const GSeg st = sld(segs + n - 1);
    if (end < pos + st.len) return false;
    if (!seg_at(P.gwords + st.wfirst, st.len, base, end - st.len)) return false;
    end -= st.len;
    i1 = n - 1;
  }
  for (uint32_t i = i0; i < i1; i++) {
    const GSeg sg = sld(segs + i);
    bool found = false;
    for (uint32_t k = pos; k + sg.len <= end; k++) {
      if (seg_at(P.gwords + sg.wfirst, sg.len, base, k)) { pos = k + sg.len; found = true; break; }
    }
    if (!found) return false;
  }
  return true;
}

__device__ __forceinline__ bool glob_atom(const DevPS& P, const Atom& A, const uint8_t* s, uint32_t sl, bool ascii) {
  if (ascii || !(sld(&A.gflags) & G_HASQ)) return glob_fast(P, A, s, sl);
  return kv_glob(P.pstr + A.s_off, A.s_len & 0x7FFFFFFFu, s, sl);
}

__device__ __forceinline__ bool bytes_eq(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
  if (al != bl) return false;
  for (uint32_t k = 0; k < al; k++)
    if (a[k] != b[k]) return false;
  return true;
}

// magnitude/sign compare of canonical quantities: returns -1/0/1 (value vs pattern)
__device__ __forceinline__ int q_cmp(uint32_t vf, int32_t ve, uint64_t vh, uint64_t vl, uint32_t pf, int32_t pe,
                                     uint64_t ph, uint64_t pl) {
  int sv = (vf & VF_Q_ZERO) ? 0 : ((vf & VF_Q_NEG) ? -1 : 1);
  int sp = (pf & VF_Q_ZERO) ? 0 : ((pf & VF_Q_NEG) ? -1 : 1);
  if (sv != sp) return sv < sp ? -1 : 1;
  if (sv == 0) return 0;
  int m;
  if (ve != pe) m = ve < pe ? -1 : 1;
  else if (vh != ph) m = vh < ph ? -1 : 1;
  else if (vl != pl) m = vl < pl ? -1 : 1;
  else m = 0;
  return sv > 0 ? m : -m;
}

__device__ __forceinline__ bool cmp_ok(uint32_t op, int r) {
  switch (op) {
    case CO_EQ: return r == 0;
    case CO_NE: return r != 0;
    case CO_GT: return r == 1;
    case CO_LT: return r == -1;
    case CO_GE: return r >= 0;
    default: return r <= 0;
  }
}

// one atom of a string pattern against a scalar/absent node (type NT_NULL == Go nil)
KV_FN bool atom_eval(const DevPS& P, const DevBatch& B, uint32_t ai, uint32_t type, const Node& n) {
  const Atom& A = P.atoms[ai];
  const uint32_t kind = sld(&A.kind);
  if (kind == AT_FALSE) return false;
  if (type == NT_MAP || type == NT_ARR) return false;
  if (kind == AT_GLOB_E) {
    if (type == NT_NULL) return false;
    bool r = glob_atom(P, A, B.bstr + n.b, n.c & NC_LEN_MASK, n.c & NC_ASCII_E);
    return sld(&A.op) == CO_NE ? !r : r;
  }
  if (type == NT_BOOL) return false;
  if (kind == AT_GLOB_N) {
    if (type == NT_NULL) return glob_atom(P, A, B.bstr, 1, true);  // convertNumberToString(nil) == "0" (bstr[0..1))
    if (type != NT_FLOAT) return glob_atom(P, A, B.bstr + n.b, n.c & NC_LEN_MASK, n.c & NC_ASCII_E);  // == e-form
    const Val& v = B.vals[n.a];
    return glob_atom(P, A, B.bstr + v.n_off, v.n_len, v.flags & VF_ASCII_N);
  }
  // AT_QCMP
  int r;
  if (type == NT_NULL) {
    r = q_cmp(VF_Q_ZERO, 0, 0, 0, A.q_flags, A.q_exp, A.q_hi, A.q_lo);
  } else {
    const Val& v = B.vals[n.a];
    if (!(v.flags & VF_Q_VALID)) return false;
    r = q_cmp(v.flags, v.q_exp, v.q_hi, v.q_lo, A.q_flags, A.q_exp, A.q_hi, A.q_lo);
  }
  return cmp_ok(sld(&A.op), r);
}

// ValidateValueWithPattern(value, pattern) for a scalar-pattern leaf; n = the
// value node (ignored when type == NT_NULL, which also stands for absent)
KV_FN bool pred_eval(const DevPS& P, const DevBatch& B, uint32_t pi, uint32_t type, const Node& n) {
  const Pred& pr = P.preds[pi];
  const uint32_t kind = sld(&pr.kind);
  switch (kind) {
    case PK_BOOL: return type == NT_BOOL && ((n.c & NC_BOOLV) ? 1u : 0u) == sld(&pr.flags);
    case PK_FLOAT: {
      if (type == NT_INT) return sld(&pr.flags) && B.vals[n.a].i == pr.fi;
      if (type == NT_FLOAT) return B.vals[n.a].f == pr.f;
      if (type == NT_STR) {
        const Val& v = B.vals[n.a];
        return (v.flags & VF_PF_OK) && v.f == pr.f;
      }
      return false;
    }
    case PK_NIL:
      if (type == NT_NULL) return true;
      if (type == NT_MAP || type == NT_ARR) return false;
      return (n.c & NC_NILLIKE) != 0;
    case PK_MAPTYPE: return type == NT_MAP;
    case PK_STRING: {
      const uint32_t af = sld(&pr.first), an = sld(&pr.count);
      for (uint32_t a = af; a < af + an; a++) {
        const Alt& al = P.alts[a];
        const uint32_t cf = sld(&al.first), cn = sld(&al.count);
        bool all = true;
        for (uint32_t c = cf; c < cf + cn && all; c++) {
          const Conj& cj = P.conjs[c];
          const uint32_t ck = sld(&cj.kind);
          bool r = atom_eval(P, B, sld(&cj.a0), type, n);
          if (ck == CJ_INRANGE) r = r && atom_eval(P, B, sld(&cj.a1), type, n);
          else if (ck == CJ_NOTINRANGE) r = r || atom_eval(P, B, sld(&cj.a1), type, n);
          all = r;
        }
        if (all) return true;
      }
      return false;
    }
    default: return false;
  }
}

__device__ __forceinline__ bool pred_node(const DevPS& P, const DevBatch& B, const Node* __restrict__ N, uint32_t pi,
                                          uint32_t node) {
  Node n{NT_NULL, 0, 0, 0};
  if (node != ABSENT) n = N[node];
  return pred_eval(P, B, pi, node_type(n.kt), n);
}

// keep-all map (labels/annotations): scan for key id
__device__ __forceinline__ uint32_t lookup(const Node* __restrict__ N, uint32_t m, uint32_t key) {
  if (m == ABSENT) return ABSENT;
  const Node n = N[m];
  if (node_type(n.kt) != NT_MAP) return ABSENT;
  for (uint32_t i = 0; i < n.b; i++)
    if (node_key(N[ni(n.a + i)].kt) == key) return ni(n.a + i);
  return ABSENT;
}

// key-lookup op operand: slot of a slot-addressed map, or key id (AUX_SCAN)
__device__ __forceinline__ uint32_t lookup_op(const Node* __restrict__ N, uint32_t m, uint32_t a, uint32_t aux) {
  if (aux & AUX_SCAN) return lookup(N, m, a);
  if (m == ABSENT) return ABSENT;
  const Node n = N[m];
  if (node_type(n.kt) != NT_MAP || a >= n.b) return ABSENT;
  const uint32_t c = ni(n.a + a);
  return node_type(N[c].kt) == NT_ABSENT ? ABSENT : c;
}

// Resolved result key of sibling spec entry (OP_KEYGLOB): returns key id and node.
KV_FN void kg_resolve(const DevPS& P, const DevBatch& B, const Node* __restrict__ N, uint32_t m, uint32_t w,
                           uint32_t ref, uint32_t* key, uint32_t* node) {
  if (!w) {  // literal sibling: key id is the key
    *key = ref;
    *node = lookup(N, m, ref);
    return;
  }
  const Atom& A = P.atoms[ref];
  const Node mn = N[m];
  for (uint32_t i = 0; i < mn.b; i++) {
    const uint32_t k = node_key(N[ni(mn.a + i)].kt);
    if (glob_atom(P, A, B.kstr + B.key_off[k], B.key_len[k], false)) {
      *key = k;
      *node = ni(mn.a + i);
      return;
    }
  }
  *key = KV_SENT;  // unresolved wildcard: unique literal result key
  *node = ABSENT;
}


// OP_KEYGLOB (ExpandInMetadata wildcard label keys, wildcards.go:38-161 with the
// canonical choice of DESIGN.md): resolves the key of sibling j of a label map.
// Returns false if the key is dropped (a later sibling resolves to the same key)
// or absent with skip semantics (aux & 1): the caller jumps to the skip target.
__device__ __forceinline__ bool keyglob_op(const DevPS& P, const DevBatch& B, const Node* __restrict__ N, uint32_t m,
                                           uint32_t opw, uint32_t ia, uint32_t ic, uint32_t* out, uint32_t* keynode) {
  const uint32_t j = opw >> 24;
  const uint32_t aux = (opw >> 16) & 0xFF;
  const Atom& at = P.atoms[ia];
  const uint32_t spec = uni((uint32_t)at.q_hi);
  const uint32_t mycls = uni((uint32_t)at.q_lo);
  const uint32_t n = P.kg_specs[spec];
  uint32_t mykey, mynode;
  const uint32_t myw = P.kg_specs[spec + 1 + 2 * j] & 1;
  kg_resolve(P, B, N, m, myw, myw ? ia : ic, &mykey, &mynode);
  bool dropped = false;
  for (uint32_t j2 = j + 1; j2 < n && !dropped; j2++) {
    const uint32_t cw = P.kg_specs[spec + 1 + 2 * j2];
    if ((cw >> 1) != mycls || mykey == KV_SENT) continue;
    uint32_t k2, n2;
    kg_resolve(P, B, N, m, cw & 1, P.kg_specs[spec + 2 + 2 * j2], &k2, &n2);
    dropped = k2 == mykey;
  }
  if (dropped) return false;
  const uint32_t node = (myw && mykey != KV_SENT) ? mynode : lookup(N, m, ic);
  *keynode = (myw && mykey != KV_SENT) ? mynode : ABSENT;
  *out = node;
  return !(node == ABSENT && (aux & 1));
}

// ------------------------------------------------------------------ match/exclude
// LabelSelectorAsSelector(ReplaceInSelector(selector, labels)).Matches(labels)
// (pkg/engine/utils.go:99-107, pkg/engine/wildcards/wildcards.go:13-63) on one
// label list; `si` must be uniform across the wave (selector fields read with sld()).
KV_FN bool selector_match(const DevPS& P, const DevBatch& B, const KV* __restrict__ labels, uint32_t nl,
                               uint32_t si) {
  const Selector& S = P.sels[si];
  const uint32_t fl = sld(&S.flags);
  if (fl & SF_STATIC_INVALID) return false;
  if (fl & SF_EVERYTHING) return true;
  const uint32_t mf = sld(&S.ml_first), mc = sld(&S.ml_count);
  auto resolve = [&](const SelLabel& E, const uint8_t** ok, uint32_t* okl, const uint8_t** ov, uint32_t* ovl,
                     bool* val) {
    if (!(E.flags & SL_WILD)) {
      *ok = P.pstr + E.k_off; *okl = E.k_len; *ov = P.pstr + E.v_off; *ovl = E.v_len;
      *val = (E.flags & SL_VALID) != 0;
      return;
    }
    for (uint32_t q = 0; q < nl; q++) {
      const KV kv = labels[q];
      const uint8_t* lk = B.bstr + kv.k_off;
      const uint8_t* lv = B.bstr + kv.v_off;
      const uint32_t lkl = kv.k_len & KV_LEN_MASK, lvl = kv.v_len & KV_LEN_MASK;
      if (kv_glob(P.pstr + E.k_off, E.k_len, lk, lkl) && kv_glob(P.pstr + E.v_off, E.v_len, lv, lvl)) {
        *ok = lk; *okl = lkl; *ov = lv; *ovl = lvl;
        *val = (kv.k_len & KV_VALID) && (kv.v_len & KV_VALID);
        return;
      }
    }
    *ok = P.pstr + E.rk_off; *okl = E.rk_len; *ov = P.pstr + E.rv_off; *ovl = E.rv_len;
    *val = (E.flags & SL_VALID) != 0;
  };
  for (uint32_t j = mf; j < mf + mc; j++) {
    const uint8_t *kp, *vp;
    uint32_t kl, vl;
    bool valid;
    resolve(P.sellabels[j], &kp, &kl, &vp, &vl, &valid);
    // dropped if a later entry resolves to the same key (results[matchK] = matchV)
    bool dropped = false;
    for (uint32_t j2 = j + 1; j2 < mf + mc && !dropped; j2++) {
      const uint8_t *k2, *v2;
      uint32_t k2l, v2l;
      bool val2;
      resolve(P.sellabels[j2], &k2, &k2l, &v2, &v2l, &val2);
      dropped = bytes_eq(kp, kl, k2, k2l);
    }
    if (dropped) continue;
    if (!valid) return false;  // NewRequirement validation error
    bool found = false;
    for (uint32_t q = 0; q < nl; q++) {
      const KV kv = labels[q];
      if (bytes_eq(B.bstr + kv.k_off, kv.k_len & KV_LEN_MASK, kp, kl)) {
        found = bytes_eq(B.bstr + kv.v_off, kv.v_len & KV_LEN_MASK, vp, vl);
        break;
      }
    }
    if (!found) return false;
  }
  const uint32_t ef = sld(&S.me_first), ec = sld(&S.me_count);
  for (uint32_t j = ef; j < ef + ec; j++) {
    const SelExpr& E = P.selexprs[j];
    bool has = false, in = false;
    for (uint32_t q = 0; q < nl; q++) {
      const KV kv = labels[q];
      if (bytes_eq(B.bstr + kv.k_off, kv.k_len & KV_LEN_MASK, P.pstr + E.k_off, E.k_len)) {
        has = true;
        for (uint32_t v = E.v_first; v < E.v_first + E.v_count && !in; v++)
          in = bytes_eq(B.bstr + kv.v_off, kv.v_len & KV_LEN_MASK, P.pstr + P.strrefs[v].off, P.strrefs[v].len);
        break;
      }
    }
    const uint32_t op = sld(&E.op);
    if ((op == 0 && !in) || (op == 1 && in) || (op == 2 && !has) || (op == 3 && has)) return false;
  }
  return true;
}

// checkAnnotations (pkg/engine/utils.go:77-97): every pattern pair is matched
// (key and value globs) by some annotation of the list
KV_FN bool annotations_match(const DevPS& P, const DevBatch& B, const KV* __restrict__ ann, uint32_t na,
                                  uint32_t first, uint32_t count) {
  for (uint32_t k = first; k < first + count; k++) {
    const StrPair sp = P.strpairs[k];
    bool m = false;
    for (uint32_t q = 0; q < na && !m; q++) {
      const KV kv = ann[q];
      m = kv_glob(P.pstr + sp.k_off, sp.k_len, B.bstr + kv.k_off, kv.k_len & KV_LEN_MASK) &&
          kv_glob(P.pstr + sp.v_off, sp.v_len, B.bstr + kv.v_off, kv.v_len & KV_LEN_MASK);
    }
    if (!m) return false;
  }
  return true;
}

// checkNameSpace (pkg/engine/utils.go:62-75): some namespace glob matches
KV_FN bool namespaces_match(const DevPS& P, const uint8_t* __restrict__ s, uint32_t sl, uint32_t first,
                                 uint32_t count) {
  for (uint32_t k = first; k < first + count; k++)
    if (kv_glob(P.pstr + P.strrefs[k].off, P.strrefs[k].len, s, sl)) return true;
  return false;
}

// bit `bit` of a match table [word][n_entities] for entity e
__device__ __forceinline__ bool mt_bit(const uint32_t* __restrict__ t, uint32_t bit, uint32_t n_entities, uint32_t e) {
  return (t[(size_t)(bit >> 5) * n_entities + e] >> (bit & 31u)) & 1u;
}

// One word of the match tables (kv_mtab grid: y = table word, uniform per
// workgroup, so the 32 criteria of the word are uniform across the wave; x =
// entity). Rows y enumerate the namespace words, then the annotation words, then
// the selector words.
// Bit k of match-table row y for entity e (row y: namespace-glob words, then annotation
// words, then selector words; e: a distinct namespace string / annotation list / label
// list of the batch), and the entity count of row y's table.
KV_FN uint32_t mtab_entities(const DevPS& P, const DevBatch& B, uint32_t y) {
  if (y < P.mt_ns_words) return B.n_nsm;
  if (y < P.mt_ns_words + P.mt_ann_words) return B.n_asets;
  return B.n_lsets;
}
KV_FN bool mtab_bit(const DevPS& P, const DevBatch& B, uint32_t y, uint32_t e, uint32_t k) {
  if (y < P.mt_ns_words + P.mt_ann_words) {
    const uint32_t f = P.mt_bitf[y * 32u + k];  // the filter owning this bit
    if (f == KV_SENT) return false;
    const MFilter& F = P.filters[f];
    if (y < P.mt_ns_words) {
      const StrRef s = B.nsms[e];
      return namespaces_match(P, B.bstr + s.off, s.len, F.nss_first, F.nss_count);
    }
    const KVSet a = B.asets[e];
    return annotations_match(P, B, B.kvs + a.first, a.count, F.ann_first, F.ann_count);
  }
  y -= P.mt_ns_words + P.mt_ann_words;
  const uint32_t si = y * 32u + k;
  if (si >= P.n_sels) return false;
  const KVSet l = B.lsets[e];
  return selector_match(P, B, B.kvs + l.first, l.count, si);
}

// Word y of the match tables for entity e, one bit after the other (host emulator; the
// device kernel evaluates the 32 bits on 32 lanes, kv_mtab_kernel)
KV_FN void mtab_word(const DevPS& P, const DevBatch& B, uint32_t y, uint32_t e, uint32_t* __restrict__ ns,
                     uint32_t* __restrict__ an, uint32_t* __restrict__ sl) {
  if (e >= mtab_entities(P, B, y)) return;
  uint32_t w = 0;
  for (uint32_t k = 0; k < 32u; k++)
    if (mtab_bit(P, B, y, e, k)) w |= 1u << k;
  if (y < P.mt_ns_words) ns[(size_t)y * B.n_nsm + e] = w;
  else if (y < P.mt_ns_words + P.mt_ann_words) an[(size_t)(y - P.mt_ns_words) * B.n_asets + e] = w;
  else sl[(size_t)(y - P.mt_ns_words - P.mt_ann_words) * B.n_lsets + e] = w;
}

// doesResourceMatchConditionBlock: number of failed criteria (0 == block matches)
// (criteria restricted to the flag bits in `mask`). Namespace globs, annotations
// and label selectors are bits of the pass's match tables.
KV_FN uint32_t block_errs_masked(const DevPS& P, const DevBatch& B, const Res* __restrict__ R, uint32_t rkind,
                                      uint32_t rflags, uint32_t f, uint32_t mask) {
  const MFilter& F = P.filters[f];
  const uint32_t fl = sld(P.fflags + f) & mask;
  uint32_t errs = 0;
  if (fl & MF_KINDS) {
    bool ok = false;
    const uint32_t kf = sld(&F.kinds_first), kc = sld(&F.kinds_count);
    for (uint32_t k = kf; k < kf + kc && !ok; k++) {
      const KindSpec ks = sld(P.kinds + k);
      switch (ks.form) {
        case 3: ok = true; break;
        case 0: ok = rkind == ks.kind; break;
        case 1: ok = rkind == ks.kind && R->version == ks.version; break;
        default: ok = R->group == ks.group && rkind == ks.kind && (R->version == ks.version || R->version == P.star_id); break;
      }
    }
    errs += ok ? 0 : 1;
    if (errs) return errs;  // later criteria cannot turn an error count back to zero
  }
  if (fl & MF_NAME) errs += kv_glob(P.pstr + F.name_off, F.name_len, B.bstr + R->name_off, R->name_len) ? 0 : 1;
  if (fl & MF_NAMES) {
    bool any = false;
    for (uint32_t k = F.names_first; k < F.names_first + F.names_count && !any; k++)
      any = kv_glob(P.pstr + P.strrefs[k].off, P.strrefs[k].len, B.bstr + R->name_off, R->name_len);
    errs += any ? 0 : 1;
  }
  if (fl & MF_NSS) errs += mt_bit(P.mt_ns, sld(&F.nss_bit), B.n_nsm, R->nsm) ? 0 : 1;
  if (fl & MF_ANN) errs += mt_bit(P.mt_ann, sld(&F.ann_bit), B.n_asets, R->aset) ? 0 : 1;
  if (fl & MF_SEL) errs += mt_bit(P.mt_sel, sld(&F.sel), B.n_lsets, R->lset) ? 0 : 1;
  if ((fl & MF_NSSEL) && !(rflags & (RF_KIND_NAMESPACE | RF_KIND_EMPTY))) {
    const uint32_t bit = F.nssel_bit;
    errs += (B.ns_bits[R->ns_index * B.ns_words + bit / 32] >> (bit % 32)) & 1 ? 0 : 1;
  }
  if (fl & MF_UI_FAIL) errs += 1;
  return errs;
}

__device__ __forceinline__ uint32_t block_errs(const DevPS& P, const DevBatch& B, const Res* __restrict__ R,
                                               uint32_t rkind, uint32_t rflags, uint32_t f) {
  return block_errs_masked(P, B, R, rkind, rflags, f, 0xFFFFFFFFu);
}

KV_FN bool rule_matches(const DevPS& P, const DevBatch& B, const Res* __restrict__ R, uint32_t rkind,
                             uint32_t rflags, const RuleRec& rr) {
  const uint32_t mm = sld(&rr.m_mode), mf = sld(&rr.m_first), mc = sld(&rr.m_count);
  bool ok;
  if (mm == 1) {
    ok = false;
    for (uint32_t f = mf; f < mf + mc && !ok; f++) ok = !(sld(P.fflags + f) & MF_EMPTY) && block_errs(P, B, R, rkind, rflags, f) == 0;
  } else if (mm == 2) {
    ok = true;
    for (uint32_t f = mf; f < mf + mc && ok; f++) ok = !(sld(P.fflags + f) & MF_EMPTY) && block_errs(P, B, R, rkind, rflags, f) == 0;
  } else {
    ok = !(sld(P.fflags + mf) & MF_EMPTY) && block_errs(P, B, R, rkind, rflags, mf) == 0;
  }
  if (!ok) return false;
  const uint32_t xm = sld(&rr.x_mode), xf = sld(&rr.x_first), xc = sld(&rr.x_count);
  if (xm == 1) {
    for (uint32_t f = xf; f < xf + xc; f++)
      if (!(sld(P.fflags + f) & MF_EMPTY) && block_errs(P, B, R, rkind, rflags, f) == 0) return false;
    return true;
  }
  if (xm == 2) {
    for (uint32_t f = xf; f < xf + xc; f++)
      if ((sld(P.fflags + f) & MF_EMPTY) || block_errs(P, B, R, rkind, rflags, f) != 0) return true;
    return false;
  }
  if (!(sld(P.fflags + xf) & MF_EMPTY) && block_errs(P, B, R, rkind, rflags, xf) == 0) return false;
  return true;
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    uint32_t x = __shfl_xor(v, o, 64);
    v = x < v ? x : v;
  }
  return v;
}


// ------------------------------------------------------------------ results
// Error state of one (resource, rule) evaluation (becomes an ErrRec)
struct EState {
  uint32_t kind, flags, pn, key, res, i0, i1, i2, i3;
};

// error record of a FAIL / ERROR / SKIP pair (kvdevtypes.h ErrRec8): the 8 B
// compact form, flagged `wide` when the indices / key do not fit. Passes with
// KV_OFULL(O) bit 2 (re-run by the host only when some record was wide) write the
// full 32 B form instead; the flag is uniform, so this is a scalar branch.
// compact record words (kvdevtypes.h ErrRec8) of an error at loop indices i0..i3 on the
// resource of lane r % 64; `wide` when they do not fit
__device__ __forceinline__ uint2 err8_pack(uint32_t kind, uint32_t flags, uint32_t pn, uint32_t key, uint32_t i0,
                                           uint32_t i1, uint32_t i2, uint32_t i3, uint32_t r) {
  const uint32_t fits = (i0 < 1024u) & (i1 < 256u) & (i2 < 256u) & (i3 == 0u) & (key == ABSENT) & (pn < (1u << 25));
  uint2 w;
  w.x = kind | (flags << 4) | ((fits ^ 1u) << 6) | (pn << 7);
  w.y = (i0 & 1023u) | ((i1 & 255u) << 10) | ((i2 & 255u) << 18) | ((r & 63u) << 26);
  return w;
}

// Record of rule ri on resource r: the rule's row base is uniform and r the only per-lane
// part of the address (a scalar base + 32-bit vector offset store).
__device__ __forceinline__ void store_err(const DevOut& O, uint32_t ri, uint32_t n_res, uint32_t r, uint32_t kind,
                                          uint32_t flags, uint32_t pn, uint32_t key, uint32_t res, uint32_t i0,
                                          uint32_t i1, uint32_t i2, uint32_t i3) {
#if defined(KV_JIT_PRELUDE) && !defined(KVEMU)
  // specialized kernels write compact records only: the host re-runs a pass that needs full
  // records on the bytecode engine (kvapi.cpp DevSession::fetch), which keeps the code of
  // every record site of these kernels small
  if (KV_OFULL(O) & 4) return;
#else
  if (KV_OFULL(O) & 4) {
    uint4* x = (uint4*)(O.err + (size_t)ri * n_res) + 2u * r;
    x[0] = make_uint4(kind | (flags << 16), pn, key, res);
    x[1] = make_uint4(i0, i1, i2, i3);
    return;
  }
#endif
  ((uint2*)(O.err8 + (size_t)ri * n_res))[r] = err8_pack(kind, flags, pn, key, i0, i1, i2, i3, r);
}

// number of bytes of w equal to the byte replicated in b4 (exact SWAR zero-byte count)
__device__ __forceinline__ uint32_t kv_count_bytes(uint32_t w, uint32_t b4) {
  const uint32_t t = w ^ b4;
  return (uint32_t)__popc(~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu));
}

// ------------------------------------------------------------------ value-predicate table
// column of the table holding the predicates of leaf node n: its Val for a scalar, else the
// pseudo column of its type (null / map / array; an absent cursor reads as null)
__device__ __forceinline__ uint32_t kv_ptab_col(const DevPS& P, uint32_t type, uint32_t a) {
  if (type - 1u < 4u) return a;
  return P.n_vals - KV_PTAB_PSEUDO + (type == NT_NULL ? 0u : type == NT_MAP ? 1u : 2u);
}

// table word `w` of the leaf predicates on node n: for an array every element must pass
// (validateValueWithPattern per element), i.e. the AND of the elements' words (all ones
// for an empty array)
__device__ __forceinline__ uint32_t kv_leaf_word(const DevPS& P, const Node* __restrict__ N, const Node& n, uint32_t w) {
  const uint32_t t = node_type(n.kt);
#ifdef KV_DIAG_XPTAB
  if (t != NT_ARR) return (n.a * 0x9E3779B9u) ^ (w * 0x85EBCA6Bu);  // (diagnostics: no table read)
#endif
  if (t != NT_ARR) return kv_gld(P.ptab, (size_t)w * P.n_vals + kv_ptab_col(P, t, n.a));
  uint32_t x = 0xFFFFFFFFu;
  for (uint32_t k = 0; k < n.b; k++) {
    const Node e = N[ni(n.a + k)];
    x &= kv_gld(P.ptab, (size_t)w * P.n_vals + kv_ptab_col(P, node_type(e.kt), e.a));
  }
  return x;
}

// record `e` of rule ri on resource r at `slot` of its wave's segment of the rule's record row
// (slot < 64: a rule ends once per lane)
__device__ __forceinline__ void kv_rec_put(const DevOut& O, uint32_t ri, uint32_t n_res, uint32_t r, uint32_t slot,
                                           const EState& e, uint32_t z) {
#ifdef KV_DIAG_NORECST
  asm volatile("" ::"v"(slot));
  return;
#endif
  ((uint2*)(O.err8 + (size_t)ri * n_res))[(r & ~63u) + (slot & 63u)] =
      err8_pack(e.kind + z, e.flags, e.pn + z, e.key + z, e.i0, e.i1, e.i2, e.i3, r);
}

// final status of one rule on this lane: its byte in status row `row` of the workgroup (s_row;
// 0xFF: no resource; copied to the status matrix and counted when the kernel ends, kv_end_flush)
// and, for FAIL / ERROR / SKIP, the error record, appended to the wave's segment of the rule's
// record row through the wave's counter byte of the row (ErrRec8 layout)
__device__ __forceinline__ void kv_final(const DevOut& O, uint32_t ri, uint32_t n_res, uint32_t r, bool valid,
                                         uint32_t st, const EState& e, uint8_t* s_row, uint32_t row) {
#ifdef KV_DIAG_NOREC
  if (false) {
#else
  if (valid && (KV_OFULL(O) & 2) && (st == ST_FAIL || st == ST_ERROR || st == ST_SKIP)) {
#endif
    uint32_t z = 0u;  // an opaque zero: the site's constant record words are built here, not
                      // hoisted out of the loops as one constant register tuple per site
#ifndef KVEMU
    asm volatile("" : "+v"(r), "+v"(z));
    asm volatile("" : "+s"(ri));
#endif
#if defined(KV_JIT_PRELUDE) && !defined(KVEMU)
    if (!(KV_OFULL(O) & 4)) {  // (full records come from a bytecode-engine re-run)
      // the row's byte of the wave's counter word; the increment is wave-uniform, so the atomic
      // optimizer issues one LDS add of popcount(exec) << sh per wave
      uint8_t* s_c = s_row - KV_ROW0 - row * KV_RSTRIDE + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * KV_KROWS;
      const uint32_t sh = 8u * (row & 3u);
      kv_rec_put(O, ri, n_res, r, atomicAdd((uint32_t*)(s_c + (row & ~3u)), 1u << sh) >> sh, e, z);
    }
#else
    store_err(O, ri, n_res, r, e.kind + z, e.flags, e.pn + z, e.key + z, e.res + z, e.i0, e.i1, e.i2, e.i3);
#endif
  }
  s_row[threadIdx.x] = valid ? (uint8_t)st : (uint8_t)0xFFu;
}

// final status `st` of the members `m` of a rule group (kvjit.cpp: rules whose programs differ
// only in their leaf predicates and pattern-node ids, evaluated once with one bit per member):
// member j is rule tab[j] (or ri0 + j * sri), its pattern nodes are the group's shifted by
// tab[n + j] (or j * spn), its status row is row0 + j (s_row0 + j * KV_RSTRIDE); `ekx` is the
// error of the group's representative (kind | flags << 4 | node << 8; 0: none).
// Records (round 4 A/B, C3 / C2 ms per pass, gpurun_out/ab2): a counter round trip per member
// 9.38 / 0.71; one wave-level add per 8 members (ballot counts) 10.73 / 0.74 (the ballots
// doubled the code); a lane-level 64-bit add per 8 members, below, 9.15 / 0.70; `slot` (the
// generator's choice per group, JitImage::rec_compact): each record at its resource slot
// instead (no counter; partial lines: C3 writes 7.55 -> 9.74 GB) 8.22 ms. A one-member group
// (C4's and C5's rules) takes the wave-level add of a single rule: 64 lanes adding to one LDS
// word serialise.
// Round 5 A/B of two other finalizations (C2 / C5 ms per pass, gpurun_out/s17): this lane's members
// one after the other, and a uniform loop over the members some lane ends: neutral, removed.
// SITE (groups of 2+ members): one site record per lane for all the
// members `m` it ends here (kvdevtypes.h GSiteDesc), appended through the wave's counter s_gc[wave]
// to the wave's segment of the group's area (gpre: the group's first record / (64 x waves)); the
// members' records are expanded at fetch (kv_gsite_expand_kernel). C2's image-glob groups end 20
// of their 21 members at one leaf site on most lanes: one store there instead of 20.
template <bool TB = false, bool SITE = false>
__device__ __forceinline__ void kv_gfin(const DevOut& O, uint32_t n_res, uint32_t r, bool valid, uint32_t m, uint32_t st,
                                        uint32_t ekx, uint32_t i0, uint32_t i1, uint32_t i2, uint32_t i3,
                                        uint8_t* s_row0, uint32_t row0, const uint32_t* tab, uint32_t n, uint32_t ri0,
                                        uint32_t sri, uint32_t spn, bool slot, uint32_t* s_gc = nullptr,
                                        uint32_t gpre = 0u) {
#if defined(KV_JIT_PRELUDE) && !defined(KVEMU)
  if (n == 1u && !slot) {  // a one-member group ends like a single rule (one wave-level add)
    if (m & 1u) {
      const uint32_t ri = __builtin_amdgcn_readfirstlane(TB ? tab[0] : ri0);
      const uint32_t ek = ekx ? ekx + ((TB ? tab[1] : 0u) << 8) : 0u;
      const EState e{ek & 15u, (ek >> 4) & 15u, ek >> 8, ABSENT, ABSENT, i0, i1, i2, i3};
      kv_final(O, ri, n_res, r, valid, st, e, s_row0, row0);
    }
    return;
  }
  if constexpr (SITE) {
    const uint8_t st8 = valid ? (uint8_t)st : (uint8_t)0xFFu;
#ifdef KV_DIAG_NOREC
    if (false) {
#else
    if (m != 0u && valid && (KV_OFULL(O) & 2) && !(KV_OFULL(O) & 4) && (st == ST_FAIL || st == ST_ERROR || st == ST_SKIP)) {
#endif
      uint32_t z = 0u, rr = r;
      asm volatile("" : "+v"(rr), "+v"(z));
      const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
      const uint32_t fits = (i0 < 1024u) & (i1 < 256u) & (i2 < 256u) & (i3 == 0u);
      const uint32_t y = (i0 & 1023u) | ((i1 & 255u) << 10) | ((i2 & 255u) << 18) | ((rr & 63u) << 26);
      // (a wave-uniform LDS address: the atomic optimizer issues one add of the wave's lanes)
      const uint32_t k = atomicAdd(s_gc + w, 1u);
      const uint32_t nw = (n_res + 63u) >> 6;
      uint4* seg = (uint4*)O.gsite + ((size_t)gpre * nw + (size_t)(rr >> 6) * n) * 64u;
#if defined(KV_DIAG_NORECST)
      asm volatile("" ::"v"(k), "v"(y));
#else
      seg[k] = make_uint4(ekx + z, y, m, fits ^ 1u);
#endif
    }
    for (uint32_t j = 0; j < n; j++)
      if ((m >> j) & 1u) s_row0[j * KV_RSTRIDE + threadIdx.x] = st8;
    return;
  }
  {
#ifdef KV_DIAG_NOREC
  const bool rec = false;
#else
  const bool rec = valid && (KV_OFULL(O) & 2) && !(KV_OFULL(O) & 4) && (st == ST_FAIL || st == ST_ERROR || st == ST_SKIP);
#endif
  constexpr uint32_t NW = 5u;  // 64-bit counter words a group of < 32 rows touches
  const uint32_t w0 = row0 >> 3;
  unsigned long long old[NW] = {0ull, 0ull, 0ull, 0ull, 0ull};
  if (!slot && rec) {
    // this lane's members as counter bytes: one lane-level add per word returns the slots of
    // all its members of the word (slots in the order the lanes' adds land; the record carries
    // its lane). The address is named lane-varying so the atomic optimizer leaves the adds alone.
    unsigned long long inc[NW] = {0ull, 0ull, 0ull, 0ull, 0ull};
    for (uint32_t j = 0; j < n; j++)
      inc[((row0 + j) >> 3) - w0] |= (unsigned long long)((m >> j) & 1u) << (8u * ((row0 + j) & 7u));
    uint32_t oz = 0u;
    asm volatile("" : "+v"(oz));
    unsigned long long* s_c = (unsigned long long*)(s_row0 - KV_ROW0 - row0 * KV_RSTRIDE +
                                                    __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * KV_KROWS) + w0 + oz;
    for (uint32_t k = 0; k < NW; k++)
      if (inc[k]) old[k] = atomicAdd(s_c + k, inc[k]);
  }
  for (uint32_t j = 0; j < n; j++) {  // uniform over the members (scalar rule ids and rows)
    if (!((m >> j) & 1u)) continue;
    // (j is uniform, so is the member's rule id: named so, the compiler keeps it scalar)
    uint32_t ri = __builtin_amdgcn_readfirstlane(TB ? tab[j] : ri0 + j * sri);
    if (rec) {
      uint32_t z = 0u, rr = r;
      // (ri named opaque here: the member's record row address is formed at its store, not
      // hoisted to the kernel entry as one live scalar pair per member: C2 spilled 319 SGPRs)
      asm volatile("" : "+v"(rr), "+v"(z), "+s"(ri));
      const uint32_t ek = ekx ? ekx + ((TB ? tab[n + j] : j * spn) << 8) : 0u;
      const EState e{ek & 15u, (ek >> 4) & 15u, ek >> 8, ABSENT, ABSENT, i0, i1, i2, i3};
      if (slot) {
#if !defined(KV_DIAG_NORECST)
        ((uint2*)(O.err8 + (size_t)ri * n_res))[rr] = err8_pack(e.kind + z, e.flags, e.pn + z, e.key + z, e.i0, e.i1, e.i2, e.i3, rr);
#endif
      } else
        kv_rec_put(O, ri, n_res, rr, (uint32_t)(old[((row0 + j) >> 3) - w0] >> (8u * ((row0 + j) & 7u))) & 0xFFu, e, z);
    }
    s_row0[j * KV_RSTRIDE + threadIdx.x] = valid ? (uint8_t)st : (uint8_t)0xFFu;
  }
  }
#else
  for (uint32_t j = 0; j < n; j++) {
    if (!((m >> j) & 1u)) continue;
    const uint32_t ri = __builtin_amdgcn_readfirstlane(TB ? tab[j] : ri0 + j * sri);
    const uint32_t ek = ekx ? ekx + ((TB ? tab[n + j] : j * spn) << 8) : 0u;
    const EState e{ek & 15u, (ek >> 4) & 15u, ek >> 8, ABSENT, ABSENT, i0, i1, i2, i3};
    kv_final(O, ri, n_res, r, valid, st, e, s_row0 + j * KV_RSTRIDE, row0 + j);
  }
#endif
}

// ------------------------------------------------------------------ status rows
// The rule kernels stage one status byte per (rule, lane) in LDS rows of the workgroup
// (KV_RSTRIDE bytes per rule: KV_RWG status bytes; the record counter bytes per wave before them), prefilled
// with NOMATCH (kv_prefill_rows); matched lanes store their status (kv_final); a fused block
// that no lane of a wave matches costs that wave nothing. When the kernel ends each wave copies
// its statuses to the status matrix and counts its segment of every row (kv_end_flush).
// Ordering inside a wave: LDS operations of one wave execute in program order; the fence
// keeps the compiler from moving the lanes' row accesses across it.
__device__ __forceinline__ void kv_wsync() {
#ifndef KVEMU
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
}

// record counters zeroed and rows [0, nr) set to NOMATCH for the lanes holding a resource (0xFF
// past the batch); s_stw = the kernel's LDS (KV_ROW0 counter bytes, then the rows), base = the
// workgroup's first resource
__device__ __forceinline__ void kv_prefill_rows(uint32_t* s_stw, uint32_t nr, uint32_t base, uint32_t n_res) {
  const uint32_t nv = n_res > base ? n_res - base : 0u;
#ifdef KVEMU
  // host emulation runs the lanes one after another: each lane fills its own bytes
  for (uint32_t q = 0; q < nr; q++)
    ((uint8_t*)s_stw)[KV_ROW0 + q * KV_RSTRIDE + threadIdx.x] = threadIdx.x < nv ? (uint8_t)ST_NOMATCH : (uint8_t)0xFFu;
#else
  for (uint32_t t = threadIdx.x; t < KV_ROW0 / 4u; t += (uint32_t)KV_RWG) s_stw[t] = 0u;
  // thread t writes status word t % WPR of rows t / WPR, t / WPR + KV_RWG / WPR, ... (one pattern
  // per thread; WPR words per row)
  constexpr uint32_t WPR = KV_RSTRIDE / 4u;
  uint32_t* rows = s_stw + KV_ROW0 / 4u;
  const uint32_t k = threadIdx.x % WPR, l = k * 4u;
  uint32_t x = 0u;
  for (uint32_t j = 0u; j < 4u; j++) x |= (l + j < nv ? (uint32_t)ST_NOMATCH : 0xFFu) << (8u * j);
  for (uint32_t q = threadIdx.x / WPR; q < nr; q += (uint32_t)KV_RWG / WPR) rows[q * WPR + k] = x;
  __syncthreads();
#endif
}

// histogram of one 64-lane status segment (16 words) restricted to the lanes of mask m (other
// bytes read as 0xFE, no status), into c[KV_HIST]
__device__ __forceinline__ void kv_count_seg(const uint32_t* w, uint64_t m, uint32_t* c) {
  uint32_t c0 = 0u, c1 = 0u, c5 = 0u, cx = 0u, n = 0u;
#pragma unroll 4
  for (uint32_t i = 0; i < 16u; i++) {
    const uint32_t b = (uint32_t)(m >> (4u * i)) & 15u;
    const uint32_t keep = (((b * 0x00204081u) & 0x01010101u) * 0xFFu);  // byte k = 0xFF if bit k
    const uint32_t x = (w[i] & keep) | (0xFEFEFEFEu & ~keep);
    c0 += kv_count_bytes(x, 0x00000000u);
    c1 += kv_count_bytes(x, 0x01010101u);
    c5 += kv_count_bytes(x, 0x05050505u);
    cx += kv_count_bytes(x, 0xFFFFFFFFu);
    n += (uint32_t)__popc(b);
  }
  for (uint32_t k = 0; k < (uint32_t)KV_HIST; k++) c[k] = 0u;
  c[ST_PASS] = c0;
  c[ST_FAIL] = c1;
  c[ST_NOMATCH] = c5;
  if (c0 + c1 + c5 + cx < n) {
    const uint32_t rest[4] = {ST_WARN, ST_ERROR, ST_SKIP, ST_CPU};
    for (uint32_t k = 0; k < 4u; k++) {
      uint32_t q = 0u;
      for (uint32_t i = 0; i < 16u; i++) {
        const uint32_t b = (uint32_t)(m >> (4u * i)) & 15u;
        const uint32_t keep = (((b * 0x00204081u) & 0x01010101u) * 0xFFu);
        q += kv_count_bytes((w[i] & keep) | (0xFEFEFEFEu & ~keep), rest[k] * 0x01010101u);
      }
      c[rest[k]] = q;
    }
  }
}

// End of the rule kernel for this wave: its statuses of the nr rules (kernel rules
// rules[0..nr)) go to the status matrix (KV_OFULL(O) & 1); lane q counts the wave's segment of row q
// (every lane, and with per-scope counts, KV_OFULL(O) & 8, the lanes of the workgroup's scope wsc;
// lanes of other scopes go straight to O.scounts) and leaves the 16 counts in that segment
// (counts[KV_HIST], scope counts[KV_HIST]); after a workgroup barrier one thread per (rule,
// count) sums the four waves' segments into O.counts / O.scounts with a global atomic. The
// store is ordered by kind and namespace, so a workgroup mostly holds one scope. `sc` is this
// lane's scope.
__device__ __forceinline__ void kv_end_flush(const DevOut& O, uint32_t* s_stw, uint32_t nr, const uint32_t* rules,
                                             uint32_t n_res, uint32_t r, bool valid, uint32_t sc, uint32_t wsc,
                                             uint32_t n_rules) {
  const uint8_t* s_b = (const uint8_t*)s_stw + KV_ROW0;
  __syncthreads();  // (the waves read each other's rows)
#ifndef KVEMU
  const uint32_t wg0 = r - threadIdx.x;
#ifdef KV_DIAG_NOCOPY
  if (false) {
#else
  if ((KV_OFULL(O) & 1u) && wg0 + (uint32_t)KV_RWG <= n_res && (n_res & 15u) == 0u) {
#endif
    // 16 B per lane, LPR lanes per row (a row = the workgroup's KV_RWG statuses of a rule): each
    // wave store writes 64 / LPR rows of the workgroup (C3 9.10 -> 8.96 ms per pass against a
    // byte per lane and row, round 4); a partial workgroup, or rows not 16 B aligned: a byte per
    // lane. A row segment of the workgroup that is NOMATCH throughout (72 % of C3's statuses) is
    // not written: its flag says so (O.sflag) and the fetch fills it
    constexpr uint32_t LPR = KV_RSTRIDE / 16u;
    const uint32_t l = threadIdx.x & 63u, c16 = (threadIdx.x % LPR) * 16u;
    const size_t nwg = (n_res + (uint32_t)KV_RWG - 1u) / (uint32_t)KV_RWG;
    for (uint32_t q = threadIdx.x / LPR; q < nr; q += (uint32_t)KV_RWG / LPR) {
      const uint4 v = *(const uint4*)(s_b + q * KV_RSTRIDE + c16);
      if (O.sflag) {
        constexpr uint32_t NM4 = 0x01010101u * (uint32_t)ST_NOMATCH;
        const bool nm = v.x == NM4 && v.y == NM4 && v.z == NM4 && v.w == NM4;
        // the row's LPR lanes
        const bool any = ((__ballot(!nm) >> (l & (64u - LPR))) & ((1ull << LPR) - 1ull)) != 0ull;
        if ((l % LPR) == 0u) O.sflag[(size_t)rules[q] * nwg + wg0 / (uint32_t)KV_RWG] = any ? 1u : 0u;
        if (!any) continue;
      }
      *(uint4*)(O.status + (size_t)rules[q] * n_res + wg0 + c16) = v;
    }
    // (a wave copies the other waves' segments, which they overwrite with counts below; the
    // condition is uniform over the workgroup)
    __syncthreads();
  } else
#endif
  if ((KV_OFULL(O) & 1u) && valid) {
#pragma unroll 4
    for (uint32_t q = 0; q < nr; q++) O.status[(size_t)rules[q] * n_res + r] = s_b[q * KV_RSTRIDE + threadIdx.x];
    if (O.sflag && (r & ((uint32_t)KV_RWG - 1u)) == 0u)  // (the workgroup's first lane: rows written)
      for (uint32_t q = 0; q < nr; q++) O.sflag[(size_t)rules[q] * ((n_res + (uint32_t)KV_RWG - 1u) / (uint32_t)KV_RWG) + r / (uint32_t)KV_RWG] = 1u;
  }
#ifdef KV_DIAG_NOCOUNT
  return;
#endif
#ifndef KVEMU
  const uint32_t l = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t vm = __ballot(valid);
  uint64_t mw = 0ull;  // the wave's lanes of the workgroup's scope
  if (KV_OFULL(O) & 8u) {
    uint64_t rem = vm;
    while (rem) {  // one pass per distinct scope among the wave's resources
      const uint32_t s = __builtin_amdgcn_readlane(sc, (uint32_t)__builtin_ctzll(rem));
      const uint64_t m = __ballot(valid && sc == s) & rem;
      rem &= ~m;
      if (s == wsc) {
        mw = m;
        continue;
      }
      for (uint32_t q = l; q < nr; q += 64u) {
        uint32_t c[KV_HIST];
        kv_count_seg((const uint32_t*)(s_b + q * KV_RSTRIDE + w * 64u), m, c);
        for (uint32_t k = 0; k < (uint32_t)KV_HIST; k++)
          if (c[k] && k != 7u) atomicAdd(&O.scounts[((size_t)s * n_rules + rules[q]) * KV_HIST + k], (unsigned long long)c[k]);
      }
    }
  }
  kv_wsync();
  for (uint32_t q = l; q < nr; q += 64u) {
    uint32_t* seg = (uint32_t*)(s_b + q * KV_RSTRIDE + w * 64u);
    uint32_t c[KV_HIST], cs[KV_HIST];
    kv_count_seg(seg, ~0ull, c);
    if (mw == vm) for (uint32_t k = 0; k < (uint32_t)KV_HIST; k++) cs[k] = c[k];  // (one scope: the common case)
    else if (mw) kv_count_seg(seg, mw, cs);
    else for (uint32_t k = 0; k < (uint32_t)KV_HIST; k++) cs[k] = 0u;
    for (uint32_t k = 0; k < (uint32_t)KV_HIST; k++) {
      seg[k] = k == 7u ? 0u : c[k];
      seg[KV_HIST + k] = k == 7u ? 0u : cs[k];
    }
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < nr * 2u * KV_HIST; t += (uint32_t)KV_RWG) {
    const uint32_t q = t / (2u * KV_HIST), k = t % (2u * KV_HIST);
    uint32_t v = 0u;
    for (uint32_t x = 0; x < KV_RWAVES; x++) v += ((const uint32_t*)(s_b + q * KV_RSTRIDE + x * 64u))[k];
#ifdef KV_DIAG_NOATOM
    asm volatile("" ::"v"(v));
    continue;
#endif
    if (!v) continue;
    if (k < (uint32_t)KV_HIST) {
      // (with per-scope counts the per-rule totals are their sum, kv_scope_totals_kernel)
      if (!(KV_OFULL(O) & 8u)) atomicAdd(&O.counts[(size_t)rules[q] * KV_HIST + k], (unsigned long long)v);
    } else if ((KV_OFULL(O) & 8u) && wsc != 0xFFFFFFFFu)
      atomicAdd(&O.scounts[((size_t)wsc * n_rules + rules[q]) * KV_HIST + (k - KV_HIST)], (unsigned long long)v);
  }
#else
  (void)sc; (void)wsc; (void)n_rules;  // (counts are not emulated)
#endif
}

// status + error record (FAIL/ERROR/SKIP) + per-rule histogram with the
// common statuses counted by one ballot each (fused specialized kernels)
__device__ __forceinline__ void store_result2(const DevOut& O, uint32_t ri, uint32_t n_res, uint32_t r, bool valid,
                                              uint32_t st, const EState& e, uint32_t* hist) {
  if (valid && (KV_OFULL(O) & 1)) {
    const size_t o = (size_t)ri * n_res + r;
    O.status[o] = (uint8_t)st;
    if ((KV_OFULL(O) & 2) && (st == ST_FAIL || st == ST_ERROR || st == ST_SKIP))
      store_err(O, ri, n_res, r, e.kind, e.flags, e.pn, e.key, e.res, e.i0, e.i1, e.i2, e.i3);
  }
  const uint64_t m_pass = __ballot(valid && st == ST_PASS), m_fail = __ballot(valid && st == ST_FAIL);
  const uint64_t m_nm = __ballot(valid && st == ST_NOMATCH);
  const uint64_t m_rest = __ballot(valid && st != ST_PASS && st != ST_FAIL && st != ST_NOMATCH);
  if ((threadIdx.x & 63) == 0) {
    if (m_pass) atomicAdd(&hist[ST_PASS], (uint32_t)__popcll(m_pass));
    if (m_fail) atomicAdd(&hist[ST_FAIL], (uint32_t)__popcll(m_fail));
    if (m_nm) atomicAdd(&hist[ST_NOMATCH], (uint32_t)__popcll(m_nm));
  }
  if (m_rest) {
    for (uint32_t s = ST_WARN; s <= ST_CPU; s++) {
      if (s == ST_NOMATCH) continue;
      const uint64_t bm = __ballot(valid && st == s);
      if (bm && (threadIdx.x & 63) == 0) atomicAdd(&hist[s], (uint32_t)__popcll(bm));
    }
  }
}

// status[rule][res] (+ error record for FAIL/ERROR/SKIP) and the per-rule
// status histogram (one LDS atomic per wave and status)
__device__ __forceinline__ void store_result(const DevOut& O, uint32_t ri, uint32_t n_res, uint32_t r, bool valid,
                                             uint32_t st, const EState& e, uint32_t* hist) {
  if (valid && (KV_OFULL(O) & 1)) {
    const size_t o = (size_t)ri * n_res + r;
    O.status[o] = (uint8_t)st;
    if ((KV_OFULL(O) & 2) && (st == ST_FAIL || st == ST_ERROR || st == ST_SKIP))
      store_err(O, ri, n_res, r, e.kind, e.flags, e.pn, e.key, e.res, e.i0, e.i1, e.i2, e.i3);
  }
  for (uint32_t s = 0; s < 7; s++) {
    const uint64_t bm = __ballot(valid && st == s);
    if (bm && (threadIdx.x & 63) == 0) atomicAdd(&hist[s], (uint32_t)__popcll(bm));
  }
}
