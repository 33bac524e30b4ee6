// Factored match (kv_mfac_kernel / kv_mtup_kernel in kvkernel.hip; the host emulator
// tools/kvemu/mtab.cpp): device functions over the helpers of kvdevfn.h, kept out of the
// specialized kernels' hiprtc prelude (the generated rule kernels only read the match words).
// Include after kvdevfn.h.
#pragma once

// ------------------------------------------------------------------ factored match
// doesResourceMatchConditionBlock (pkg/engine/utils.go:265-336) of one filter is a conjunction
// of per-attribute criteria; fac_crit is the factor of entity type t (DevPS::fac_*): the
// filter's criteria on that attribute, every other criterion taken as true. The kind factor
// carries the launch-folded flags (MF_EMPTY, user info); the namespaceSelector factor is
// exempt for kind Namespace / empty kinds (utils.go:323), applied per tuple (mtup_word).
KV_FN uint32_t fac_entities(const DevBatch& B, uint32_t t) {
  switch (t) {
    case KV_FAC_KIND: return B.n_kent;
    case KV_FAC_NSM: return B.n_nsm;
    case KV_FAC_ANN: return B.n_asets;
    case KV_FAC_SEL: return B.n_lsets;
    default: return B.n_ns;
  }
}
KV_FN bool fac_crit(const DevPS& P, const DevBatch& B, uint32_t t, uint32_t e, uint32_t f) {
  const uint32_t fl = P.fflags[f];
  const MFilter& F = P.filters[f];
  switch (t) {
    case KV_FAC_KIND: {
      if (fl & (MF_EMPTY | MF_UI_FAIL)) return false;
      if (!(fl & MF_KINDS)) return true;
      const Res* __restrict__ R = B.res + B.kent_rep[e];
      const uint32_t rkind = R->kind, kf = F.kinds_first, kc = F.kinds_count;
      for (uint32_t k = kf; k < kf + kc; k++) {  // checkKind (utils.go:47-60), as block_errs_masked
        const KindSpec ks = P.kinds[k];
        bool ok;
        switch (ks.form) {
          case 3: ok = true; break;
          case 0: ok = rkind == ks.kind; break;
          case 1: ok = rkind == ks.kind && R->version == ks.version; break;
          default: ok = R->group == ks.group && rkind == ks.kind && (R->version == ks.version || R->version == P.star_id); break;
        }
        if (ok) return true;
      }
      return false;
    }
    case KV_FAC_NSM: return !(fl & MF_NSS) || mt_bit(P.mt_ns, F.nss_bit, B.n_nsm, e);
    case KV_FAC_ANN: return !(fl & MF_ANN) || mt_bit(P.mt_ann, F.ann_bit, B.n_asets, e);
    case KV_FAC_SEL: return !(fl & MF_SEL) || mt_bit(P.mt_sel, F.sel, B.n_lsets, e);
    default: {
      if (!(fl & MF_NSSEL)) return true;
      const uint32_t bit = F.nssel_bit;
      return (B.ns_bits[(size_t)e * B.ns_words + bit / 32u] >> (bit % 32u)) & 1u;
    }
  }
}
// Bit b of the word of slot s for entity e of type t: every filter of the plane at bit b passes
// the type-t factor (an absent plane is 0). Table layout [slot][entity] per type; the kernel
// evaluates the 32 bits of a word on 32 lanes (kv_mfac_kernel), the host emulator in turn.
KV_FN bool fac_bit_of(const DevPS& P, const DevBatch& B, uint32_t t, uint32_t e, uint32_t s, uint32_t b) {
  const uint32_t first = P.fac_bit[2u * (s * 32u + b)], cnt = P.fac_bit[2u * (s * 32u + b) + 1u];
  if (!(cnt & KV_FAC_PRESENT)) return false;
  bool ok = true;
  for (uint32_t k = first; k < first + (cnt & ~KV_FAC_PRESENT) && ok; k++) ok = fac_crit(P, B, t, e, P.fac_flist[k]);
  return ok;
}
KV_FN uint32_t fac_cell(const DevPS& P, const DevBatch& B, uint32_t t, uint32_t e, uint32_t s) {
  uint32_t w = 0;
  for (uint32_t b = 0; b < 32u; b++) w |= (fac_bit_of(P, B, t, e, s, b) ? 1u : 0u) << b;
  return w;
}
KV_FN const uint32_t* fac_table(const DevPS& P, uint32_t t) { return P.fac_tab + P.fac_off[t]; }
// Match word w of tuple t: OR over the match planes of the AND of the five factors, minus the
// OR of the exclude planes; rules with name filters keep bit 1 (their rule kernel evaluates
// the match per resource), rules with more planes than KV_FAC_MAXP run rule_matches here.
// a tuple's entities (read once per tuple, for all the words a thread computes)
struct MtupIn {
  const Res* R;
  uint32_t eK, eN, eA, eL, eS, rflags, kex;
};
KV_FN MtupIn mtup_in(const DevBatch& B, uint32_t t) {
  const Res* __restrict__ R = B.res + B.tup_rep[t];
  MtupIn in{R, B.tup_kent[t], R->nsm, R->aset, R->lset, R->ns_index, R->flags, 0u};
  in.kex = (in.rflags & (RF_KIND_NAMESPACE | RF_KIND_EMPTY)) ? 0xFFFFFFFFu : 0u;
  return in;
}
KV_FN uint32_t mtup_word_in(const DevPS& P, const DevBatch& B, const MtupIn& in, uint32_t w) {
  const uint32_t s0 = sld(P.fac_word + 4u * w), np = sld(P.fac_word + 4u * w + 1u);
  const uint32_t named = sld(P.fac_word + 4u * w + 2u), cx = sld(P.fac_word + 4u * w + 3u);
  const uint32_t nm = np & 0xFFu, nx = (np >> 8) & 0xFFu;
  const uint32_t nK = B.n_kent, nN = B.n_nsm, nA = B.n_asets, nL = B.n_lsets, nS = B.n_ns;
  const uint32_t* __restrict__ tK = fac_table(P, KV_FAC_KIND);
  const uint32_t* __restrict__ tN = fac_table(P, KV_FAC_NSM);
  const uint32_t* __restrict__ tA = fac_table(P, KV_FAC_ANN);
  const uint32_t* __restrict__ tL = fac_table(P, KV_FAC_SEL);
  const uint32_t* __restrict__ tS = fac_table(P, KV_FAC_NS);
  uint32_t m = 0u, x = 0u;
  for (uint32_t p = 0; p < nm + nx; p++) {
    const size_t s = s0 + p;
    const uint32_t v =
        tK[s * nK + in.eK] & tN[s * nN + in.eN] & tA[s * nA + in.eA] & tL[s * nL + in.eL] & (tS[s * nS + in.eS] | in.kex);
    if (p < nm) m |= v;
    else x |= v;
  }
  m = (m & ~x) | named;
  for (uint32_t c = cx; c; c &= c - 1u) {
    const uint32_t b = (uint32_t)__builtin_ctz(c);
    if (rule_matches(P, B, in.R, in.R->kind, in.rflags, P.rules[sld(P.fac_rule + 32u * w + b)])) m |= 1u << b;
  }
  return m;
}
KV_FN uint32_t mtup_word(const DevPS& P, const DevBatch& B, uint32_t t, uint32_t w) {
  return mtup_word_in(P, B, mtup_in(B, t), w);
}

