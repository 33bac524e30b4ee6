// kvemu: host build of the pass's match-table builder (kvdevfn.h mtab_word, the
// body of kv_mtab_kernel) and of the factored match (fac_cell / mtup_word, the bodies of
// kv_mfac_kernel / kv_mtup_kernel), with the same prelude the specialized kernels see.
#include "shim.h"
#include "../../build/kvgpu/kvjit_prelude.h"
#include "../../kyverno_amd/csrc/kvfac.h"

extern "C" void kvemu_mtab(const DevPS* P, const DevBatch* B, uint32_t words, uint32_t max_entities, uint32_t* ns,
                           uint32_t* an, uint32_t* sl) {
  for (uint32_t y = 0; y < words; y++)
    for (uint32_t e = 0; e < max_entities; e++) mtab_word(*P, *B, y, e, ns, an, sl);
}

extern "C" void kvemu_mfac(const DevPS* P, const DevBatch* B, uint32_t* mtup) {
  for (uint32_t t = 0; t < KV_FAC_TYPES; t++)
    for (uint32_t s = 0; s < P->fac_slots; s++)
      for (uint32_t e = 0, ne = fac_entities(*B, t); e < ne; e++)
        P->fac_tab[P->fac_off[t] + (size_t)s * ne + e] = fac_cell(*P, *B, t, e, s);
  for (uint32_t w = 0; w < P->fac_words; w++)
    for (uint32_t t = 0; t < B->n_tup; t++) mtup[(size_t)w * B->n_tup + t] = mtup_word(*P, *B, t, w);
}
