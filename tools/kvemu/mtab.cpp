// kvemu: host build of the pass's match-table builder (kvdevfn.h mtab_word, the
// body of kv_mtab_kernel) and of the factored match (fac_cell / mtup_word, the bodies of
// kv_mfac_kernel / kv_mtup_kernel), with the same prelude the specialized kernels see.
#include "shim.h"
#include "../../build/kvgpu/kvjit_prelude.h"
#include "../../kyverno_amd/csrc/kvfac.h"
#include "../../kyverno_amd/csrc/kvcol.h"

#include <algorithm>
#include <stdexcept>
#include <vector>

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

// path columns (as build_pcol in kvapi.cpp, the kv_pcol_* kernels lane by lane): family 0,
// the element rows of every wave group and family (max over the group's lanes, exclusive
// prefix), the families' offsets, then the element columns; returns the pool
std::vector<uint32_t> kvemu_pcol(const DevBatch* B, const std::vector<ColDesc>& cols, const std::vector<uint32_t>& fam_arr,
                             const std::vector<uint32_t>& fam_ncols, std::vector<uint32_t>* erow) {
  const uint32_t nf = (uint32_t)fam_ncols.size(), j0 = fam_ncols.at(0);
  const uint32_t groups = (uint32_t)((B->n_res + KV_WG - 1) / KV_WG * (KV_WG / KV_LANES));
  erow->assign((size_t)std::max<uint32_t>(1u, nf - 1) * (groups + 1), 0u);
  std::vector<ColFam> fams(nf);
  for (uint32_t f = 0; f < nf; f++) {
    fams[f].arr_col = fam_arr[f];
    fams[f].ncols = fam_ncols[f];
    fams[f].erow = f ? erow->data() + (size_t)(f - 1) * (groups + 1) : nullptr;
  }
  for (uint32_t f = 1; f < nf; f++) {
    uint32_t* e = fams[f].erow;
    for (uint32_t r = 0; r < groups * KV_LANES; r++) {
      threadIdx.x = r % KV_WG;
      e[r / KV_LANES] = std::max(e[r / KV_LANES], col_rows(*B, cols.data(), fams.data(), f, r));
    }
    uint32_t run = 0;
    for (uint32_t g = 0; g <= groups; g++) {
      const uint32_t c = g < groups ? e[g] : 0u;
      e[g] = run;
      run += c;
    }
  }
  uint64_t cells = (uint64_t)groups * j0 * KV_LANES;
  for (uint32_t f = 1; f < nf; f++) {
    fams[f].off_lo = (uint32_t)cells;
    fams[f].off_hi = (uint32_t)(cells >> 32);
    cells += (uint64_t)fams[f].erow[groups] * fams[f].ncols * KV_LANES;
  }
  if (cells >= (1ull << 32)) throw std::runtime_error("kvemu: more than 2^32 column cells");
  // two planes: (kt, a, c) 12 B per cell, then b 4 B per cell
  const uint64_t nc = std::max<uint64_t>(cells, 1);
  std::vector<uint32_t> pool(4 * nc, 0u);
  for (uint32_t c = 0; c < cols.size(); c++)
    for (uint32_t r = 0; r < groups * KV_LANES; r++) {
      threadIdx.x = r % KV_WG;
      if (c < j0) col_build_root(*B, cols.data(), fams.data(), j0, c, r, pool.data(), nc);
      else col_build_elem(*B, cols.data(), fams.data(), j0, c, r, pool.data(), nc);
    }
  return pool;
}
