// kvemu: host build of the pass's match-table builder (kvdevfn.h mtab_word, the
// body of kv_mtab_kernel), with the same prelude the specialized kernels see.
#include "shim.h"
#include "../../build/kvgpu/kvjit_prelude.h"

extern "C" void kvemu_mtab(const DevPS* P, const DevBatch* B, uint32_t words, uint32_t max_entities, uint32_t* ns,
                           uint32_t* an, uint32_t* sl) {
  for (uint32_t y = 0; y < words; y++)
    for (uint32_t e = 0; e < max_entities; e++) mtab_word(*P, *B, y, e, ns, an, sl);
}
