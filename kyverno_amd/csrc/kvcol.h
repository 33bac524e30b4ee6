// Path columns (kvdevtypes.h ColDesc / ColFam): built once per batch and device from the node
// rows, read by the specialized kernels in place of their row walks (kvjit.cpp hoist). Device
// functions over the kvdevfn.h helpers: the kv_pcol_* kernels (kvkernel.hip) and the host
// emulator (tools/kvemu/mtab.cpp) run these bodies. Include after kvdevfn.h.
//
// A column cell is what the specialized kernels' row walk leaves in its hoisted node
// (kvjit.cpp hoist): the node at the path, or all zero when a step finds no node (a missing
// key, a non-map parent, a slot past the map's slots); the present cells carry
// KV_COL_PRESENT in kt (their key is dropped: the walk never reads a hoisted node's key) and
// in c the node's own index when it is a map (the cursor of a wildcard-key lookup) or the
// cell offset of its element rows when it holds a family's array.
#pragma once

// the node one step below n (held in cell *idx, ABSENT: none)
KV_FN Node col_step(const Node* __restrict__ N, const Node& n, uint32_t step, uint32_t* idx) {
  const Node z{0u, 0u, 0u, 0u};
  if (*idx == ABSENT || node_type(n.kt) != NT_MAP) {
    *idx = ABSENT;
    return z;
  }
  if (step & KV_COL_SCAN) {  // keep-all map (labels / annotations): the child with that key
    const uint32_t key = step & ~KV_COL_SCAN;
    for (uint32_t q = 0; q < n.b; q++) {
      const uint32_t c = ni(n.a + q);
      const Node t = N[c];
      if (node_key(t.kt) == key) {
        *idx = c;
        return t;
      }
    }
    *idx = ABSENT;
    return z;
  }
  if (step >= n.b) {  // slot-addressed map: slot `step`, NT_ABSENT when the resource lacks it
    *idx = ABSENT;
    return z;
  }
  const uint32_t c = ni(n.a + step);
  const Node t = N[c];
  if (node_type(t.kt) == NT_ABSENT) {
    *idx = ABSENT;
    return z;
  }
  *idx = c;
  return t;
}

// the node at column path d below cell idx (ABSENT: none), its cell in *out
KV_FN Node col_walk(const Node* __restrict__ N, uint32_t idx, const ColDesc& d, uint32_t* out) {
  Node n{0u, 0u, 0u, 0u};
  if (idx != ABSENT) n = N[idx];
  for (uint32_t s = 0; s < d.nsteps && s < KV_COL_MAXD; s++) n = col_step(N, n, d.steps[s], &idx);
  *out = idx;
  return n;
}

KV_FN Node col_cell(const Node& n, uint32_t idx, uint32_t arr_c) {
  if (idx == ABSENT) return Node{0u, 0u, 0u, 0u};
  const uint32_t t = node_type(n.kt);
  return Node{t | KV_COL_PRESENT, n.a, n.b, t == NT_MAP ? idx : t == NT_ARR ? arr_c : n.c};
}

KV_FN uint64_t col_fam_off(const ColFam& F) { return (uint64_t)F.off_lo | (uint64_t)F.off_hi << 32; }

// cell i of a pool of `cells` cells in two planes (DevBatch::pcol): (kt, a, c) at word 3i, b at
// word 3 cells + i
KV_FN void col_put(uint32_t* __restrict__ pool, uint64_t cells, uint64_t i, const Node& n) {
  pool[3 * i] = n.kt;
  pool[3 * i + 1] = n.a;
  pool[3 * i + 2] = n.c;
  pool[3 * cells + i] = n.b;
}
KV_FN Node col_get(const uint32_t* __restrict__ pool, uint64_t cells, uint64_t i) {
  return Node{pool[3 * i], pool[3 * i + 1], pool[3 * cells + i], pool[3 * i + 2]};
}

// element rows lane r needs in family f (its array's element count; 0 without an array)
KV_FN uint32_t col_rows(const DevBatch& B, const ColDesc* cols, const ColFam* fams, uint32_t f, uint32_t r) {
  if (r >= B.n_res) return 0u;
  uint32_t idx;
  const Node n = col_walk(B.nodes, ni(B.res[r].root), cols[fams[f].arr_col], &idx);
  return idx != ABSENT && node_type(n.kt) == NT_ARR ? n.b : 0u;
}

// cell of family-0 column `c` for lane r (r >= n_res: the zero cell), written into the pool
KV_FN void col_build_root(const DevBatch& B, const ColDesc* cols, const ColFam* fams, uint32_t j0, uint32_t c,
                          uint32_t r, uint32_t* __restrict__ pool, uint64_t cells) {
  const ColDesc& d = cols[c];
  Node cell{0u, 0u, 0u, 0u};
  if (r < B.n_res) {
    uint32_t idx;
    const Node n = col_walk(B.nodes, ni(B.res[r].root), d, &idx);
    uint32_t arr_c = 0u;
    if (d.arr_fam) {  // a family array: the offset of this wave group's element rows
      const ColFam& F = fams[d.arr_fam];
      arr_c = (uint32_t)(col_fam_off(F) + (uint64_t)F.erow[r >> 6] * F.ncols * KV_LANES);
    }
    cell = col_cell(n, idx, arr_c);
  }
  col_put(pool, cells, ((size_t)(r >> 6) * j0 + d.j) * KV_LANES + (r & (KV_LANES - 1)), cell);
}

// cells of element column `c` (family f > 0) for every element of lane r's family array
KV_FN void col_build_elem(const DevBatch& B, const ColDesc* cols, const ColFam* fams, uint32_t j0, uint32_t c,
                          uint32_t r, uint32_t* __restrict__ pool, uint64_t cells) {
  const ColDesc& d = cols[c];
  const ColFam& F = fams[d.fam];
  const uint32_t lane = r & (KV_LANES - 1);
  const Node a = col_get(pool, cells, ((size_t)(r >> 6) * j0 + F.arr_col) * KV_LANES + lane);
  if (node_type(a.kt) != NT_ARR || a.kt == 0u) return;
  for (uint32_t i = 0; i < a.b; i++) {
    uint32_t idx;
    const Node n = col_walk(B.nodes, ni(a.a + i), d, &idx);
    col_put(pool, cells, (size_t)a.c + ((size_t)i * F.ncols + d.j) * KV_LANES + lane, col_cell(n, idx, 0u));
  }
}
