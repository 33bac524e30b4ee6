// Transfer form of the store's node cells (host ingest -> HBM, kv_expand_rows_kernel). Kept out
// of kv_layout.h, whose text is the specialized kernels' hiprtc prelude (their rule kernels read
// only the expanded Nodes).
#pragma once
#include "kv_layout.h"

namespace kv {

// Transfer form of a node cell (Batch::tcells, host -> HBM; kv_expand_rows_kernel rebuilds the
// 16-byte Node): 8 bytes, lo = kt, hi =
//   BOOL / INT / FLOAT / STR: the Val id (b = Val::e_off and c = e_len | NC_* follow from the Val)
//   MAP / ARR: first-child row - the cell's own row, | child count << 24 (when both fit), or
//              KV_TC_DETACHED for a = b = 0 (a map the projection does not descend into)
//   NULL / ABSENT: 0 (a = b = c = 0)
// Any other cell crosses as its 16-byte Node, flagged in its row's wide mask (Batch::rwide).
// The container form is relative to the cell's row, so rebasing rows (batch merge, shards)
// leaves it unchanged.
constexpr uint32_t KV_TC_DETACHED = 0xFFFFFFFFu;
KV_HD inline bool node_scalar_t(uint32_t t) { return t == NT_BOOL || t == NT_INT || t == NT_FLOAT || t == NT_STR; }
KV_HD inline uint32_t val_c(const Val& v) {
  return v.e_len | ((v.flags & VF_ASCII_E) ? NC_ASCII_E : 0u) | ((v.flags & VF_BOOLV) ? NC_BOOLV : 0u) |
         ((v.flags & VF_NILLIKE) ? NC_NILLIKE : 0u);
}
// the hi word of the 8-byte form of `n` (in row `row`), or false when it needs 16 bytes
KV_HD inline bool cell_narrow(const Node& n, uint64_t row, const Val* vals, uint32_t* hi) {
  const uint32_t t = node_type(n.kt);
  if (node_scalar_t(t)) {
    const Val& v = vals[n.a];
    if (n.b != v.e_off || n.c != val_c(v)) return false;
    *hi = n.a;
    return true;
  }
  if (t == NT_MAP || t == NT_ARR) {
    if (n.c) return false;
    if (n.a == 0 && n.b == 0) {
      *hi = KV_TC_DETACHED;
      return true;
    }
    if (n.a < row || n.a - row >= 0xFFFFFFu || n.b >= 256u) return false;
    *hi = (uint32_t)(n.a - row) | n.b << 24;
    return true;
  }
  if (n.a | n.b | n.c) return false;
  *hi = 0;
  return true;
}
KV_HD inline Node cell_widen(uint32_t kt, uint32_t hi, uint64_t row, const Val* vals) {
  const uint32_t t = node_type(kt);
  if (node_scalar_t(t)) {
    const Val& v = vals[hi];
    return Node{kt, hi, v.e_off, val_c(v)};
  }
  if (t == NT_MAP || t == NT_ARR) {
    if (hi == KV_TC_DETACHED) return Node{kt, 0u, 0u, 0u};
    return Node{kt, (uint32_t)row + (hi & 0xFFFFFFu), hi >> 24, 0u};
  }
  return Node{kt, 0u, 0u, 0u};
}

}  // namespace kv
