// Device-side views of a compiled policy set and an ingested batch, shared by
// the HIP kernels (kvkernel.hip) and the host runtime (kvapi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kvcell.h"
#include "kv_layout.h"
#include "kvdevtypes.h"

namespace kv {

// Launch one pass over rules [rule_begin, rule_end) for every resource.
// P and B point to device-resident copies of the views (uniform scalar loads).
hipError_t launch_validate(const DevPS* P, const DevBatch* B, uint32_t n_res, const DevOut& O, uint32_t rule_begin,
                           uint32_t rule_end, hipStream_t stream);

// Match tables of a pass (DevPS::mt_*): `words` = mt_ns_words + mt_ann_words +
// mt_sel_words rows, max_entities = max(n_nsm, n_asets, n_lsets).
hipError_t launch_mtab(const DevPS* P, const DevBatch* B, uint32_t words, uint32_t max_entities, uint32_t* ns,
                       uint32_t* an, uint32_t* sl, hipStream_t stream);

// Factored match of a pass (after launch_mtab): the per-entity factor tables of every slot
// (DevPS::fac_tab; max_entities = the largest entity count of the five types), then the match
// words of every tuple into mtup[word][tuple].
hipError_t launch_mfac(const DevPS* P, const DevBatch* B, uint32_t slots, uint32_t max_entities, uint32_t words,
                       uint32_t n_tup, uint32_t* mtup, hipStream_t stream);

// out[rule][j] = in[rule][inv[j]] (caller-order status matrix)
hipError_t launch_gather_rows(const uint8_t* in, const uint32_t* inv, uint64_t n_rules, uint64_t n_res, uint8_t* out,
                              hipStream_t stream);

// a[i] = map[a[i]] for i < n
hipError_t launch_remap_u32(uint32_t* a, uint64_t n, const uint32_t* map, hipStream_t stream);

// Error-record compaction in rule-major, resource order. phase 0: offs[rule][tile]
// (exclusive, tiles of KV_WG resources), totals[rule], base[rule] (base[n_rules] =
// all records) over `status`, and with `masks` every wave's record lanes
// (masks[rule][res / 64]); phase 1: scatter the records (compact: appended per wave segment by
// the specialized kernels, else at their pair's slot; with errw/outw also the full ones) of the
// store-order `status` to out8[base[rule] + offs[rule][tile] + rank]; *wide |= 1 if a compact
// record is flagged ERR8_WIDE. With `order` (store index -> caller index) phase 0 ran over the
// caller-order statuses and phase 1 puts each record at its caller index's place.
// NOMATCH into the status segments the specialized kernels did not write (DevOut::sflag)
// the status transfer form: out == nullptr counts the written segments per (rule, chunk of KV_WG
// segments) into ccnt[rule][chunk]; otherwise packs them (4 bits a status) at cbase[rule][chunk] * KV_RWG / 2
hipError_t launch_status_pack(const uint8_t* status, const uint8_t* sflag, uint32_t n_res, uint32_t n_rules,
                              const unsigned long long* cbase, uint32_t* ccnt, uint8_t* out, hipStream_t stream);

// site records of the specialized rule groups -> the members' records at their slots (kvdevtypes.h
// GSiteDesc; fetch time, before launch_rec_compact's scatter)
hipError_t launch_gsite_expand(const uint32_t* gsite, const uint32_t* gcnt, const GSiteDesc* desc, const uint32_t* mem,
                               uint32_t n_groups, uint32_t n_res, ErrRec8* err8, hipStream_t stream);
hipError_t launch_rec_compact(const uint8_t* status, const ErrRec8* err8, const ErrRec* errw, uint32_t n_res,
                              uint32_t n_rules, uint32_t* offs, unsigned long long* totals, unsigned long long* base,
                              ErrRec8* out8, ErrRec* outw, uint32_t* wide, int phase, const uint8_t* compact,
                              const uint32_t* order, unsigned long long* masks, const uint8_t* sflag, hipStream_t stream);

// Record codes of a compacted record array (rule-major, rule r at [base[r], base[r + 1])): phase 0
// writes each record's slot in its rule's table of KV_REC_CODES distinct records (tkey, keys w0 << 32
// | w1 without the lane, preset ~0) as a 1-byte code, and flags raw[rule] (preset 0) when the table
// fills up; phase 1 copies the raw rules' records to out[nbase[rule] ...)
constexpr uint32_t KV_REC_CODES = 256;
hipError_t launch_rec_codes(const ErrRec8* rec, const unsigned long long* base, uint32_t n_rules,
                            unsigned long long* tkey, uint8_t* code, uint32_t* raw, const unsigned long long* nbase,
                            ErrRec8* out, int phase, hipStream_t stream);

constexpr uint32_t KV_SCOPE_CHUNK = 65536;  // resources per workgroup of the scope-count kernel
constexpr uint32_t KV_SCOPE_LDS = 2048;     // scopes held in LDS (2048 x 8 x 4 B = 64 KB)

// counts[scope][rule][KV_HIST] += histogram of status[rule][res] by scope[res]
hipError_t launch_scope_totals(const unsigned long long* scounts, uint32_t n_scopes, uint32_t n_rules,
                               unsigned long long* counts, hipStream_t stream);
hipError_t launch_scope_counts(const uint8_t* status, const uint32_t* scope, uint32_t n_res, uint32_t n_rules,
                               uint32_t n_scopes, unsigned long long* out, hipStream_t stream);

// nodes[row][lane] = the packed cell of (row, lane) when bit `lane` of rmask[row] is set
// (rank among the row's set bits, from roff[row]), else the zero cell (row padding)
hipError_t launch_expand_rows(const uint64_t* tcells, const uint64_t* rmask, const uint64_t* rwide, const uint32_t* roff,
                              const Val* vals, uint64_t n_rows, Node* nodes, hipStream_t stream);

// Path columns of a batch (kvcol.h, kvdevtypes.h ColDesc / ColFam; n_groups: 64-lane wave
// groups, a multiple of 4). rows: for every family f > 0 the element rows of each wave group
// (the most any of its lanes needs) into fams[f].erow, then their exclusive prefix (the
// family's total at erow[n_groups]). build: the cells of columns [c0, c0 + n) of every lane
// into the pool (family-0 columns first; element columns read their family arrays' cells).
hipError_t launch_pcol_rows(const DevBatch* B, const ColDesc* cols, const ColFam* fams, uint32_t n_fam,
                            uint32_t n_groups, hipStream_t stream);
hipError_t launch_pcol_build(const DevBatch* B, const ColDesc* cols, const ColFam* fams, uint32_t j0, uint32_t c0,
                             uint32_t n, uint32_t n_groups, bool elem, uint32_t* pool, uint64_t cells, hipStream_t stream);

}  // namespace kv
