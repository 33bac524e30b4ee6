// Device-side views of a compiled policy set and an ingested batch, shared by
// the HIP kernels (kvkernel.hip, generated kernels of kvjit.cpp) and the host
// runtime (kvapi.cpp). Plain structs, no includes (embedded in the hiprtc prelude).
#pragma once

namespace kv {

struct ErrRec {
  uint32_t kind_flags;  // kind | flags << 16
  uint32_t pnode;
  uint32_t keynode;
  uint32_t resnode;
  uint32_t idx[4];
};

// Compact error record (8 B per FAIL / ERROR / SKIP pair, the one written per pass):
//   w0 = kind | flags << 4 | wide << 6 | pnode << 7          (pnode < 2^25)
//   w1 = idx0 | idx1 << 10 | idx2 << 18 | lane << 26  (idx0 < 1024, idx1 / idx2 < 256, idx3 == 0;
//        lane = the resource's lane in its wave)
// A record that does not fit (larger loop indices, a fourth loop level, a resolved
// wildcard key) sets `wide`; the host then re-runs the pass with full records
// (DevOut::full bit 2) into the 32 B ErrRec array.
// Layout in err8[rule][res]: the bytecode engine writes a record at its pair's slot; the
// specialized kernels append the records of a wave to the front of the wave's 64-slot segment
// (err8[rule][wave first resource + k], k in order of writing), so a wave writes whole lines
// instead of 8 B into 32 B sectors; the fetch restores resource order from the lane field
// (kv_rec_scatter_kernel).
struct ErrRec8 {
  uint32_t w0, w1;
};
constexpr uint32_t ERR8_WIDE = 1u << 6;
constexpr uint32_t ERR8_IDX_MASK = (1u << 26) - 1u;  // w1 without the lane

struct DevPS {
  const Inst* prog;
  const Pred* preds;
  const Alt* alts;
  const Conj* conjs;
  const Atom* atoms;
  const RuleRec* rules;
  const MFilter* filters;
  const uint32_t* fflags;  // per-filter flags folded with the launch's admission info
  const KindSpec* kinds;
  const StrRef* strrefs;
  const StrPair* strpairs;
  const Selector* sels;
  const SelLabel* sellabels;
  const SelExpr* selexprs;
  const uint32_t* kg_specs;
  const GSeg* gsegs;
  const GWord* gwords;
  const uint8_t* pstr;
  uint32_t star_id;
  uint32_t n_rules;
  uint32_t n_filters, n_sels;
  // value-predicate table of the specialized kernels (per launch configuration):
  // ptab[word * n_vals + val] bit b = leaf predicate of memo slot 32*word+b on
  // the scalar Val `val`, and on the three pseudo values after the batch's values: a
  // null, a map and an array node (n_vals = values + KV_PTAB_PSEUDO; built each pass by
  // kvj_ptab before the rule kernels)
  const uint32_t* ptab;
  uint32_t n_vals;
  // match tables (per launch configuration, built each pass by kv_mtab before the rule
  // kernels): bit b of word w at [w * n_entities + e] = filter criterion b on entity e
  //   mt_ns  [nss_bit]  namespace globs   x distinct checkNameSpace strings (DevBatch::nsms)
  //   mt_ann [ann_bit]  annotation globs  x distinct annotation lists       (DevBatch::asets)
  //   mt_sel [sel]      label selectors   x distinct label lists            (DevBatch::lsets)
  uint32_t mt_ns_words, mt_ann_words, mt_sel_words;
  const uint32_t* mt_ns;
  const uint32_t* mt_ann;
  const uint32_t* mt_sel;
  // match bits of the specialized kernels per match tuple (Res::tup): mtup[w * n_tup + tup]
  // bit b = rule at bit position 32*w+b (kernel order, kvjit.cpp) matches the tuple's
  // resources (1 for rules with name filters: evaluated per resource); built each pass by
  // kv_mfac + kv_mtup after kv_mtab (factored match, below)
  const uint32_t* mtup;
  uint32_t mtup_words;
  // filter of each namespace-glob bit (mt_ns_words * 32 entries), then of each annotation bit
  // (mt_ann_words * 32); KV_SENT for unused bits (mtab_bit_filters, kvfold.cpp)
  const uint32_t* mt_bitf;
  // Factored match (kv_mfac + kv_mtup, kvkernel.hip). MatchesResourceDescription of one
  // filter is a conjunction of per-attribute criteria (pkg/engine/utils.go:265-336), so a
  // rule's match is an OR of "planes" (one per `any` filter; `all` filters AND into one
  // plane), each the AND of five per-entity words: kind entity, checkNameSpace string,
  // annotation list, label list, namespace (namespaceSelector). A *slot* is one plane of one
  // 32-rule word (bit b = rule at bit position 32*w+b); per slot and bit, fac_bit holds the
  // plane's filter list (first, count | KV_FAC_PRESENT) in fac_flist.
  //   fac_word[4w..4w+3] = first slot of word w, match planes | exclude planes << 8,
  //                        bits evaluated per resource (name filters), bits evaluated per
  //                        tuple by rule_matches (rules with more planes than KV_FAC_MAXP)
  //   fac_rule[32w+b]    = rule at bit position 32w+b (KV_SENT: padding)
  // Tables (built each pass by kv_mfac after kv_mtab): fac_tab + fac_off[t], [slot][entity]
  // for entity type t (KV_FAC_KIND .. KV_FAC_NS).
  const uint32_t* fac_word;
  const uint32_t* fac_bit;
  const uint32_t* fac_flist;
  const uint32_t* fac_rule;
  uint32_t fac_slots, fac_words;
  uint32_t* fac_tab;
  uint64_t fac_off[5];
};
constexpr uint32_t KV_FAC_PRESENT = 0x80000000u;
constexpr uint32_t KV_FAC_MAXP = 8;  // match (and exclude) planes per word factored; beyond: rule_matches
enum FacType : uint32_t { KV_FAC_KIND = 0, KV_FAC_NSM = 1, KV_FAC_ANN = 2, KV_FAC_SEL = 3, KV_FAC_NS = 4, KV_FAC_TYPES = 5 };

struct DevBatch {
  const Node* nodes;
  const Val* vals;
  const Res* res;
  const KV* kvs;
  const uint8_t* bstr;
  const uint32_t* ns_bits;
  const uint32_t* key_off;
  const uint32_t* key_len;
  const uint8_t* kstr;
  const StrRef* nsms;   // distinct checkNameSpace strings (bstr offsets)
  const KVSet* lsets;   // distinct label lists
  const KVSet* asets;   // distinct annotation lists
  uint32_t n_nsm, n_lsets, n_asets;
  uint32_t ns_words;
  uint32_t n_res;
  const uint32_t* tup_rep;  // a resource of each match tuple (its Res is the tuple's inputs)
  uint32_t n_tup;
  // kind entities: distinct (kind, group, version, kind flags) of the batch's tuples
  const uint32_t* tup_kent;  // kind entity of each tuple
  const uint32_t* kent_rep;  // a resource of each kind entity
  uint32_t n_kent, n_ns;     // kind entities, namespaces (rows of ns_bits)
  // pattern variables (kvvars.cpp build_dyn): predicate table of the batch's distinct
  // substituted leaves, outcome (= predicate) id per [dynamic leaf][res], and the status
  // substitution decides per [dynamic rule][res] (0: evaluate, ST_ERROR, ST_CPU)
  const DevPS* dps;
  const uint32_t* dleaf;
  const uint8_t* dyn_st;
  // path columns of the specialized kernels (kvcol.h; null without them), in two planes: the
  // (kt, a, c) words of every cell, then its b words (pcolb = pcol + 3 x cells), so a lookup
  // of a map or a scalar (everything but an array's element count) loads 12 of its 16 bytes
  const uint32_t* pcol;
  const uint32_t* pcolb;
};

// ------------------------------------------------------------------ path columns
// The specialized kernels read every lookup whose path from the resource root (or from the
// element of a fused array loop) is static from a column of the batch's nodes at that path,
// one coalesced 16 B load, instead of chasing the path through the node rows (kvjit.cpp
// hoist). Columns come in families: family 0 has one column per root path, laid out
// [wave group][column][lane]; family f > 0 belongs to one array path (its "family array", a
// column of family 0) and holds one column per path relative to that array's elements, laid
// out [element row][column][lane] with the element rows of each wave group together
// (element i of a lane's array: row E + i, E = the family array cell's `c`). Cell of a present
// node: {type | KV_COL_PRESENT, a, b, c'} with c' = the node's own index for a map, the cell
// offset of its element rows for a family array, the node's c otherwise; absent: all zero.
// Built once per batch and device (kvcol.h, kv_pcol_* in kvkernel.hip).
constexpr uint32_t KV_COL_MAXD = 12;            // steps of a column path
constexpr uint32_t KV_COL_SCAN = 0x80000000u;   // step: key id of a keep-all map (else a slot)
constexpr uint32_t KV_COL_PRESENT = 16u;        // kt of a present cell: type | KV_COL_PRESENT
struct ColDesc {
  uint32_t fam;      // 0: a root path, f > 0: a path relative to the elements of family f
  uint32_t j;        // column within its family
  uint32_t nsteps;   // path length
  uint32_t arr_fam;  // family columns 0: the family whose array this column holds (0: none)
  uint32_t steps[KV_COL_MAXD];
};
// per family: its array's column in family 0 (family 0: unused), its columns; set per batch:
// the first cell of its element rows in the pool, and (device pointer) the exclusive prefix of
// element rows per wave group (n_groups + 1 entries: the last one is the family's row count)
struct ColFam {
  uint32_t arr_col, ncols;
  uint32_t off_lo, off_hi;
  uint32_t* erow;
};

struct DevOut {
  uint8_t* status;             // [rule][res]
  ErrRec8* err8;               // [rule][res] (written for fail/error/skip)
  ErrRec* err;                 // [rule][res] (only records flagged ERR8_WIDE)
  unsigned long long* counts;  // [rule][8]
  uint32_t full;               // bit0 status, bit1 error records, bit2 full 32 B records (not 8 B),
                               // bit3 per-scope counts (specialized kernels: counted in the pass)
  unsigned long long* scounts; // [scope][rule][8] (bit3)
  const uint32_t* scope;       // scope of every resource (bit3)
  // site records of the specialized rule groups (bit1, below; null without such groups)
  uint32_t* gsite;             // 16 B records, [group area][wave][64 x members]
  uint32_t* gcnt;              // [group][wave] records written
  // specialized kernels (bit0): 1 = the workgroup's 256 statuses of the rule were written, 0 = all
  // NOMATCH and not written (kv_end_flush; the fetch fills them, kv_status_fill_kernel)
  uint8_t* sflag;              // [rule][workgroup]
};

// Site records (specialized kernels, rule groups of 2+ members; kvdevfn.h kv_gfin): the members a
// lane ends at one error site share the site's record but for their pattern nodes (the group's
// representative's node + the member's shift), so the kernel writes one 16 B record per (lane,
// site) - {kind | flags << 4 | pn << 8 of the representative (0: none), ErrRec8::w1, member mask,
// indices do not fit} - appended to the wave's segment of the group's area (64 x members slots per
// wave: a member ends once per lane), and the count per (group, wave) when the wave ends. At fetch
// kv_gsite_expand_kernel writes each member's ErrRec8 to its [rule][res] slot. Group g's area
// starts at record gpre * 64 * waves (gpre = members of the groups before it); its members are
// gs_mem[2 * (moff + j)] (rule) and [2 * (moff + j) + 1] (pattern-node shift).
struct GSiteDesc {
  uint32_t n, gpre, moff, pad;
};

constexpr int KV_WG = 256;
// Workgroup of the specialized rule kernels: one wave. A workgroup's LDS (its status rows) is
// released when its last wave ends, so with four waves per workgroup a wave that finished its
// blocks early held its slot until the slowest wave of the four reached the end-of-kernel flush
// (C2: 14 % of wave lifetime at that barrier, KVGPU_JIT_STAMPS); one-wave workgroups hand their
// LDS and registers to the next workgroup as soon as they end.
constexpr int KV_RWG = 256;
constexpr uint32_t KV_RWAVES = (uint32_t)KV_RWG / 64u;
// LDS of a specialized rule kernel: the waves' record counters (a byte per (wave, row), wave
// stride KV_KROWS), then one status row per rule of the kernel (KV_RSTRIDE bytes: a byte per lane)
constexpr uint32_t KV_RSTRIDE = KV_RWG;
constexpr uint32_t KV_KROWS = 128u;                  // most rules (rows) per specialized kernel
constexpr uint32_t KV_ROW0 = KV_RWAVES * KV_KROWS;   // byte offset of row 0
constexpr uint32_t KV_PTAB_PSEUDO = 3;  // ptab columns of a null, a map and an array node
constexpr int KV_HIST = 8;

}  // namespace kv
