// HBM layout shared by the host compiler/ingest (C++) and the HIP kernels.
// Everything here is plain-old-data; offsets are element indices into the
// per-batch / per-policyset arrays described in DESIGN.md §Data layout.
#pragma once
#include <stdint.h>

#if defined(__HIP__)
#define KV_HD __host__ __device__
#else
#define KV_HD
#endif

namespace kv {

// ---------------------------------------------------------------- resources
// Node types (Go dynamic types of unstructured values). NT_ABSENT marks an
// empty slot of a slot-addressed map (the resource lacks that pattern key).
enum NodeType : uint32_t {
  NT_NULL = 0, NT_BOOL = 1, NT_INT = 2, NT_FLOAT = 3, NT_STR = 4, NT_MAP = 5, NT_ARR = 6, NT_ABSENT = 7
};

constexpr uint32_t ABSENT = 0xFFFFFFFFu;  // "key not present" (Go: nil interface, ok=false)

// One JSON value of a projected resource tree (16 B).
//   kt = key id << 4 | type (key id: this node's key in its parent map, KEY_NONE28 for array elements/roots)
// Nodes live in rows of KV_LANES cells (wave-group layout): node index =
// row * KV_LANES + lane, where lane = resource index % KV_LANES.
//   MAP/ARR: a = ROW of the first child (the child block is shared by the group), b = child count
//   scalars: a = Val id, b = e_off, c = e_len | NC_ASCII_E | NC_BOOLV | NC_NILLIKE (validateString form inline,
//            so string globs need no Val load)
// Map children are either slot-addressed (the map's projection-trie node has a
// fixed, byte-sorted key list: child i is slot i, NT_ABSENT when missing) or,
// for keep-all maps (metadata labels/annotations), every key sorted by bytes.
// Array children are contiguous in index order.
struct Node {
  uint32_t kt;
  uint32_t a;
  uint32_t b;
  uint32_t c;
};
constexpr uint32_t KEY_NONE28 = 0x0FFFFFFFu;
constexpr uint32_t KV_LANES = 64;  // resources per node-row group (one wavefront)
constexpr uint32_t NC_ASCII_E = 1u << 31;
constexpr uint32_t NC_BOOLV = 1u << 30;
constexpr uint32_t NC_NILLIKE = 1u << 29;  // validateValueWithNilPattern true (0, 0.0, "", false)
constexpr uint32_t NC_LEN_MASK = 0x1FFFFFFFu;
KV_HD inline uint32_t node_type(uint32_t kt) { return kt & 15u; }
// Position classes of stored values (value-predicate table pruning): a value's
// position is its projection-trie node, or for an array element the trie's
// element node (kv_pos_elem: a pseudo id when the trie has none); -1 = a child
// of a keep-all map or an element of an unknown position. Both ingest and the
// specialized-kernel generator derive the same ids from the same trie.
KV_HD inline int32_t kv_pos_elem(int32_t pos, int32_t trie_node) {
  (void)trie_node;
  return pos < 0 ? -1 : (int32_t)(0x100000 + pos);
}
KV_HD inline uint32_t kv_tcls(int32_t pos) { return 1u << (pos < 0 ? 31u : (uint32_t)pos % 31u); }
KV_HD inline uint32_t node_key(uint32_t kt) { return kt >> 4; }

constexpr uint32_t KEY_NONE = 0xFFFFFFFFu;

// Deduplicated scalar value record (per batch). String forms refer to the
// batch string heap. Precomputed at ingest from the Go semantics of
// pkg/engine/validate/pattern.go (validateString / validateNumberWithStr /
// validateValueWithFloatPattern / validateValueWithNilPattern).
struct Val {
  uint32_t type;      // NT_BOOL/INT/FLOAT/STR
  uint32_t flags;     // VF_*
  uint32_t e_off, e_len;  // validateString form: FormatFloat 'E' / decimal / raw / "true"|"false"
  uint32_t n_off, n_len;  // validateNumberWithStr form: %f / decimal / raw (invalid for bool)
  int32_t q_exp;          // quantity of the n-form: order of magnitude (digits + exp10)
  uint32_t cls;           // position classes referencing this value: bit kv_tcls(trie node) of every node
                          // holding it (value-predicate table pruning, kvjit.cpp ptab_kernel)
  uint64_t q_hi, q_lo;    // 38 left-aligned significant decimal digits (19 + 19)
  double f;               // FLOAT: value; STR: ParseFloat(value) when VF_PF_OK
  int64_t i;              // INT: value
};

enum ValFlags : uint32_t {
  VF_Q_VALID = 1u << 0,   // n-form parses as a resource.Quantity
  VF_Q_NEG = 1u << 1,
  VF_Q_ZERO = 1u << 2,
  VF_PF_OK = 1u << 3,     // STR: strconv.ParseFloat succeeded
  VF_NILLIKE = 1u << 4,   // validateValueWithNilPattern true (0, 0.0, "", false)
  VF_BOOLV = 1u << 5,     // BOOL value
  VF_ASCII_E = 1u << 6,   // e-form is ASCII
  VF_ASCII_N = 1u << 7,   // n-form is ASCII
  VF_N_VALID = 1u << 8,   // n-form exists (not bool)
};

// Per-resource header used by the match/exclude prefilter and as the tree root.
// The match inputs that repeat across resources are interned per batch and
// referenced by id, so the match tables (DevPS::mt_*) evaluate each glob /
// selector / annotation filter once per distinct input (kv_mtab):
//   nsm  = the string checkNameSpace globs (the namespace; the name for kind
//          Namespace, pkg/engine/utils.go:62-75), Batch::nsms
//   lset = the resource's label list (selector + wildcard expansion, utils.go:99-107)
//   aset = the resource's annotation list (checkAnnotations, utils.go:77-97)
struct Res {
  uint32_t root;          // ROW of the root node (node index root * KV_LANES + r % KV_LANES)
  uint32_t kind;          // key-dictionary id of .kind (KEY_NONE if not in dictionary)
  uint32_t group, version;// dictionary ids of the apiVersion group / version
  uint32_t name_off, name_len;
  uint32_t nsm, lset, aset;
  uint32_t ns_index;      // index into the batch namespace table (namespaceSelector bits, report scope)
  uint32_t flags;         // RF_*
  uint32_t tup;           // match tuple: resources with equal match inputs (every field above
                          // but root and name) share one (Batch::tup_rep, kv_mtup_kernel)
  uint32_t pad[4];
};

// a label / annotation list of a batch: kvs[first, first + count), sorted by key bytes
// (count 0 when the field is not a string map: NestedStringMap error -> nil map)
struct KVSet {
  uint32_t first, count;
};

enum ResFlags : uint32_t {
  RF_KIND_NAMESPACE = 1u << 0,  // kind == "Namespace"
  RF_KIND_EMPTY = 1u << 1,      // kind == ""
  RF_BAD_META = 1u << 2,        // some metadata/labels/annotations shape would make ExpandInMetadata panic
  RF_MAGIC = 1u << 3,           // a string/key contains "conditional anchor mismatch" / "global anchor mismatch"
  RF_NAME_ASCII = 1u << 4,      // metadata.name is ASCII (word globs exact for '?')
  RF_BAD_LABELS = 1u << 5,      // ... through a labels map (a non-map metadata, or non-string label values)
  RF_BAD_ANN = 1u << 6,         // ... through an annotations map
};

struct KV {
  uint32_t k_off, k_len;  // k_len high bit: label key is a valid qualified name
  uint32_t v_off, v_len;  // v_len high bit: label value is valid
};
constexpr uint32_t KV_VALID = 0x80000000u;
constexpr uint32_t KV_LEN_MASK = 0x7FFFFFFFu;

// ---------------------------------------------------------------- program
// Status codes (response.RuleStatus, pkg/engine/response/status.go:14-28) + extras
enum Status : uint8_t { ST_PASS = 0, ST_FAIL = 1, ST_WARN = 2, ST_ERROR = 3, ST_SKIP = 4, ST_NOMATCH = 5, ST_CPU = 6 };

// Error kinds raised by the pattern VM (one per reference error message form)
enum ErrKind : uint32_t {
  E_NONE = 0,
  E_TYPE_MAP = 1,       // "pattern and resource have different structures..."   validate.go:62
  E_TYPE_ARR = 2,       // "validation rule Failed at path %s, resource does not satisfy..." validate.go:72
  E_VALUE = 3,          // "resource value '%v' does not match '%v' at path %s"  validate.go:83,89
  E_EMPTY_PATARR = 4,   // "pattern Array empty" validate.go:142
  E_LEN = 5,            // "validate Array failed, array length mismatch..." validate.go:172 (path "")
  E_NEG = 6,            // "%s/%s is not allowed" anchor.go:62
  E_STAR = 7,           // "%s/%s not found" anchor.go:139 (parent path)
  E_EXIST_PATLIST = 8,  // anchor.go:235
  E_EXIST_PATMAP = 9,   // anchor.go:243
  E_EXIST_RESTYPE = 10, // anchor.go:252
  E_EXIST_FAIL = 11,    // anchor.go:261
  E_CPU = 12,           // route this pair to the CPU engine (would-panic shapes)
};
enum ErrFlags : uint32_t { EF_COND = 1, EF_GLOBAL = 2 };

// Opcodes of the structured pattern program (uniform-pc SIMT interpreter).
enum Op : uint32_t {
  OP_NOP = 0,
  OP_MAPCHK,      // d, node: cur[d] must be a map                     (validateResourceElement map case)
  OP_ARRCHK,      // d, node: cur[d] must be an array
  OP_AREG,        // d, key, bit: anchor registration (CheckAnchorInResource)
  OP_METACHK,     // resource must not have panicking metadata shapes
  OP_KEY,         // d, key, end: cur[d+1] = cur[d][key]; absent lanes skip to `end`
  OP_KEYV,        // d, key: cur[d+1] = cur[d][key] or ABSENT (default handler)
  OP_KEYGLOB,     // d, str, key(literal), end|0: wildcard label key resolution (ExpandInMetadata)
  OP_SCOPE_END,   // end of a key-present scope; wrap flags in aux (EF_COND / EF_GLOBAL)
  OP_NEG,         // d, key, node: negation anchor
  OP_STAR,        // d, key, node(parent): "*" default shortcut
  OP_LEAF,        // d, pred, node: scalar compare (all elements when cur[d] is an array)
  OP_RAISE,       // node, kind: constant error for active lanes
  OP_LOOP_BEGIN,  // d, loop level, end: iterate children of cur[d] into cur[d+1]
  OP_LOOP_END,    // begin, loop level: array-of-maps (swallow conditional errors)
  OP_EXIST_BEGIN, // d, loop level, end: existence search over children of cur[d]
  OP_EXIST_END,   // begin, loop level, node: first success wins; none -> E_EXIST_FAIL at node
  OP_EXISTCHK,    // d, node: existence anchor value must be an array
  OP_LENCHK,      // d, n: positional nested array length check
  OP_INDEX,       // d, i: cur[d+1] = child i of cur[d]
  OP_POS_END,     // end of a positional element scope (swallow conditional errors)
  OP_ALT_BEGIN,   // anyPattern alternative start: reset error / anchors
  OP_ALT_END,     // anyPattern alternative end: PASS lanes finish
  OP_DONE,        // program end
  OP_VLEAF,       // d, dynamic leaf, node: OP_LEAF with the per-resource predicate of a pattern
                  // string holding variables (DevBatch::dleaf -> DevBatch::dps, kvvars.cpp)
};

// Key-lookup ops (KEY, KEYV, AREG, NEG): `a` is the slot index of the key in
// the parent map's slot list, or (aux & AUX_SCAN) the key id for a keep-all map.
constexpr uint32_t AUX_SCAN = 0x80;

struct Inst {
  uint32_t op;     // Op | (depth << 8) | (aux << 16)
  uint32_t a;
  uint32_t b;
  uint32_t c;      // catch pc (where a raised error goes next)
};

// Predicates (per pattern leaf), pkg/engine/validate/pattern.go:25-318
enum PredKind : uint32_t { PK_BOOL = 0, PK_FLOAT = 1, PK_NIL = 2, PK_STRING = 3, PK_FALSE = 4, PK_MAPTYPE = 5 };
struct Pred {
  uint32_t kind;
  uint32_t first, count;  // PK_STRING: alternatives [first, first+count) in alts[]
  uint32_t flags;         // PK_BOOL: value; PK_FLOAT: 1 if integral
  double f;               // PK_FLOAT value
  int64_t fi;             // PK_FLOAT: int64(pattern) (amd64 conversion)
};
struct Alt {              // one '|' alternative: AND of conjuncts
  uint32_t first, count;  // conjuncts [first, first+count) in conjs[]
};
enum ConjKind : uint32_t { CJ_ATOM = 0, CJ_INRANGE = 1, CJ_NOTINRANGE = 2 };
struct Conj {             // one '&' part
  uint32_t kind;
  uint32_t a0, a1;        // atom indices (a1 for ranges)
  uint32_t pad;
};
enum AtomKind : uint32_t { AT_FALSE = 0, AT_GLOB_E = 1, AT_GLOB_N = 2, AT_QCMP = 3 };
enum CmpOp : uint32_t { CO_EQ = 0, CO_NE = 1, CO_GT = 2, CO_LT = 3, CO_GE = 4, CO_LE = 5 };
struct Atom {
  uint32_t kind;
  uint32_t op;            // CmpOp (AT_GLOB_E: CO_EQ or CO_NE)
  uint32_t s_off, s_len;  // glob pattern bytes in the program string table (s_len high bit: ASCII)
  int32_t q_exp;
  uint32_t q_flags;       // VF_Q_NEG | VF_Q_ZERO
  uint64_t q_hi, q_lo;
  // compiled glob (segments between '*'): see GlobFlags
  uint32_t gflags, gfirst, gcount, gmin;
};

// Glob patterns are compiled into '*'-separated segments matched on 4-byte
// words of 4-byte aligned value strings: anchored prefix, anchored suffix,
// then middle segments leftmost-first. Exact for ASCII values, and for any
// UTF-8 value when the pattern has no '?' (a '?' consumes one rune).
enum GlobFlags : uint32_t {
  G_ALL = 1,    // pattern "*" (or only stars): matches everything
  G_LEAD = 2,   // pattern starts with '*'
  G_TRAIL = 4,  // pattern ends with '*'
  G_HASQ = 8,   // some segment contains '?'
  G_EMPTY = 16, // empty pattern: matches only ""
};
struct GSeg { uint32_t wfirst, len; };   // words [wfirst, wfirst + (len+3)/4) in gwords[]
struct GWord { uint32_t w, mask; };      // little-endian bytes, mask 0 on '?' and past the end

// ---------------------------------------------------------------- match/exclude
struct MFilter {          // one ResourceFilter / condition block
  uint32_t flags;         // MF_*
  uint32_t kinds_first, kinds_count;       // KindSpec[]
  uint32_t name_off, name_len;             // `name` glob
  uint32_t names_first, names_count;       // StrRef[] globs
  uint32_t nss_first, nss_count;           // StrRef[] namespace globs
  uint32_t ann_first, ann_count;           // StrPair[] annotation globs
  uint32_t sel;                            // Selector index (MF_SEL): bit of the label-set match table
  uint32_t nssel_bit;                      // bit in the per-namespace table (MF_NSSEL)
  uint32_t nss_bit;                        // bit of the namespace-glob match table (MF_NSS)
  uint32_t ann_bit;                        // bit of the annotation match table (MF_ANN)
};
enum MFilterFlags : uint32_t {
  MF_EMPTY = 1u << 0,     // ResourceDescription and UserInfo empty ("match cannot be empty")
  MF_KINDS = 1u << 1, MF_NAME = 1u << 2, MF_NAMES = 1u << 3, MF_NSS = 1u << 4, MF_ANN = 1u << 5,
  MF_SEL = 1u << 6, MF_NSSEL = 1u << 7,
  MF_UI_FAIL = 1u << 8,   // user-info part adds errors (batch constant, folded per launch)
};
struct KindSpec { uint32_t form, kind, version, group; };  // form 0: kind or '*'(kind==KEY_NONE... see compiler), 1: v/K, 2: g/v/K
struct StrRef { uint32_t off, len; };
struct StrPair { uint32_t k_off, k_len, v_off, v_len; };
struct Selector {
  uint32_t flags;           // SF_*
  uint32_t ml_first, ml_count;   // SelLabel[]
  uint32_t me_first, me_count;   // SelExpr[]
};
enum SelFlags : uint32_t { SF_EVERYTHING = 1, SF_STATIC_INVALID = 2 };
struct SelLabel {           // one matchLabels entry (canonical order)
  uint32_t flags;           // SL_WILD | SL_VALID (static entry / unmatched-replacement validity)
  uint32_t k_off, k_len, v_off, v_len;     // pattern key / value (globs if SL_WILD)
  uint32_t rk_off, rk_len, rv_off, rv_len; // '*'/'?' -> '0' replacements (SL_WILD)
};
enum SelLabelFlags : uint32_t { SL_WILD = 1, SL_VALID = 2 };
struct SelExpr {
  uint32_t op;              // 0 In, 1 NotIn, 2 Exists, 3 DoesNotExist
  uint32_t k_off, k_len;
  uint32_t v_first, v_count;   // StrRef[]
};

// Per-rule record.
struct RuleRec {
  uint32_t route;           // 0 GPU, 1 CPU (status ST_CPU), 2 no response (ST_NOMATCH), 3 constant status
  uint32_t const_status;    // route 3
  uint32_t prog;            // first instruction
  uint32_t flags;           // RR_*
  uint32_t m_mode, m_first, m_count;  // match: 0 legacy, 1 any, 2 all; filters
  uint32_t x_mode, x_first, x_count;  // exclude
  uint32_t n_alts;          // 0: pattern; >0: anyPattern alternatives
  uint32_t dyn;             // pattern variables: 1 + dynamic-rule index (DevBatch::dyn_st), 0 none
};
// RR_META_LABELS / RR_META_ANN: the pattern's ExpandInMetadata sites read labels / annotations
// (wildcards.go:69-139 panics on a resource whose map of that tag is not a string map)
enum RuleFlags : uint32_t { RR_META_EXPAND = 1, RR_META_LABELS = 2, RR_META_ANN = 4 };
// resource flags that make rule flags `rf` panic in ExpandInMetadata (routed: ST_CPU)
KV_HD constexpr uint32_t meta_bad_flags(uint32_t rf) {
  return ((rf & RR_META_LABELS) ? (uint32_t)RF_BAD_LABELS : 0u) | ((rf & RR_META_ANN) ? (uint32_t)RF_BAD_ANN : 0u);
}

}  // namespace kv
