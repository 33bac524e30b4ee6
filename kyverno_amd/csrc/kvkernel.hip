// HIP kernels of libkvgpu (gfx950 / CDNA4).
//
// kv_validate_kernel: one lane = one resource; a workgroup owns 256 resources
// and a chunk of rules, and every wave walks its rules in order, so the rule's
// program, predicates and compiled glob segments are wave-uniform (scalar
// loads), while resource nodes are per-lane gathers from the projected HBM
// store. Per rule:
//   1. match/exclude prefilter (MatchesResourceDescription, pkg/engine/utils.go:265-336)
//   2. pattern VM: a uniform-pc SIMT interpreter over the structured program
//      emitted by kvcompile.cpp (validate.go:29-194, anchor.go:21-277). Lanes
//      that skip a subtree (absent anchored key) or raise an error park on a
//      wake-up pc (the scope end / catch point) instead of branching, so the
//      wave never diverges in program position; loops over resource arrays
//      (containers[], volumes[] ...) run max(len) uniform iterations.
//   3. MatchPattern epilogue (validate.go:29-50) -> status, error record.
// Workgroup -> (resource block, rule chunk) mapping is XCD-aware: all rule
// chunks of one resource block land on the same XCD (same L2) back to back.
// Output: status[rule][res] (+ error records) and a per-rule histogram
// accumulated in LDS and flushed with one atomic per counter per workgroup.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "kvdev.h"

using namespace kv;

#define KV_MAXD 16
#define KV_MAXL 4
#define KV_RCHUNK 64

#include "kvdevfn.h"
#include "kvfac.h"
#include "kvcol.h"

// ------------------------------------------------------------------ kernel
extern "C" __global__ __launch_bounds__(KV_WG) __attribute__((amdgpu_waves_per_eu(4))) void kv_validate_kernel(const DevPS* __restrict__ Pp,
                                                                      const DevBatch* __restrict__ Bp, DevOut O,
                                                                      uint32_t rule_begin, uint32_t rule_end,
                                                                      uint32_t n_chunks, uint32_t rblocks) {
  __shared__ uint32_t s_cur[KV_MAXD][KV_WG];
  __shared__ uint32_t s_lfirst[KV_MAXL][KV_WG];
  __shared__ uint32_t s_llen[KV_MAXL][KV_WG];
  __shared__ uint32_t s_li[KV_WG / 64][KV_MAXL];
  __shared__ uint32_t s_hist[KV_RCHUNK][KV_HIST];

  const DevPS& P = *Pp;
  const DevBatch& B = *Bp;
  const Node* __restrict__ N = B.nodes;
  // XCD-aware work mapping: block ids b and b+8 share an XCD (and its L2), so
  // every rule chunk of one resource block is placed on the same XCD.
  const uint32_t xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const uint32_t rblock = (slot / n_chunks) * 8 + xcd;
  const uint32_t chunk = slot % n_chunks;
  if (rblock >= rblocks) return;
  const uint32_t per = (rule_end - rule_begin + n_chunks - 1) / n_chunks;
  const uint32_t cb = rule_begin + chunk * per;
  const uint32_t ce = cb + per < rule_end ? cb + per : rule_end;
  if (cb >= ce) return;

  const uint32_t lane = threadIdx.x;
  const uint32_t wv = lane >> 6;
  const uint32_t r = rblock * KV_WG + lane;
  const uint32_t n_res = B.n_res;
  const bool valid = r < n_res;
  const Res* R = B.res + (valid ? r : 0);
  uint32_t rroot = ABSENT, rkind = KEY_NONE, rflags = 0;
  if (valid) {
    rroot = ni(R->root);
    rkind = R->kind;
    rflags = R->flags;
  }

  for (uint32_t rb = cb; rb < ce; rb += KV_RCHUNK) {
    const uint32_t re = rb + KV_RCHUNK < ce ? rb + KV_RCHUNK : ce;
    for (uint32_t q = lane; q < KV_RCHUNK * KV_HIST; q += KV_WG) (&s_hist[0][0])[q] = 0;
    __syncthreads();
    for (uint32_t ri = rb; ri < re; ri++) {
      const RuleRec& rr = P.rules[ri];
      const uint32_t route = uni(rr.route);
      uint32_t st = ST_NOMATCH;
      bool run = false;
      if (valid && rule_matches(P, B, R, rkind, rflags, rr)) {
        if (route == 1) st = ST_CPU;
        else if (route == 2) st = ST_NOMATCH;
        else if (route == 3) st = (uint8_t)uni(rr.const_status);
        else if (rflags & RF_MAGIC) st = ST_CPU;
        else if (rflags & meta_bad_flags(uni(rr.flags))) st = ST_CPU;
        else if (uni(rr.dyn) && B.dyn_st[(size_t)(uni(rr.dyn) - 1u) * n_res + r]) st = B.dyn_st[(size_t)(uni(rr.dyn) - 1u) * n_res + r];
        else run = true;
      }
      uint32_t ekind = 0, eflags = 0, epn = 0, ekey = ABSENT, eres = ABSENT;
      uint32_t eidx0 = 0, eidx1 = 0, eidx2 = 0, eidx3 = 0;
      if (__ballot(run)) {
        uint64_t areg = 0, apres = 0;
        uint32_t keynode = ABSENT;
        uint32_t wait = run ? 0u : KV_SENT;
        uint32_t pc = uni(rr.prog);
        s_cur[0][lane] = rroot;
        auto raise = [&](uint32_t kind, uint32_t pn, uint32_t rn, uint32_t cpc) {
          ekind = kind;
          eflags = 0;
          epn = pn;
          eres = rn;
          ekey = keynode;
          eidx0 = s_li[wv][0];
          eidx1 = s_li[wv][1];
          eidx2 = s_li[wv][2];
          eidx3 = s_li[wv][3];
          wait = cpc;
        };
        uint32_t guard = 0;
        while (true) {
          // every program terminates (forward pcs, loops bounded by array lengths);
          // the guard only turns an interpreter bug into a CPU-routed verdict instead of a hung wave
          if (++guard > (1u << 24)) {
            if (wait != KV_SENT) st = ST_CPU;
            break;
          }
          if (wait == pc) wait = 0;
          if (!__ballot(wait == 0)) {
            const uint32_t m = uni(wave_min(wait));
            if (m == KV_SENT) break;
            pc = m;
            continue;
          }
          const Inst& in = P.prog[pc];
          const uint32_t opw = uni(in.op);
          const uint32_t op = opw & 0xFF;
          const uint32_t d = (opw >> 8) & 0xFF;
          const uint32_t aux = (opw >> 16) & 0xFF;
          const uint32_t ia = uni(in.a), ib = uni(in.b), ic = uni(in.c);
          const bool A = wait == 0;
          uint32_t next = pc + 1;
          switch (op) {
            case OP_MAPCHK:
            case OP_ARRCHK:
              if (A) {
                const uint32_t v = s_cur[d][lane];
                const uint32_t want = op == OP_MAPCHK ? NT_MAP : NT_ARR;
                if (v == ABSENT || node_type(N[v].kt) != want) raise(op == OP_MAPCHK ? E_TYPE_MAP : E_TYPE_ARR, ia, v, ic);
              }
              break;
            case OP_AREG:
              if (A) {
                areg |= 1ull << (aux & 63);
                if (lookup_op(N, s_cur[d][lane], ia, aux) != ABSENT) apres |= 1ull << (aux & 63);
              }
              break;
            case OP_KEY:
            case OP_KEYV:
              if (A) {
                const uint32_t c = lookup_op(N, s_cur[d][lane], ia, aux);
                s_cur[d + 1][lane] = c;
                if (op == OP_KEY && c == ABSENT) wait = ib;
              }
              break;
            case OP_KEYGLOB:
              if (A) {
                uint32_t node;
                if (keyglob_op(P, B, N, s_cur[d][lane], opw, ia, ic, &node, &keynode)) s_cur[d + 1][lane] = node;
                else wait = ib;
              }
              break;
            case OP_SCOPE_END:
            case OP_POS_END:
              if (A && ekind) {
                if (op == OP_POS_END) {
                  if (eflags & EF_COND) ekind = 0;
                  else wait = ic;
                } else {
                  eflags |= aux;
                  wait = ic;
                }
              }
              break;
            case OP_NEG:
              if (A && lookup_op(N, s_cur[d][lane], ia, aux) != ABSENT) raise(E_NEG, ib, ABSENT, ic);
              break;
            case OP_STAR:
              if (A) {
                const uint32_t v = s_cur[d + 1][lane];
                if (v == ABSENT || node_type(N[v].kt) == NT_NULL) raise(E_STAR, ib, ABSENT, ic);
              }
              break;
            case OP_LEAF:
              if (A) {
                const uint32_t v = s_cur[d][lane];
                Node vn{NT_NULL, 0, 0, 0};
                if (v != ABSENT) vn = N[v];
                const uint32_t vt = node_type(vn.kt);
                bool ok;
                if (vt == NT_ARR) {
                  ok = true;
                  for (uint32_t k = 0; k < vn.b && ok; k++) ok = pred_node(P, B, N, ia, ni(vn.a + k));
                } else {
                  ok = pred_eval(P, B, ia, vt, vn);
                }
                if (!ok) raise(E_VALUE, ib, v, ic);
              }
              break;
            case OP_VLEAF:  // the resource's substituted pattern value (kvvars.cpp): batch predicate table
              if (A) {
                const uint32_t v = s_cur[d][lane];
                const uint32_t dp = B.dleaf[(size_t)ia * n_res + r];
                Node vn{NT_NULL, 0, 0, 0};
                if (v != ABSENT) vn = N[v];
                const uint32_t vt = node_type(vn.kt);
                bool ok;
                if (vt == NT_ARR) {
                  ok = true;
                  for (uint32_t k = 0; k < vn.b && ok; k++) ok = pred_node(*B.dps, B, N, dp, ni(vn.a + k));
                } else {
                  ok = pred_eval(*B.dps, B, dp, vt, vn);
                }
                if (!ok) raise(E_VALUE, ib, v, ic);
              }
              break;
            case OP_RAISE:
              if (A) raise(ib, ia, s_cur[d][lane], ic);
              break;
            case OP_EXISTCHK:
              if (A) {
                const uint32_t v = s_cur[d][lane];
                if (v == ABSENT || node_type(N[v].kt) != NT_ARR) raise(E_EXIST_RESTYPE, ia, v, ic);
              }
              break;
            case OP_LENCHK:
              if (A && N[s_cur[d][lane]].b < ia) raise(E_LEN, ib, s_cur[d][lane], ic);
              break;
            case OP_INDEX:
              if (A) s_cur[d + 1][lane] = ni(N[s_cur[d][lane]].a + ia);
              break;
            case OP_LOOP_BEGIN:
            case OP_EXIST_BEGIN: {
              if (A) {
                const Node an = N[s_cur[d][lane]];
                s_lfirst[aux][lane] = an.a;
                s_llen[aux][lane] = an.b;
                if (an.b == 0) {
                  if (op == OP_LOOP_BEGIN) wait = ia + 1;
                  else raise(E_EXIST_FAIL, ib, s_cur[d][lane], ic);
                } else {
                  s_cur[d + 1][lane] = ni(an.a);
                }
              }
              if (lane % 64 == 0) s_li[wv][aux] = 0;
              break;
            }
            case OP_LOOP_END:
            case OP_EXIST_END: {
              bool cont = false;
              if (A) {
                if (op == OP_LOOP_END) {
                  if (ekind) {
                    if (eflags & EF_COND) { ekind = 0; cont = true; }
                    else wait = ic;
                  } else {
                    cont = true;
                  }
                } else {
                  if (ekind) { ekind = 0; cont = true; }  // element failed: try the next one
                  else wait = pc + 1;                       // found
                }
                if (cont) {
                  const uint32_t i = s_li[wv][aux] + 1;
                  if (i < s_llen[aux][lane]) {
                    s_cur[d + 1][lane] = ni(s_lfirst[aux][lane] + i);
                  } else {
                    cont = false;
                    if (op == OP_LOOP_END) wait = pc + 1;
                    else raise(E_EXIST_FAIL, ib, s_cur[d][lane], ic);
                  }
                }
              }
              if (__ballot(cont)) {
                if (lane % 64 == 0) s_li[wv][aux] += 1;
                next = ia + 1;
              }
              break;
            }
            case OP_ALT_BEGIN:
              if (A) { ekind = 0; eflags = 0; areg = 0; apres = 0; }
              break;
            case OP_ALT_END:
              if (A) {
                if (ekind == 0) { st = ST_PASS; wait = KV_SENT; }
                else if (ekind == E_CPU) { st = ST_CPU; wait = KV_SENT; }
                else if (ib) { st = ST_FAIL; wait = KV_SENT; }
                else { ekind = 0; eflags = 0; areg = 0; apres = 0; }
              }
              break;
            case OP_DONE:
              if (A) {
                if (ekind == 0) st = ST_PASS;
                else if (ekind == E_CPU) st = ST_CPU;
                else if (eflags & (EF_COND | EF_GLOBAL)) st = ST_SKIP;
                else if (areg & ~apres) st = ST_ERROR;
                else if (ekind == E_LEN) st = ST_ERROR;
                else st = ST_FAIL;
                wait = KV_SENT;
              }
              next = KV_SENT;
              break;
            default:
              break;
          }
          if (next == KV_SENT) break;
          pc = next;
        }
      }
      if (valid && (O.full & 1)) {
        const size_t o = (size_t)ri * n_res + r;
        O.status[o] = (uint8_t)st;
        if ((O.full & 2) && (st == ST_FAIL || st == ST_ERROR || st == ST_SKIP))
          store_err(O, ri, n_res, r, ekind, eflags, epn, ekey, eres, eidx0, eidx1, eidx2, eidx3);
      }
      // histogram: one LDS atomic per (wave, status) via ballot popcount
      for (uint32_t s = 0; s < 7; s++) {
        const uint64_t bm = __ballot(valid && st == s);
        if (bm && (lane % 64) == 0) atomicAdd(&s_hist[ri - rb][s], (uint32_t)__popcll(bm));
      }
    }
    __syncthreads();
    for (uint32_t q = lane; q < (re - rb) * KV_HIST; q += KV_WG) {
      const uint32_t v = (&s_hist[0][0])[q];
      if (v) atomicAdd(&O.counts[(size_t)rb * KV_HIST + q], (unsigned long long)v);
    }
    __syncthreads();
  }
}

namespace kv {
hipError_t launch_validate(const DevPS* P, const DevBatch* B, uint32_t n_res, const DevOut& O, uint32_t rule_begin,
                           uint32_t rule_end, hipStream_t stream) {
  if (n_res == 0 || rule_end <= rule_begin) return hipSuccess;
  const uint32_t rblocks = (n_res + KV_WG - 1) / KV_WG;
  const uint32_t nrules = rule_end - rule_begin;
  // enough workgroups to fill 256 CUs several times over; each chunk re-reads
  // its resources from L2, so chunks stay >= 8 rules
  uint32_t n_chunks = (16384 + rblocks - 1) / rblocks;
  uint32_t max_chunks = (nrules + 7) / 8;
  if (n_chunks > max_chunks) n_chunks = max_chunks;
  if (n_chunks < 1) n_chunks = 1;
  const uint32_t rb8 = (rblocks + 7) / 8 * 8;
  dim3 grid(rb8 * n_chunks);
  hipLaunchKernelGGL(kv_validate_kernel, grid, dim3(KV_WG), 0, stream, P, B, O, rule_begin, rule_end, n_chunks,
                     rblocks);
  return hipGetLastError();
}
}  // namespace kv

// ---------------------------------------------------------------------------
// Match tables of one pass (both engines): every namespace glob set, annotation
// filter and label selector of the policy set, once per distinct input of the
// batch (DevPS::mt_*). grid.y = table word, grid.x = entities.
namespace kv {

// 32 lanes per (row y, entity): lane k evaluates bit k, a ballot assembles the words of
// the wave's two entities (a batch has few distinct match inputs, so one thread per word
// ran 32 criteria serially on a handful of waves: C4 108 us per pass)
__global__ __launch_bounds__(KV_WG) void kv_mtab_kernel(const DevPS* __restrict__ Pp, const DevBatch* __restrict__ Bp,
                                                         uint32_t* __restrict__ ns, uint32_t* __restrict__ an,
                                                         uint32_t* __restrict__ sl) {
  const DevPS& P = *Pp;
  const DevBatch& B = *Bp;
  const uint32_t y = blockIdx.y, k = threadIdx.x & 31u;
  const uint32_t e = blockIdx.x * (KV_WG / 32) + threadIdx.x / 32u;
  const uint32_t ne = mtab_entities(P, B, y);
  const bool v = e < ne && mtab_bit(P, B, y, e, k);
  const uint64_t m = __ballot(v);
  if (k != 0 || e >= ne) return;
  const uint32_t w = (threadIdx.x & 32u) ? (uint32_t)(m >> 32) : (uint32_t)m;
  if (y < P.mt_ns_words) ns[(size_t)y * B.n_nsm + e] = w;
  else if (y < P.mt_ns_words + P.mt_ann_words) an[(size_t)(y - P.mt_ns_words) * B.n_asets + e] = w;
  else sl[(size_t)(y - P.mt_ns_words - P.mt_ann_words) * B.n_lsets + e] = w;
}

hipError_t launch_mtab(const DevPS* P, const DevBatch* B, uint32_t words, uint32_t max_entities, uint32_t* ns,
                       uint32_t* an, uint32_t* sl, hipStream_t stream) {
  if (words == 0 || max_entities == 0) return hipSuccess;
  hipLaunchKernelGGL(kv_mtab_kernel, dim3((max_entities + KV_WG / 32 - 1) / (KV_WG / 32), words), dim3(KV_WG), 0, stream,
                     P, B, ns, an, sl);
  return hipGetLastError();
}

// Factored match tables (DevPS::fac_*): grid.z = entity type, grid.y = slot, grid.x = groups
// of 8 entities; 32 lanes per (entity, slot) evaluate the word's 32 bits at once (lane k: bit
// k) and a ballot assembles the word (one lane per word walked the 32 filter lists one after
// the other: 33 us per pass on C2, a chain of dependent loads)
__global__ __launch_bounds__(KV_WG) void kv_mfac_kernel(const DevPS* __restrict__ Pp, const DevBatch* __restrict__ Bp) {
  const DevPS& P = *Pp;
  const DevBatch& B = *Bp;
  const uint32_t t = blockIdx.z, s = blockIdx.y, k = threadIdx.x & 31u;
  const uint32_t e = blockIdx.x * (KV_WG / 32) + threadIdx.x / 32u;
  const uint32_t ne = fac_entities(B, t);
  const bool v = e < ne && fac_bit_of(P, B, t, e, s, k);
  const uint64_t m = __ballot(v);
  if (k != 0 || e >= ne) return;
  P.fac_tab[P.fac_off[t] + (size_t)s * ne + e] = (threadIdx.x & 32u) ? (uint32_t)(m >> 32) : (uint32_t)m;
}

// Match words per tuple: grid.x = tuples, grid.y = runs of KV_MTUP_WORDS words (uniform plane
// counts and masks); a thread reads its tuple's entities once for its run of words (one word
// per thread re-read the tuple's Res for every word: C3, 62 words, 2.9 GB per pass);
// mtup[w * n_tup + t] (word-major: a wave writes 256 contiguous bytes per word)
constexpr uint32_t KV_MTUP_WORDS = 8u;
__global__ __launch_bounds__(KV_WG) void kv_mtup_kernel(const DevPS* __restrict__ Pp, const DevBatch* __restrict__ Bp,
                                                         uint32_t* __restrict__ out) {
  const DevPS& P = *Pp;
  const DevBatch& B = *Bp;
  const uint32_t t = blockIdx.x * KV_WG + threadIdx.x, w0 = blockIdx.y * KV_MTUP_WORDS;
  if (t >= B.n_tup) return;
  const MtupIn in = mtup_in(B, t);
  const uint32_t w1 = min(w0 + KV_MTUP_WORDS, P.fac_words);
  for (uint32_t w = w0; w < w1; w++) out[(size_t)w * B.n_tup + t] = mtup_word_in(P, B, in, w);
}

// out[rule][j] = in[rule][inv[j]]: a status matrix in store order gathered into the caller's
// resource order (writes coalesced; reads follow the permutation, which keeps runs of a kind
// and namespace together)
__global__ __launch_bounds__(KV_WG) void kv_gather_rows_kernel(const uint8_t* __restrict__ in,
                                                                const uint32_t* __restrict__ inv, uint64_t n_res,
                                                                uint8_t* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * KV_WG + threadIdx.x, rule = blockIdx.y;
  if (j < n_res) out[rule * n_res + j] = in[rule * n_res + inv[j]];
}

hipError_t launch_gather_rows(const uint8_t* in, const uint32_t* inv, uint64_t n_rules, uint64_t n_res, uint8_t* out,
                              hipStream_t stream) {
  if (!n_rules || !n_res) return hipSuccess;
  hipLaunchKernelGGL(kv_gather_rows_kernel, dim3((uint32_t)((n_res + KV_WG - 1) / KV_WG), (uint32_t)n_rules), dim3(KV_WG),
                     0, stream, in, inv, n_res, out);
  return hipGetLastError();
}

// a[i] = map[a[i]] (scope renumbering of a parts session, kv_session_attach_part)
__global__ __launch_bounds__(KV_WG) void kv_remap_kernel(uint32_t* __restrict__ a, uint64_t n,
                                                          const uint32_t* __restrict__ map) {
  const uint64_t i = (uint64_t)blockIdx.x * KV_WG + threadIdx.x;
  if (i < n) a[i] = map[a[i]];
}

hipError_t launch_remap_u32(uint32_t* a, uint64_t n, const uint32_t* map, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(kv_remap_kernel, dim3((uint32_t)((n + KV_WG - 1) / KV_WG)), dim3(KV_WG), 0, stream, a, n, map);
  return hipGetLastError();
}

hipError_t launch_mfac(const DevPS* P, const DevBatch* B, uint32_t slots, uint32_t max_entities, uint32_t words,
                       uint32_t n_tup, uint32_t* mtup, hipStream_t stream) {
  if (slots && max_entities)
    hipLaunchKernelGGL(kv_mfac_kernel, dim3((max_entities + KV_WG / 32 - 1) / (KV_WG / 32), slots, KV_FAC_TYPES),
                       dim3(KV_WG), 0, stream, P, B);
  if (words && n_tup)
    hipLaunchKernelGGL(kv_mtup_kernel, dim3((n_tup + KV_WG - 1) / KV_WG, (words + KV_MTUP_WORDS - 1) / KV_MTUP_WORDS),
                       dim3(KV_WG), 0, stream, P, B, mtup);
  return hipGetLastError();
}

}  // namespace kv

// ---------------------------------------------------------------------------
// Error-record compaction (fetch time, outside the timed passes): the rule
// kernels write an 8 B record per FAIL / ERROR / SKIP pair, at its [rule][res] slot
// (bytecode engine; specialized rule-group members) or appended to its wave's 64-slot
// segment of the rule's row (the other specialized rules, compact[rule] = 1; the record
// carries its lane); these kernels gather them, rule-major and in resource order, into a
// compact array, so only the records cross PCIe. Tiles of KV_WG resources: count -> per-rule exclusive scan over tiles -> rule
// bases -> scatter.
namespace kv {

__device__ __forceinline__ bool has_record(uint8_t s) { return s == ST_FAIL || s == ST_ERROR || s == ST_SKIP; }

// A workgroup walks tiles blockIdx.x, + gridDim.x, ... of one rule (a workgroup per (tile, rule)
// was 9.6 M workgroups at C3, 8 ms of dispatch for 2.5 GB of statuses)
static_assert(KV_WG == KV_RWG, "a record tile is one status segment of a rule kernel's workgroup (sflag)");
// sflag (specialized passes): a tile whose segment the pass did not write is all NOMATCH: no
// records, and its statuses (never written, never filled) are not read
__global__ __launch_bounds__(KV_WG) void kv_rec_count_kernel(const uint8_t* __restrict__ status, uint32_t n_res,
                                                              uint32_t tiles, uint32_t* __restrict__ counts,
                                                              unsigned long long* __restrict__ masks,
                                                              const uint8_t* __restrict__ sflag, uint32_t rule0) {
  __shared__ uint32_t s_w[KV_WG / 64];
  const uint32_t rule = rule0 + blockIdx.y;
  for (uint32_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    if (sflag && !sflag[(size_t)rule * tiles + t]) {  // (uniform: the whole workgroup skips)
      if (threadIdx.x == 0) counts[(size_t)rule * tiles + t] = 0u;
      if (masks && (threadIdx.x & 63) == 0) masks[(size_t)rule * tiles * (KV_WG / 64) + ((t * KV_WG + threadIdx.x) >> 6)] = 0ull;
      continue;
    }
    const uint32_t r = t * KV_WG + threadIdx.x;
    const bool f = r < n_res && has_record(status[(size_t)rule * n_res + r]);
    const uint64_t m = __ballot(f);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = (uint32_t)__popcll(m);
    // (caller-order fetch: every wave's record lanes, the ranks of the scatter below)
    if (masks && (threadIdx.x & 63) == 0) masks[(size_t)rule * tiles * (KV_WG / 64) + (r >> 6)] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t n = 0;
      for (int w = 0; w < KV_WG / 64; w++) n += s_w[w];
      counts[(size_t)rule * tiles + t] = n;
    }
    __syncthreads();
  }
}

// in place exclusive scan of counts[rule][0..tiles); totals[rule] = the rule's records
__global__ __launch_bounds__(KV_WG) void kv_rec_scan_kernel(uint32_t* __restrict__ counts, uint32_t tiles,
                                                             unsigned long long* __restrict__ totals) {
  __shared__ uint32_t s_v[KV_WG];
  uint32_t* c = counts + (size_t)blockIdx.x * tiles;
  uint32_t carry = 0;
  for (uint32_t b = 0; b < tiles; b += KV_WG) {
    const uint32_t i = b + threadIdx.x;
    const uint32_t v = i < tiles ? c[i] : 0u;
    s_v[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t o = 1; o < KV_WG; o <<= 1) {  // Hillis-Steele inclusive scan
      const uint32_t x = threadIdx.x >= o ? s_v[threadIdx.x - o] : 0u;
      __syncthreads();
      s_v[threadIdx.x] += x;
      __syncthreads();
    }
    if (i < tiles) c[i] = carry + s_v[threadIdx.x] - v;
    carry += s_v[KV_WG - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

// base[rule] = records of rules < rule; base[n_rules] = all records (one workgroup)
__global__ __launch_bounds__(KV_WG) void kv_rec_base_kernel(const unsigned long long* __restrict__ totals,
                                                             uint32_t n_rules, unsigned long long* __restrict__ base) {
  __shared__ unsigned long long s_v[KV_WG];
  unsigned long long carry = 0;
  for (uint32_t b = 0; b < n_rules; b += KV_WG) {
    const uint32_t i = b + threadIdx.x;
    const unsigned long long v = i < n_rules ? totals[i] : 0ull;
    s_v[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t o = 1; o < KV_WG; o <<= 1) {
      const unsigned long long x = threadIdx.x >= o ? s_v[threadIdx.x - o] : 0ull;
      __syncthreads();
      s_v[threadIdx.x] += x;
      __syncthreads();
    }
    if (i < n_rules) base[i] = carry + s_v[threadIdx.x] - v;
    carry += s_v[KV_WG - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) base[n_rules] = carry;
}

__global__ __launch_bounds__(KV_WG) void kv_rec_scatter_kernel(const uint8_t* __restrict__ status,
                                                                const ErrRec8* __restrict__ err8,
                                                                const ErrRec* __restrict__ errw, uint32_t n_res,
                                                                uint32_t tiles, const uint32_t* __restrict__ offs,
                                                                const unsigned long long* __restrict__ base,
                                                                ErrRec8* __restrict__ out8, ErrRec* __restrict__ outw,
                                                                uint32_t* __restrict__ wide,
                                                                const uint8_t* __restrict__ compact,
                                                                const uint32_t* __restrict__ order,
                                                                const unsigned long long* __restrict__ masks,
                                                                const uint8_t* __restrict__ sflag, uint32_t rule0) {
  __shared__ uint32_t s_w[KV_WG / 64];
  const uint32_t rule = rule0 + blockIdx.y, lane = threadIdx.x & 63;
  const bool cmp = compact && compact[rule];  // (rule is uniform: a scalar branch)
  const unsigned long long rb = base[rule];
  for (uint32_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    if (sflag && !sflag[(size_t)rule * tiles + t]) continue;  // (no records; uniform)
    const uint32_t r = t * KV_WG + threadIdx.x;
    const size_t o = (size_t)rule * n_res + r;
    const bool f = r < n_res && has_record(status[o]);
    const uint64_t m = __ballot(f);
    if (lane == 0) s_w[threadIdx.x >> 6] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0;  // records of the tile's earlier waves
    for (uint32_t w = 0; w < (threadIdx.x >> 6); w++) before += s_w[w];
    const unsigned long long tile0 = rb + offs[(size_t)rule * tiles + t] + before;
    // destination of the record of store slot s (rank `rk` among the wave's record lanes): the store
    // order, or with `order` the caller's (offs / base over the caller-order statuses, `masks` their
    // record lanes per wave: the rank of caller index j in its tile)
    auto dest = [&](uint32_t s, uint32_t rk) -> unsigned long long {
      if (!order) return tile0 + rk;
      const uint32_t j = order[s];
      const unsigned long long* mr = masks + (size_t)rule * tiles * (KV_WG / 64);
      uint32_t q = (uint32_t)__popcll(mr[j >> 6] & ((1ull << (j & 63u)) - 1ull));
      for (uint32_t w = (j >> 6) & ~3u; w < (j >> 6); w++) q += (uint32_t)__popcll(mr[w]);
      return rb + offs[(size_t)rule * tiles + (j >> 8)] + q;
    };
    if (cmp) {
      // slot `lane` of the wave's segment holds the wave's lane-th record written; its lane field
      // gives its rank among the wave's record lanes
      if (lane < (uint32_t)__popcll(m)) {
        const ErrRec8 e = err8[o];
        const uint32_t l = e.w1 >> 26;
        out8[dest((r & ~63u) + l, (uint32_t)__popcll(m & ((1ull << l) - 1ull)))] = e;
        if (e.w0 & ERR8_WIDE) atomicOr(wide, 1u);
      }
    } else if (f) {
      const unsigned long long idx = dest(r, (uint32_t)__popcll(m & ((1ull << lane) - 1ull)));
      const ErrRec8 e = err8[o];
      out8[idx] = e;
      if (outw) outw[idx] = errw[o];
      if (e.w0 & ERR8_WIDE) atomicOr(wide, 1u);
    }
    __syncthreads();
  }
}

// Record codes (fetch): the records of one rule take few distinct values once their lane field is
// dropped (the failing pattern node and the loop indices: C3's image globs fail at one of a Pod's
// few containers), so a rule's records cross PCIe as a 1-byte code per record into a per-rule table
// of KV_REC_CODES distinct records. Per record: its key (w0, w1 without the lane) is looked up in
// the rule's open-addressing table (keys in tkey, ~0: empty; a plain read first, a CAS only for a
// key not seen yet) and its slot written as the code; a rule whose table fills up is flagged raw
// (its records then cross whole, kv_rec_gather_kernel). Grid (x blocks, rules).
__global__ __launch_bounds__(KV_WG) void kv_rec_code_kernel(const ErrRec8* __restrict__ rec,
                                                             const unsigned long long* __restrict__ base,
                                                             unsigned long long* __restrict__ tkey,
                                                             uint8_t* __restrict__ code, uint32_t* __restrict__ raw,
                                                             uint32_t rule0) {
  const uint32_t rule = rule0 + blockIdx.y, lane = threadIdx.x & 63u;
  const unsigned long long b0 = base[rule], b1 = base[rule + 1];
  unsigned long long* T = tkey + (size_t)rule * KV_REC_CODES;
  // a wave takes 64 consecutive records; its distinct keys are probed once each, by the first lane
  // holding the key (a rule's records are few distinct values: one probe per lane would send every
  // wave's loads of the same slot to one L2 channel)
  for (unsigned long long w0 = b0 + (unsigned long long)blockIdx.x * KV_WG + (threadIdx.x & ~63u); w0 < b1;
       w0 += (unsigned long long)gridDim.x * KV_WG) {
    const unsigned long long i = w0 + lane;
    const bool act = i < b1;
    unsigned long long k = 0;
    if (act) {
      const ErrRec8 e = rec[i];
      k = (unsigned long long)e.w0 << 32 | (e.w1 & ERR8_IDX_MASK);
    }
    uint32_t slot = 0;
    unsigned long long pending = __ballot(act);
    while (pending) {
      const int lead = __ffsll((long long)pending) - 1;
      const unsigned long long lk = __shfl(k, lead);
      const bool mine = ((pending >> lane) & 1ull) && k == lk;
      const unsigned long long same = __ballot(mine);
      int h = -1;
      if (lane == (uint32_t)lead) {
        uint32_t x = (uint32_t)((lk * 0x9E3779B97F4A7C15ull) >> 56) & (KV_REC_CODES - 1u);
        for (uint32_t n = 0; n < KV_REC_CODES; n++, x = (x + 1u) & (KV_REC_CODES - 1u)) {
          unsigned long long t = __hip_atomic_load(T + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (t == ~0ull) t = atomicCAS(T + x, ~0ull, lk);  // (returns the old key: ~0 when this lane set it)
          if (t == ~0ull || t == lk) {
            h = (int)x;
            break;
          }
        }
        if (h < 0) raw[rule] = 1u;  // more than KV_REC_CODES distinct records: the rule crosses raw
      }
      h = __shfl(h, lead);
      if (mine) slot = (uint32_t)h;
      pending &= ~same;
    }
    if (act) code[i] = (uint8_t)slot;  // (a raw rule's codes are not read)
  }
}

// the records of the raw rules, rule by rule, to out[nbase[rule] ...)
__global__ __launch_bounds__(KV_WG) void kv_rec_gather_kernel(const ErrRec8* __restrict__ rec,
                                                               const unsigned long long* __restrict__ base,
                                                               const unsigned long long* __restrict__ nbase,
                                                               const uint32_t* __restrict__ raw, ErrRec8* __restrict__ out,
                                                               uint32_t rule0) {
  const uint32_t rule = rule0 + blockIdx.y;
  if (!raw[rule]) return;
  const unsigned long long b0 = base[rule], b1 = base[rule + 1], d = nbase[rule];
  for (unsigned long long i = b0 + (unsigned long long)blockIdx.x * KV_WG + threadIdx.x; i < b1;
       i += (unsigned long long)gridDim.x * KV_WG)
    out[d + (i - b0)] = rec[i];
}

constexpr uint32_t kMaxGridY = 65535u;

hipError_t launch_rec_codes(const ErrRec8* rec, const unsigned long long* base, uint32_t n_rules,
                            unsigned long long* tkey, uint8_t* code, uint32_t* raw, const unsigned long long* nbase,
                            ErrRec8* out, int phase, hipStream_t stream) {
  if (n_rules == 0) return hipSuccess;
  for (uint32_t q0 = 0; q0 < n_rules; q0 += kMaxGridY) {
    const dim3 grid(64, std::min(kMaxGridY, n_rules - q0));
    if (phase == 0)
      hipLaunchKernelGGL(kv_rec_code_kernel, grid, dim3(KV_WG), 0, stream, rec, base, tkey, code, raw, q0);
    else
      hipLaunchKernelGGL(kv_rec_gather_kernel, grid, dim3(KV_WG), 0, stream, rec, base, nbase, raw, out, q0);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Site records -> the members' ErrRec8 at their [rule][res] slots (kvdevtypes.h GSiteDesc): one
// wave per (group, wave of resources), lane k handles records k, k + 64, ... of the segment.
__global__ __launch_bounds__(KV_WG) void kv_gsite_expand_kernel(const uint4* __restrict__ gsite,
                                                                 const uint32_t* __restrict__ gcnt,
                                                                 const GSiteDesc* __restrict__ desc,
                                                                 const uint32_t* __restrict__ mem, uint32_t n_res,
                                                                 ErrRec8* __restrict__ err8, uint32_t g0) {
  const uint32_t nw = (n_res + 63u) >> 6, w = blockIdx.x * (KV_WG / 64) + (threadIdx.x >> 6), g = g0 + blockIdx.y;
  if (w >= nw) return;
  const GSiteDesc d = desc[g];
  const uint32_t cnt = gcnt[(size_t)g * nw + w];
  const uint4* seg = gsite + ((size_t)d.gpre * nw + (size_t)w * d.n) * 64u;
  for (uint32_t k = threadIdx.x & 63u; k < cnt; k += 64u) {
    const uint4 x = seg[k];  // {ekx, w1, member mask, indices do not fit}
    const uint32_t r = w * 64u + (x.y >> 26);
    for (uint32_t m = x.z; m; m &= m - 1u) {
      const uint32_t j = (uint32_t)__builtin_ctz(m);
      const uint32_t ri = mem[2u * (d.moff + j)];
      // the member's error: the representative's node shifted (ekx 0: no error node)
      const uint32_t pn = x.x ? (x.x >> 8) + mem[2u * (d.moff + j) + 1u] : 0u;
      const uint32_t wide = x.w | (pn >= (1u << 25) ? 1u : 0u);
      ErrRec8 e;
      e.w0 = (x.x & 15u) | (((x.x >> 4) & 15u) << 4) | (wide << 6) | (pn << 7);
      e.w1 = x.y;
      err8[(size_t)ri * n_res + r] = e;
    }
  }
}

hipError_t launch_gsite_expand(const uint32_t* gsite, const uint32_t* gcnt, const GSiteDesc* desc, const uint32_t* mem,
                               uint32_t n_groups, uint32_t n_res, ErrRec8* err8, hipStream_t stream) {
  if (n_res == 0 || n_groups == 0) return hipSuccess;
  const uint32_t nw = (n_res + 63u) >> 6;
  for (uint32_t g0 = 0; g0 < n_groups; g0 += kMaxGridY) {  // (grid y holds at most 65535 groups)
    hipLaunchKernelGGL(kv_gsite_expand_kernel, dim3((nw + KV_WG / 64 - 1) / (KV_WG / 64), std::min(kMaxGridY, n_groups - g0)),
                       dim3(KV_WG), 0, stream, (const uint4*)gsite, gcnt, desc, mem, n_res, err8, g0);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Status transfer form (kv_result materialises it on the host): the (rule, segment) status segments
// the pass wrote (DevOut::sflag), 4 bits a status (ST_* < 16), KV_RWG / 2 bytes a segment,
// rule-major in segment order. One workgroup per (chunk of KV_WG segments, rule): phase 0 counts
// the chunk's written segments into ccnt[rule][chunk], phase 1 packs them at cbase[rule][chunk]
// (the host's exclusive scan of ccnt, in segments).
__device__ __forceinline__ uint32_t kv_nib4(uint32_t x) {  // 4 status bytes -> 16 bits
  return (x & 0xFu) | ((x >> 4) & 0xF0u) | ((x >> 8) & 0xF00u) | ((x >> 12) & 0xF000u);
}

__global__ __launch_bounds__(KV_WG) void kv_status_pack_kernel(const uint8_t* __restrict__ status,
                                                                const uint8_t* __restrict__ sflag,
                                                                const unsigned long long* __restrict__ cbase,
                                                                uint32_t* __restrict__ ccnt, uint32_t n_res,
                                                                uint32_t nwg, uint32_t nch, uint8_t* __restrict__ out,
                                                                uint32_t rule0) {
  __shared__ uint32_t s_w[KV_WG / 64];
  __shared__ uint32_t s_list[KV_WG];
  const uint32_t rule = rule0 + blockIdx.y, g = blockIdx.x * KV_WG + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const bool f = g < nwg && sflag[(size_t)rule * nwg + g];
  const unsigned long long m = __ballot(f);
  if (lane == 0) s_w[w] = (uint32_t)__popcll(m);
  __syncthreads();
  uint32_t pre = (uint32_t)__popcll(m & ((1ull << lane) - 1ull)), cnt = 0;
  for (uint32_t k = 0; k < KV_WG / 64; k++) {
    if (k < w) pre += s_w[k];
    cnt += s_w[k];
  }
  if (!out) {
    if (threadIdx.x == 0) ccnt[(size_t)rule * nch + blockIdx.x] = cnt;
    return;
  }
  if (f) s_list[pre] = g;
  __syncthreads();
  const uint8_t* row = status + (size_t)rule * n_res;
  uint8_t* o = out + (size_t)cbase[(size_t)rule * nch + blockIdx.x] * (KV_RWG / 2);
  constexpr uint32_t TPS = KV_RWG / 8;  // threads per segment, 8 statuses each
  const uint32_t j = threadIdx.x % TPS;
  const bool al = (((size_t)rule * n_res) & 7u) == 0;
  for (uint32_t k = threadIdx.x / TPS; k < cnt; k += KV_WG / TPS) {
    const uint64_t q = (uint64_t)s_list[k] * KV_RWG + 8u * j;
    uint32_t v = 0;
    if (al && q + 8u <= n_res) {
      const uint2 x = *(const uint2*)(row + q);
      v = kv_nib4(x.x) | kv_nib4(x.y) << 16;
    } else {
      for (uint32_t t = 0; t < 8u; t++)
        if (q + t < n_res) v |= (uint32_t)(row[q + t] & 15u) << (4u * t);
    }
    *(uint32_t*)(o + (size_t)k * (KV_RWG / 2) + 4u * j) = v;
  }
}

hipError_t launch_status_pack(const uint8_t* status, const uint8_t* sflag, uint32_t n_res, uint32_t n_rules,
                              const unsigned long long* cbase, uint32_t* ccnt, uint8_t* out, hipStream_t stream) {
  if (n_res == 0 || n_rules == 0) return hipSuccess;
  const uint32_t nwg = (n_res + KV_RWG - 1) / KV_RWG, nch = (nwg + KV_WG - 1) / KV_WG;
  for (uint32_t q0 = 0; q0 < n_rules; q0 += kMaxGridY) {
    hipLaunchKernelGGL(kv_status_pack_kernel, dim3(nch, std::min(kMaxGridY, n_rules - q0)), dim3(KV_WG), 0, stream,
                       status, sflag, cbase, ccnt, n_res, nwg, nch, out, q0);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  }
  return hipSuccess;
}


hipError_t launch_rec_compact(const uint8_t* status, const ErrRec8* err8, const ErrRec* errw, uint32_t n_res,
                              uint32_t n_rules, uint32_t* offs, unsigned long long* totals, unsigned long long* base,
                              ErrRec8* out8, ErrRec* outw, uint32_t* wide, int phase, const uint8_t* compact,
                              const uint32_t* order, unsigned long long* masks, const uint8_t* sflag,
                              hipStream_t stream) {
  if (n_res == 0 || n_rules == 0) return hipSuccess;
  const uint32_t tiles = (n_res + KV_WG - 1) / KV_WG;
  // about 65 536 workgroups in all, each walking its rule's tiles (C3: 16 384 in all left the
  // scatter latency-bound at 6 ms, 9.6 M dispatch-bound at 8.4 ms)
  const uint32_t gx = std::max(1u, std::min(tiles, 65536u / n_rules));
  for (uint32_t q0 = 0; q0 < n_rules; q0 += kMaxGridY) {
    const dim3 grid(gx, std::min(kMaxGridY, n_rules - q0));
    if (phase == 0)  // offsets (the scan and bases below)
      hipLaunchKernelGGL(kv_rec_count_kernel, grid, dim3(KV_WG), 0, stream, status, n_res, tiles, offs, masks, sflag, q0);
    else
      hipLaunchKernelGGL(kv_rec_scatter_kernel, grid, dim3(KV_WG), 0, stream, status, err8, errw, n_res, tiles, offs,
                         base, out8, outw, wide, compact, order, masks, sflag, q0);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  }
  if (phase == 0) {
    hipLaunchKernelGGL(kv_rec_scan_kernel, dim3(n_rules), dim3(KV_WG), 0, stream, offs, tiles, totals);
    hipLaunchKernelGGL(kv_rec_base_kernel, dim3(1), dim3(KV_WG), 0, stream, totals, n_rules, base);
  }
  return hipGetLastError();
}

}  // namespace kv

// ---------------------------------------------------------------------------
// Per-scope PolicyReport counts: counts[scope][rule][KV_HIST] from status[rule][res]
// and the namespace index of every resource (scope = namespace, "" = cluster
// scope), the summaries of pkg/kyverno/apply/report.go:76-179 and
// pkg/policyreport/builder.go:245-308. One workgroup per (rule, chunk of
// KV_SCOPE_CHUNK resources): coalesced 4-byte status / 16-byte scope loads,
// LDS histogram over all scopes when it fits (<= KV_SCOPE_LDS scopes), then one
// global atomic per non-zero (scope, status) of the chunk. HBM-bound: reads
// n_rules x n_res status bytes (+ the scope array once per rule, L2/MALL hits).
namespace kv {

__global__ __launch_bounds__(KV_WG) void kv_scope_count_kernel(const uint8_t* __restrict__ status,
                                                                const uint32_t* __restrict__ scope, uint32_t n_res,
                                                                uint32_t n_rules, uint32_t n_scopes,
                                                                unsigned long long* __restrict__ out) {
  extern __shared__ uint32_t s_cnt[];
  const uint32_t rule = blockIdx.x % n_rules;
  const uint32_t chunk = blockIdx.x / n_rules;
  const bool in_lds = n_scopes <= KV_SCOPE_LDS;
  if (in_lds)
    for (uint32_t q = threadIdx.x; q < n_scopes * KV_HIST; q += KV_WG) s_cnt[q] = 0;
  __syncthreads();
  const uint64_t row = (uint64_t)rule * n_res;
  const uint32_t base = chunk * KV_SCOPE_CHUNK;
  const uint32_t end = min(base + KV_SCOPE_CHUNK, n_res);
  for (uint32_t i = base + threadIdx.x * 4; i < end; i += KV_WG * 4) {
    uint32_t sc[4];
    uint32_t st[4];
    if (i + 4 <= end) {
      const uint4 s4 = *(const uint4*)(scope + i);  // base and i are multiples of 4
      sc[0] = s4.x; sc[1] = s4.y; sc[2] = s4.z; sc[3] = s4.w;
#pragma unroll
      for (int k = 0; k < 4; k++) st[k] = status[row + i + k];
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        sc[k] = i + k < end ? scope[i + k] : 0xFFFFFFFFu;
        st[k] = i + k < end ? status[row + i + k] : 0;
      }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (sc[k] >= n_scopes || st[k] >= KV_HIST) continue;
      if (in_lds) atomicAdd(&s_cnt[sc[k] * KV_HIST + st[k]], 1u);
      else atomicAdd(&out[((uint64_t)sc[k] * n_rules + rule) * KV_HIST + st[k]], 1ull);
    }
  }
  if (!in_lds) return;
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < n_scopes * KV_HIST; q += KV_WG) {
    const uint32_t v = s_cnt[q];
    if (v) atomicAdd(&out[((uint64_t)(q / KV_HIST) * n_rules + rule) * KV_HIST + q % KV_HIST], (unsigned long long)v);
  }
}

hipError_t launch_scope_counts(const uint8_t* status, const uint32_t* scope, uint32_t n_res, uint32_t n_rules,
                               uint32_t n_scopes, unsigned long long* out, hipStream_t stream) {
  if (n_res == 0 || n_rules == 0 || n_scopes == 0) return hipSuccess;
  const uint32_t chunks = (n_res + KV_SCOPE_CHUNK - 1) / KV_SCOPE_CHUNK;
  const size_t shm = n_scopes <= KV_SCOPE_LDS ? (size_t)n_scopes * KV_HIST * sizeof(uint32_t) : 0;
  hipLaunchKernelGGL(kv_scope_count_kernel, dim3(chunks * n_rules), dim3(KV_WG), shm, stream, status, scope, n_res,
                     n_rules, n_scopes, out);
  return hipGetLastError();
}

// counts[rule][k] = sum over scopes of scounts[scope][rule][k]: the per-rule histogram of a
// SCOPES pass of the specialized kernels, which add to the per-scope counts only
// (kvdevfn.h kv_end_flush); one thread per (rule, status), coalesced over the scopes' rows
__global__ __launch_bounds__(KV_WG) void kv_scope_totals_kernel(const unsigned long long* __restrict__ sc,
                                                                uint32_t n_scopes, uint32_t n,
                                                                unsigned long long* __restrict__ counts) {
  const uint32_t i = blockIdx.x * KV_WG + threadIdx.x;
  if (i >= n) return;
  unsigned long long t = 0ull;
  for (uint32_t s = 0; s < n_scopes; s++) t += sc[(size_t)s * n + i];
  counts[i] = t;
}

hipError_t launch_scope_totals(const unsigned long long* scounts, uint32_t n_scopes, uint32_t n_rules,
                               unsigned long long* counts, hipStream_t stream) {
  const uint32_t n = n_rules * (uint32_t)KV_HIST;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(kv_scope_totals_kernel, dim3((n + KV_WG - 1) / KV_WG), dim3(KV_WG), 0, stream, scounts, n_scopes,
                     n, counts);
  return hipGetLastError();
}

// One wave per row of the wave-group layout: lane l takes its packed cell (its units start at
// the row's first unit + the set mask bits below l + the wide-mask bits below l) rebuilt into a
// Node (kv_layout.h cell_widen: a scalar's string form from its Val), or the zero cell. Reads the
// units and masks once, writes every cell once (coalesced 1 KB per row).
__global__ __launch_bounds__(KV_WG) void kv_expand_rows_kernel(const uint64_t* __restrict__ tcells,
                                                               const uint64_t* __restrict__ rmask,
                                                               const uint64_t* __restrict__ rwide,
                                                               const uint32_t* __restrict__ roff,
                                                               const Val* __restrict__ vals, uint64_t n_rows,
                                                               Node* __restrict__ nodes) {
  const uint64_t row = (uint64_t)blockIdx.x * (KV_WG / KV_LANES) + threadIdx.x / KV_LANES;
  if (row >= n_rows) return;
  const uint32_t lane = threadIdx.x & (KV_LANES - 1);
  const uint64_t m = rmask[row], below = (1ull << lane) - 1ull;
  Node v{0u, 0u, 0u, 0u};
  if ((m >> lane) & 1ull) {
    const uint64_t w = rwide[row];
    const uint64_t* u = tcells + roff[row] + (uint32_t)__popcll(m & below) + (uint32_t)__popcll(w & below);
    const uint64_t x = u[0];
    if ((w >> lane) & 1ull) {
      const uint64_t y = u[1];
      v = Node{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32)};
    } else {
      v = cell_widen((uint32_t)x, (uint32_t)(x >> 32), row, vals);
    }
  }
  nodes[row * KV_LANES + lane] = v;
}

hipError_t launch_expand_rows(const uint64_t* tcells, const uint64_t* rmask, const uint64_t* rwide, const uint32_t* roff,
                              const Val* vals, uint64_t n_rows, Node* nodes, hipStream_t stream) {
  if (n_rows == 0) return hipSuccess;
  const uint64_t blocks = (n_rows + KV_WG / KV_LANES - 1) / (KV_WG / KV_LANES);
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kv_expand_rows_kernel, dim3((uint32_t)blocks), dim3(KV_WG), 0, stream, tcells, rmask, rwide, roff,
                     vals, n_rows, nodes);
  return hipGetLastError();
}

// ------------------------------------------------------------------ path columns (kvcol.h)
// element rows of family f = 1 + blockIdx.y per wave group: the most any lane of the group needs
__global__ __launch_bounds__(KV_WG) void kv_pcol_rows_kernel(const DevBatch* __restrict__ Bp,
                                                             const ColDesc* __restrict__ cols,
                                                             const ColFam* __restrict__ fams) {
  const uint32_t r = blockIdx.x * KV_WG + threadIdx.x, f = 1u + blockIdx.y;
  uint32_t v = col_rows(*Bp, cols, fams, f, r);
#pragma unroll
  for (int m = 1; m < (int)KV_LANES; m <<= 1) v = max(v, (uint32_t)__shfl_xor((int)v, m, (int)KV_LANES));
  if ((threadIdx.x & (KV_LANES - 1)) == 0) fams[f].erow[r >> 6] = v;
}

// exclusive prefix of each family's per-group element rows (one workgroup per family; its
// total lands at erow[n_groups])
__global__ __launch_bounds__(1024) void kv_pcol_scan_kernel(const ColFam* __restrict__ fams, uint32_t n_groups) {
  __shared__ uint32_t s_sum[1024];
  uint32_t* __restrict__ e = fams[1u + blockIdx.x].erow;
  const uint32_t per = (n_groups + 1023u) / 1024u, a = threadIdx.x * per, b = min(a + per, n_groups);
  uint32_t t = 0;
  for (uint32_t i = a; i < b; i++) t += e[i];
  s_sum[threadIdx.x] = t;
  __syncthreads();
  for (uint32_t o = 1; o < 1024u; o <<= 1) {  // inclusive scan of the chunk sums
    const uint32_t x = threadIdx.x >= o ? s_sum[threadIdx.x - o] : 0u;
    __syncthreads();
    s_sum[threadIdx.x] += x;
    __syncthreads();
  }
  uint32_t run = s_sum[threadIdx.x] - t;
  for (uint32_t i = a; i < b; i++) {
    const uint32_t c = e[i];
    e[i] = run;
    run += c;
  }
  if (threadIdx.x == 1023u) e[n_groups] = s_sum[1023];
}

// cells of columns [c0, c0 + gridDim.y) for every lane (family-0 columns, or element columns
// after them: their family arrays' cells must be built)
__global__ __launch_bounds__(KV_WG) void kv_pcol_build_kernel(const DevBatch* __restrict__ Bp,
                                                              const ColDesc* __restrict__ cols,
                                                              const ColFam* __restrict__ fams, uint32_t j0,
                                                              uint32_t c0, uint32_t elem, uint32_t* __restrict__ pool, uint64_t cells) {
  const uint32_t r = blockIdx.x * KV_WG + threadIdx.x, c = c0 + blockIdx.y;
  if (elem) col_build_elem(*Bp, cols, fams, j0, c, r, pool, cells);
  else col_build_root(*Bp, cols, fams, j0, c, r, pool, cells);
}

hipError_t launch_pcol_rows(const DevBatch* B, const ColDesc* cols, const ColFam* fams, uint32_t n_fam,
                            uint32_t n_groups, hipStream_t stream) {
  if (n_fam < 2 || n_groups == 0) return hipSuccess;
  hipLaunchKernelGGL(kv_pcol_rows_kernel, dim3(n_groups * KV_LANES / KV_WG, n_fam - 1), dim3(KV_WG), 0, stream, B, cols,
                     fams);
  if (hipError_t e = hipGetLastError()) return e;
  hipLaunchKernelGGL(kv_pcol_scan_kernel, dim3(n_fam - 1), dim3(1024), 0, stream, fams, n_groups);
  return hipGetLastError();
}

hipError_t launch_pcol_build(const DevBatch* B, const ColDesc* cols, const ColFam* fams, uint32_t j0, uint32_t c0,
                             uint32_t n, uint32_t n_groups, bool elem, uint32_t* pool, uint64_t cells,
                             hipStream_t stream) {
  if (n == 0 || n_groups == 0) return hipSuccess;
  if (n > 65535u) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kv_pcol_build_kernel, dim3(n_groups * KV_LANES / KV_WG, n), dim3(KV_WG), 0, stream, B, cols, fams,
                     j0, c0, elem ? 1u : 0u, pool, cells);
  return hipGetLastError();
}

}  // namespace kv
