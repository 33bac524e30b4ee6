// Specialized kernels: the compiled policy set (bytecode, predicates, globs) is
// lowered once more, to HIP C++ with every rule as straight-line device code
// (constants as immediates, cursors in registers, per-lane control flow done by
// the hardware exec mask instead of the interpreter's uniform-pc emulation),
// and compiled for gfx950 with hiprtc when the policy set is compiled.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "kvinternal.hpp"
#include "kvdevtypes.h"

namespace kvh {

struct JitChunk {
  std::vector<uint32_t> rules;  // the rules evaluated by kernel `name`
  std::string name;
};

// One specialized rule kernel: rules [first, first + count) of the signature-sorted
// rule order as consecutive fused blocks of `blocks[i]` rules (sum = count), compiled with
// a `waves`-per-SIMD launch bound (0: none). Every array a block's rules walk is walked
// once per resource and block; the rules of a block keep their state in registers across
// the whole block, so the block sizes bound the kernel's register use.
struct JitKernelPlan {
  uint32_t first, count;
  int waves;
  std::vector<uint32_t> blocks;
};

struct JitImage {
  std::vector<JitKernelPlan> plan;     // kernel grouping (empty: default groups; kept across re-plans)
  std::vector<uint32_t> kernel_scratch;  // private segment bytes per lane of each planned kernel
  std::string source;       // generated HIP source, all of it (diagnostics, tools/kvemu)
  std::string common;       // prelude + helper functions shared by the kernels
  std::vector<std::string> kernel_name, kernel_src;  // one hiprtc program per kernel: common + kernel_src[i]
  std::vector<std::vector<char>> codes;              // gfx950 code object per kernel program
  uint32_t cache_hits = 0;  // programs loaded from the code-object cache
  std::vector<JitChunk> chunks;
  // leaf predicates memoized per distinct scalar value: slot k = memo_preds[k];
  // kernel "kvj_ptab" fills DevPS::ptab (memo_words words per value)
  std::vector<uint32_t> memo_preds;
  uint32_t memo_words = 0;
  uint32_t ptab_row = 1;    // predicates per kvj_ptab grid row (one row: every predicate of a value)
  // match bits per tuple (kv_mtup_kernel, DevPS::mtup): words of 32 rules in kernel order,
  // from the factored-match descriptors (DevPS::fac_*, kvjit.cpp build_fac)
  uint32_t mtup_words = 0;
  std::vector<uint32_t> fac_word, fac_bit, fac_flist, fac_rule;
  uint32_t fac_slots = 0;
  // per rule: 1 = its records are appended to its wave's 64-slot segment (lane in the record),
  // 0 = at the resource's slot (members of large rule groups, kvjit.cpp gslot_members; members of
  // groups with site records, expanded there at fetch)
  std::vector<uint8_t> rec_compact;
  // site-record groups (kvdevtypes.h GSiteDesc): 4 words per group, (rule, node shift) per member,
  // members in all
  std::vector<uint32_t> gs_desc, gs_mem;
  uint32_t gs_members = 0;
  // path columns the kernels read (kvdevtypes.h ColDesc, built per batch by kvcol.h): every
  // column; per family its array's column in family 0 and its column count
  std::vector<kv::ColDesc> cols;
  std::vector<uint32_t> fam_arr, fam_ncols;
  bool probe = false;      // a block-probe image (jit_refine_blocks): rule kernels only
  double gen_ms = 0, compile_ms = 0;
  // Output-mode variants (jit_compile_variants): the final plan's rule kernels compiled once more
  // per DevOut::full value the benchmarks and callers run most (KVJ_FULL a constant), so a kernel
  // carries no code for outputs its launches never write. codes[i] is program i's variant; empty
  // where the program is not a rule kernel or its variant spilled (the generic code runs there).
  struct Variant {
    uint32_t full = 0;
    std::vector<std::vector<char>> codes;
  };
  std::vector<Variant> variants;
};

// Generate the specialized source for every rule of `ps` (chunks of at most
// `chunk_rules` rules per kernel).
// most rules per kernel (one fused block): KVGPU_JIT_CHUNK, default 128
uint32_t jit_chunk_rules();
// diagnostics (KVGPU_JIT_STAMPS): stamps per wave of the rule kernels' segment boundaries
constexpr uint32_t kJitStamps = 16;
void jit_generate(const PolicySet& ps, uint32_t chunk_rules, JitImage* out);
// Compile every kernel program with hiprtc for gfx950, on parallel host threads
// (KVGPU_JIT_THREADS, default: hardware threads), through the code-object cache
// (KVGPU_JIT_CACHE directory, default $XDG_CACHE_HOME/kvgpu or ~/.cache/kvgpu;
// "0" disables; entries keyed by a hash of compiler options + program text).
// Throws std::runtime_error with the log on failure.
void jit_compile(JitImage* img);
uint64_t code_bytes(const JitImage& img);
// Register budget of the plan: no kernel ships with a private (scratch) segment, and a wave
// bound is kept only when the compiler met it. A multi-block kernel that spills (or exceeds the
// registers) under a bound of w > 6 waves per SIMD is recompiled at w - 1; otherwise its
// largest block is split in two; a kernel of one-rule blocks is compiled at w - 1, then
// without a bound (a one-rule kernel that still spills: std::runtime_error).
// Returns true when the plan changed (regenerate + compile again; the kernels that did not
// change come from the code-object cache).
bool jit_plan_spills(JitImage* img);
// The output-mode variants of the final plan (JitImage::variants): FULL (status + records, DevOut::
// full 3) and SCOPES-only (per-scope counts, 8); through the code-object cache.
void jit_compile_variants(JitImage* img);
// Block sizes of the plan from probe compiles: every multi-rule block of a multi-block kernel
// is compiled alone under its kernel's bound, and the blocks that spill or exceed the bound's
// registers are split in two, until every probe meets its bound (then regenerate the image).
void jit_refine_blocks(const PolicySet& ps, uint32_t chunk_rules, JitImage* img);
// Plan cache (in the code-object cache directory): the final kernel plan of a policy set,
// keyed by a hash of its first generated image (jit_plan_key), so a later compile of the
// same set goes straight to its final kernels (plan-<key>.txt, which also lists their
// code-object files).
std::string jit_plan_key(const JitImage& img);
bool jit_load_plan(const std::string& key, JitImage* img);
void jit_save_plan(const std::string& key, const JitImage& img);
bool co_kernel_info(const std::vector<char>& co, const std::string& name, uint32_t* private_seg, uint64_t* code,
                    uint32_t* vgprs = nullptr);
// SGPRs the compiler spilled into VGPR lanes (AMDGPU metadata .sgpr_spill_count)
uint32_t co_sgpr_spills(const std::vector<char>& co);

}  // namespace kvh
