// kvemu: host (x86) execution of the generated gfx950 kernel source, for
// debugging and sanitizer runs only (test infrastructure, never the product
// path: libkvgpu has no CPU evaluation). The generated source (kvjit.cpp,
// dumped with KVGPU_JIT_DUMP) is compiled by g++/clang++ with this header
// force-included; every lane of every workgroup then runs the kernel body on
// its own, one after the other (tools/kvemu/driver.cpp). Cross-lane parts
// (wave ballots of the per-rule histogram, the LDS histogram) are not
// emulated: statuses and error records are exact, counts are not.
#pragma once
#include <stdint.h>
#include <string.h>

#define KVEMU 1  // host emulation: no AMDGPU inline asm (kvdevfn.h)
#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __noinline__ __attribute__((noinline))
#define __shared__ static thread_local
#define __launch_bounds__(...)
#define __restrict__ __restrict
#define KV_SCONST

struct kvemu_dim3 {
  uint32_t x, y, z;
};
extern thread_local kvemu_dim3 threadIdx, blockIdx, gridDim;

struct uint2 {
  uint32_t x, y;
};
struct uint4 {
  uint32_t x, y, z, w;
};
static inline uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return uint4{a, b, c, d}; }

static inline void __syncthreads() {}
static inline uint64_t __ballot(bool p) { return p ? (1ull << (threadIdx.x & 63)) : 0ull; }
static inline int __popcll(uint64_t v) { return __builtin_popcountll(v); }
static inline int __popc(uint32_t v) { return __builtin_popcount(v); }
static inline uint32_t __shfl_xor(uint32_t v, int, int) { return v; }
static inline uint32_t atomicAdd(uint32_t* p, uint32_t v) {
  uint32_t o = *p;
  *p += v;
  return o;
}
static inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) {
  unsigned long long o = *p;
  *p += v;
  return o;
}
static inline double __longlong_as_double(long long v) {
  double d;
  memcpy(&d, &v, 8);
  return d;
}
static inline uint32_t kvemu_readfirstlane(uint32_t v) { return v; }
// v_alignbyte_b32: ({hi, lo} >> (8 * (sh & 3)))[31:0]
static inline uint32_t kvemu_alignbyte(uint32_t hi, uint32_t lo, uint32_t sh) {
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (sh & 3)));
}
// v_perm_b32: byte i of the result = byte sel[i] of {s0 (bytes 4-7), s1 (bytes 0-3)}; 0x0c -> 0x00, >= 0x0d -> 0xff
static inline uint32_t kvemu_perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  const uint64_t v = ((uint64_t)s0 << 32) | s1;
  uint32_t r = 0;
  for (int i = 0; i < 4; i++) {
    const uint32_t b = (sel >> (8 * i)) & 0xFF;
    const uint32_t x = b < 8 ? (uint32_t)(v >> (8 * b)) & 0xFF : b == 0x0c ? 0u : 0xFFu;
    r |= x << (8 * i);
  }
  return r;
}
#define __builtin_amdgcn_perm(s0, s1, sel) kvemu_perm(s0, s1, sel)
#define __builtin_amdgcn_readfirstlane(v) kvemu_readfirstlane(v)
#define __builtin_amdgcn_alignbyte(hi, lo, sh) kvemu_alignbyte(hi, lo, sh)
