// Residency probe: how many 1-wave workgroups (64 threads) a CU holds at once, with LDS per
// workgroup `lds` bytes and a launch bound of `w` waves per SIMD. Each workgroup adds one to a
// global counter, records the maximum it saw, waits ~20 us (bounded), and leaves.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int LDS, int T>
__global__ __launch_bounds__(T) void probe(unsigned* active, unsigned* peak) {
  __shared__ unsigned s[LDS / 4];
  if (threadIdx.x == 0) {
    s[0] = 1u;
    unsigned a = atomicAdd(active, 1u) + 1u;
    atomicMax(peak, a);
    const long long t0 = clock64();
    while (clock64() - t0 < 400000) __builtin_amdgcn_s_sleep(2);
    atomicSub(active, s[0]);
  }
}

template <int LDS, int T = 64>
void run(const char* tag) {
  unsigned *a, *p;
  hipMalloc(&a, 4); hipMalloc(&p, 4);
  hipMemset(a, 0, 4); hipMemset(p, 0, 4);
  hipLaunchKernelGGL((probe<LDS, T>), dim3(256 * 64), dim3(T), 0, 0, a, p);
  hipDeviceSynchronize();
  unsigned h = 0;
  hipMemcpy(&h, p, 4, hipMemcpyDeviceToHost);
  printf("%s lds=%d threads=%d: peak resident workgroups %u = %.2f per CU\n", tag, LDS, T, h, h / 256.0);
  hipFree(a); hipFree(p);
}

int main() {
  run<256>("tiny");
  run<4096>("4k");
  run<5120>("5k");
  run<6144>("6k");
  run<6656>("c2-like");
  run<6912>("c5-like");
  run<8192>("8k");
  run<26112, 256>("c2-now");
  run<27392, 256>("c5-now");
  return 0;
}
