// Residency census: how many waves of a kernel with a given VGPR / SGPR / LDS footprint the hardware
// keeps resident per SIMD at once.  Each wave spins ~20 us (s_memrealtime) and records its start, end
// and HW_ID | XCC_ID; the host counts the maximum overlap per SIMD.  The forward k_query_fwd_parts
// (168 VGPRs, 106 SGPRs, 5952 B LDS, 256-thread blocks) was measured at 2 waves per SIMD where the
// VGPR table says 3 (tools/probes/wave_timeline.py); this separates the candidate causes.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/census.hip -o tools/probes/census
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

// the footprints are forced with inline asm that names the highest register
#define KERNEL_VS(NAME, VREG, SREG, LDSB)                                                         \
  __global__ __launch_bounds__(256) void NAME(unsigned long long* out, int ticks) {              \
    __shared__ float lds[(LDSB) > 0 ? (LDSB) / 4 : 1];                                            \
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();                               \
    asm volatile("v_mov_b32 " VREG ", 0\n s_mov_b32 " SREG ", 0" ::: VREG, SREG);                \
    if ((LDSB) > 0) lds[threadIdx.x % ((LDSB) > 0 ? (LDSB) / 4 : 1)] = (float)t0;                 \
    unsigned long long t = t0;                                                                     \
    while (t - t0 < (unsigned long long)ticks) {                                                   \
      __builtin_amdgcn_s_sleep(8);                                                                 \
      t = __builtin_amdgcn_s_memrealtime();                                                        \
    }                                                                                              \
    if ((threadIdx.x & 63) == 0) {                                                                 \
      const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);                                \
      out[w * 3 + 0] = t0;                                                                         \
      out[w * 3 + 1] = t;                                                                          \
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);                               \
      const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);                             \
      out[w * 3 + 2] = (unsigned long long)hw | ((unsigned long long)(xcc & 15) << 32);           \
    }                                                                                              \
    if ((LDSB) > 0 && lds[(threadIdx.x + 1) % ((LDSB) > 0 ? (LDSB) / 4 : 1)] == -1.f) out[0] = 0; \
  }

KERNEL_VS(k_v168_s100_l5952, "v167", "s99", 5952)
KERNEL_VS(k_v168_s16_l0, "v167", "s15", 0)
KERNEL_VS(k_v168_s100_l0, "v167", "s99", 0)
KERNEL_VS(k_v168_s16_l5952, "v167", "s15", 5952)
KERNEL_VS(k_v128_s100_l5952, "v127", "s99", 5952)
KERNEL_VS(k_v104_s100_l8192, "v103", "s99", 8192)
KERNEL_VS(k_v160_s100_l5952, "v159", "s99", 5952)

typedef void (*kfn)(unsigned long long*, int);

static void census(const char* name, kfn k, unsigned long long* d, std::vector<unsigned long long>& h, int blocks,
                   int ticks = 2000) {
  hipMemset(d, 0, (size_t)blocks * 4 * 3 * 8);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, ticks);
  hipDeviceSynchronize();
  hipMemcpy(h.data(), d, (size_t)blocks * 4 * 3 * 8, hipMemcpyDeviceToHost);
  std::map<unsigned long long, std::vector<std::pair<unsigned long long, int>>> ev;
  for (int w = 0; w < blocks * 4; ++w) {
    const unsigned long long hw = h[w * 3 + 2];
    const unsigned long long simd = ((hw >> 4) & 3) | (((hw >> 8) & 15) << 2) | (((hw >> 12) & 1) << 6) |
                                    (((hw >> 13) & 7) << 7) | (((hw >> 32) & 15) << 10);
    ev[simd].push_back({h[w * 3 + 0], 1});
    ev[simd].push_back({h[w * 3 + 1], -1});
  }
  std::map<int, int> hist;
  for (auto& kv : ev) {
    auto& v = kv.second;
    std::sort(v.begin(), v.end(), [](auto a, auto b) { return a.first != b.first ? a.first < b.first : a.second < b.second; });
    int c = 0, m = 0;
    for (auto& e : v) {
      c += e.second;
      m = std::max(m, c);
    }
    hist[m]++;
  }
  printf("%-22s %5d WGs  SIMDs %zu  max resident per SIMD:", name, blocks, ev.size());
  for (auto& kv : hist) printf(" %d:%d", kv.first, kv.second);
  printf("\n");
}

int main() {
  const int blocks = 256 * 8;  // 8 workgroups of 4 waves per CU: 8 waves per SIMD offered
  unsigned long long* d;
  hipMalloc(&d, (size_t)blocks * 4 * 3 * 8);
  std::vector<unsigned long long> h((size_t)blocks * 4 * 3);
  census("v168 s100 lds5952", k_v168_s100_l5952, d, h, blocks);
  census("v168 s16 lds0", k_v168_s16_l0, d, h, blocks);
  census("v168 s100 lds0", k_v168_s100_l0, d, h, blocks);
  census("v168 s16 lds5952", k_v168_s16_l5952, d, h, blocks);
  census("v160 s100 lds5952", k_v160_s100_l5952, d, h, blocks);
  census("v128 s100 lds5952", k_v128_s100_l5952, d, h, blocks);
  census("v104 s100 lds8192", k_v104_s100_l8192, d, h, blocks);
  // partial grids (the forward's room0 launch: 750 workgroups, 2.93 per CU), 40 us waves
  for (int b : {750, 768, 512, 1024}) census("v168 s100 lds5952", k_v168_s100_l5952, d, h, b, 4000);
  for (int b : {750, 1000}) census("v128 s100 lds5952", k_v128_s100_l5952, d, h, b, 4000);
  hipFree(d);
  return 0;
}
