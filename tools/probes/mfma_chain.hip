// Micro-benchmark: issue rate of v_mfma_f32_32x32x2_f32 on ONE accumulator (each MFMA's C is the
// previous one's D, as in the decoders' GEMM chains) vs 2 and 4 independent accumulators, at 1..4
// waves per SIMD.  hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_chain.hip -o tools/probes/mfma_chain
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(64) void k_chain(float* out, int iters, float a0, float b0) {
  f32x16 acc[NACC];
#pragma unroll
  for (int k = 0; k < NACC; ++k)
    for (int r = 0; r < 16; ++r) acc[k][r] = 0.f;
  float a = a0 + threadIdx.x * 1e-7f, b = b0;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int s = 0; s < 16; s += NACC) {
#pragma unroll
      for (int k = 0; k < NACC; ++k) acc[k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[k], 0, 0, 0);
    }
  }
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < NACC; ++k)
    for (int r = 0; r < 16; ++r) t += acc[k][r];
  out[blockIdx.x * 64 + threadIdx.x] = t;
}

template <int NACC>
double run(float* out, int waves_per_simd, int iters) {
  const int blocks = 1024 * waves_per_simd;  // 256 CUs x 4 SIMDs
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k_chain<NACC><<<blocks, 64>>>(out, iters, 1e-3f, 1e-3f);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) k_chain<NACC><<<blocks, 64>>>(out, iters, 1e-3f, 1e-3f);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flop = 5.0 * blocks * (double)iters * 16 * 32 * 32 * 2 * 2;
  return flop / (ms * 1e-3) / 1e12;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 4096 * 64 * sizeof(float));
  const int iters = 2048;
  for (int w = 1; w <= 4; ++w)
    printf("waves/SIMD %d: 1 acc %.1f TF/s, 2 acc %.1f, 4 acc %.1f (fp32 peak 157.3)\n", w, run<1>(out, w, iters),
           run<2>(out, w, iters), run<4>(out, w, iters));
  (void)hipFree(out);
  return 0;
}
