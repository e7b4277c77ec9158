// nslam_composite.hip — volume compositing (occupancy mode) on gfx950 and its backward.
//
// Replaces raw2outputs_nerf_color (src/common.py:204-245) with occupancy=True
// (configs/nice_slam.yaml:5) and its autograd backward:
//   alpha_k = sigmoid(10 raw_k[3]);  T_k = prod_{j<k} (1 - alpha_j + 1e-10);  w_k = alpha_k T_k
//   rgb = sum_k w_k raw_k[:3] (f32);  depth = sum_k w_k z_k (f64);  var = sum_k w_k (z_k-depth)^2 (f64)
// One wave per ray, one lane per sample; the transmittance is a wave prefix product and the sums
// are wave shuffle reductions.  Rays with more than 64 samples are processed in 64-sample chunks
// with a carried transmittance.
#include "nslam_dev.h"

namespace {

constexpr int kMaxS = 256;  // 4 chunks

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}
__device__ __forceinline__ double wave_sumd(double v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}
// inclusive prefix product over lanes
__device__ __forceinline__ float wave_prefix_prod(float v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const float o = __shfl_up(v, d, 64);
    if (lane >= d) v *= o;
  }
  return v;
}
// inclusive suffix sum over lanes
__device__ __forceinline__ float wave_suffix_sum(float v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const float o = __shfl_down(v, d, 64);
    if (lane + d < 64) v += o;
  }
  return v;
}

__device__ __forceinline__ float sigmoid10(float occ) {
  const float x = 10.f * occ;  // torch: 10*raw[..., -1] then sigmoid
  return 1.f / (1.f + expf(-x));
}

struct RaySample {
  float a, f, T, w;
  f32x4 raw;
  double z;
};

// Fill chunk `c` of a ray: alpha, factor, exclusive transmittance, weight.  carry = T entering.
__device__ __forceinline__ RaySample load_sample(const float* raw, const double* z, int S, int k, int lane,
                                                 float& carry) {
  RaySample s;
  const bool act = k < S;
  s.raw = act ? *reinterpret_cast<const f32x4*>(raw + (size_t)k * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
  s.z = act ? z[k] : 0.0;
  s.a = act ? sigmoid10(s.raw[3]) : 0.f;
  s.f = act ? (1.f - s.a) + 1e-10f : 1.f;
  const float incl = wave_prefix_prod(s.f, lane);
  float excl = __shfl_up(incl, 1, 64);
  if (lane == 0) excl = 1.f;
  s.T = carry * excl;
  s.w = s.a * s.T;
  carry = carry * __shfl(incl, 63, 64);
  return s;
}

__global__ __launch_bounds__(256) void k_composite_fwd(const float* __restrict__ raw, const double* __restrict__ zv,
                                                       int64_t n, int S, double* __restrict__ depth,
                                                       double* __restrict__ var, float* __restrict__ color) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ray >= n) return;
  const float* rr = raw + ray * (int64_t)S * 4;
  const double* zz = zv + ray * (int64_t)S;
  float carry = 1.f;
  float c0 = 0.f, c1 = 0.f, c2 = 0.f;
  double d = 0.0;
  const int nch = (S + 63) / 64;
  float wk[kMaxS / 64];
  double zk[kMaxS / 64];
#pragma unroll
  for (int c = 0; c < kMaxS / 64; ++c) {
    if (c >= nch) break;
    const RaySample s = load_sample(rr, zz, S, c * 64 + lane, lane, carry);
    c0 += s.w * s.raw[0];
    c1 += s.w * s.raw[1];
    c2 += s.w * s.raw[2];
    d += (double)s.w * s.z;
    wk[c] = s.w;
    zk[c] = s.z;
  }
  c0 = wave_sum(c0);
  c1 = wave_sum(c1);
  c2 = wave_sum(c2);
  d = wave_sumd(d);
  double v = 0.0;
#pragma unroll
  for (int c = 0; c < kMaxS / 64; ++c) {
    if (c >= nch) break;
    const double dz = zk[c] - d;
    v += ((double)wk[c] * dz) * dz;  // (weights*tmp)*tmp
  }
  v = wave_sumd(v);
  if (lane == 0) {
    depth[ray] = d;
    var[ray] = v;
    color[ray * 3 + 0] = c0;
    color[ray * 3 + 1] = c1;
    color[ray * 3 + 2] = c2;
  }
}

__global__ __launch_bounds__(256) void k_composite_bwd(const float* __restrict__ raw, const double* __restrict__ zv,
                                                       int64_t n, int S, const double* __restrict__ gdep,
                                                       const double* __restrict__ gvar,
                                                       const float* __restrict__ gcol, float* __restrict__ graw) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ray >= n) return;
  const float* rr = raw + ray * (int64_t)S * 4;
  const double* zz = zv + ray * (int64_t)S;
  const int nch = (S + 63) / 64;
  RaySample sm[kMaxS / 64];
  float carry = 1.f;
  double d = 0.0;
#pragma unroll
  for (int c = 0; c < kMaxS / 64; ++c) {
    if (c >= nch) break;
    sm[c] = load_sample(rr, zz, S, c * 64 + lane, lane, carry);
    d += (double)sm[c].w * sm[c].z;
  }
  d = wave_sumd(d);
  const double gd = gdep ? gdep[ray] : 0.0;
  const double gv = gvar ? gvar[ray] : 0.0;
  const float gc0 = gcol ? gcol[ray * 3 + 0] : 0.f;
  const float gc1 = gcol ? gcol[ray * 3 + 1] : 0.f;
  const float gc2 = gcol ? gcol[ray * 3 + 2] : 0.f;
  // d var / d depth = -sum_k [gv*(w dz) + (gv dz) w]
  double sdep = 0.0;
#pragma unroll
  for (int c = 0; c < kMaxS / 64; ++c) {
    if (c >= nch) break;
    const double dz = sm[c].z - d;
    const double w = (double)sm[c].w;
    sdep += gv * (w * dz) + (gv * dz) * w;
  }
  const double gdepth = gd - wave_sumd(sdep);
  // per-sample weight cotangent, then transmittance cotangent
  float gw[kMaxS / 64], gT[kMaxS / 64];
#pragma unroll
  for (int c = 0; c < kMaxS / 64; ++c) {
    if (c >= nch) break;
    const RaySample& s = sm[c];
    const double dz = s.z - d;
    const float g_dep = (float)(gdepth * s.z);
    const float g_var = (float)((gv * dz) * dz);
    const float g_rgb = gc0 * s.raw[0] + gc1 * s.raw[1] + gc2 * s.raw[2];
    gw[c] = (g_rgb + g_dep) + g_var;
    gT[c] = gw[c] * s.a;
  }
  // R_k = sum_{m>k} gT_m T_m (suffix over chunks, processed back to front)
  float tail = 0.f;
#pragma unroll
  for (int c = kMaxS / 64 - 1; c >= 0; --c) {
    if (c >= nch) continue;
    const RaySample& s = sm[c];
    const int k = c * 64 + lane;
    const float prod = (k < S) ? gT[c] * s.T : 0.f;
    const float incl = wave_suffix_sum(prod, lane);  // sum_{m>=k} within chunk
    const float nxt = __shfl_down(incl, 1, 64);
    const float R = (lane < 63 ? nxt : 0.f) + tail;  // sum_{m>k}
    tail += __shfl(incl, 0, 64);
    const float g_f = R / s.f;                       // cumprod backward: reversed_cumsum(w*grad)/input
    const float g_a = gw[c] * s.T - g_f;             // f = 1 - alpha + 1e-10
    const float g_occ = ((g_a * (1.f - s.a)) * s.a) * 10.f;  // sigmoid_backward, then the 10*
    if (k < S) {
      f32x4 o;
      o[0] = gc0 * s.w;
      o[1] = gc1 * s.w;
      o[2] = gc2 * s.w;
      o[3] = g_occ;
      *reinterpret_cast<f32x4*>(graw + (ray * (int64_t)S + k) * 4) = o;
    }
  }
}

int hip_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? NSLAM_OK : NSLAM_EHIP - (int)e;
}

}  // namespace

extern "C" int nslam_composite_fwd(const float* raw, const double* z_vals, int64_t n_rays, int32_t n_samples,
                                   double* depth, double* var, float* color, void* stream) {
  if (n_rays < 0 || n_samples <= 0) return NSLAM_EINVAL;
  if (n_samples > kMaxS) return NSLAM_EUNSUPPORTED;
  if (n_rays == 0) return NSLAM_OK;
  if (!raw || !z_vals || !depth || !var || !color) return NSLAM_EINVAL;
  const dim3 grid((unsigned)((n_rays + 3) / 4)), block(256);
  hipLaunchKernelGGL(k_composite_fwd, grid, block, 0, reinterpret_cast<hipStream_t>(stream), raw, z_vals, n_rays,
                     (int)n_samples, depth, var, color);
  return hip_status();
}

extern "C" int nslam_composite_bwd(const float* raw, const double* z_vals, int64_t n_rays, int32_t n_samples,
                                   const double* g_depth, const double* g_var, const float* g_color, float* g_raw,
                                   void* stream) {
  if (n_rays < 0 || n_samples <= 0) return NSLAM_EINVAL;
  if (n_samples > kMaxS) return NSLAM_EUNSUPPORTED;
  if (n_rays == 0) return NSLAM_OK;
  if (!raw || !z_vals || !g_raw) return NSLAM_EINVAL;
  const dim3 grid((unsigned)((n_rays + 3) / 4)), block(256);
  hipLaunchKernelGGL(k_composite_bwd, grid, block, 0, reinterpret_cast<hipStream_t>(stream), raw, z_vals, n_rays,
                     (int)n_samples, g_depth, g_var, g_color, g_raw);
  return hip_status();
}
