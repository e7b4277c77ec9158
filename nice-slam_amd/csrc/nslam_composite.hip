// nslam_composite.hip — volume compositing (occupancy mode) on gfx950 and its backward.
//
// Replaces raw2outputs_nerf_color (src/common.py:204-245) with occupancy=True
// (configs/nice_slam.yaml:5) and its autograd backward:
//   alpha_k = sigmoid(10 raw_k[3]);  T_k = prod_{j<k} (1 - alpha_j + 1e-10);  w_k = alpha_k T_k
//   rgb = sum_k w_k raw_k[:3] (f32);  depth = sum_k w_k z_k (f64);  var = sum_k w_k (z_k-depth)^2 (f64)
// One wave per ray, one lane per sample; the transmittance is a wave prefix product and the sums
// are wave shuffle reductions.  Rays with more than 64 samples are processed in 64-sample chunks
// with a carried transmittance.
#include <cstdlib>
#include <cstring>

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
// occ (may be NULL): the middle occupancy of a deferred-combine query, added to raw[...,3] in the
// reference's operand order (fine + middle, decoder.py:331-334) — what k_occ_combine would store.
__device__ __forceinline__ RaySample load_sample(const float* raw, const double* z, int S, int k, int lane,
                                                 float& carry, const float* occ = nullptr) {
  RaySample s;
  const bool act = k < S;
  s.raw = act ? *reinterpret_cast<const f32x4*>(raw + (size_t)k * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
  if (occ && act) s.raw[3] = s.raw[3] + occ[k];
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
  const int64_t ray = (int64_t)blockIdx.x * 4 + wave_id();
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

// Backward of one ray (the wave owns it) given its loaded samples, depth and cotangents
// (g_depth, g_var float64; g_color float32); writes g_raw for the ray's samples.
__device__ __forceinline__ void ray_bwd(const RaySample (&sm)[kMaxS / 64], int nch, int S, double d, double gd,
                                        double gv, float gc0, float gc1, float gc2, float* __restrict__ gr,
                                        int lane) {
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
      *reinterpret_cast<f32x4*>(gr + (int64_t)k * 4) = o;
    }
  }
}

// Forward of one ray: loads all its samples (kept in registers for a backward) and returns
// depth (float64), var (float64) and colour (float32 x3) exactly as k_composite_fwd.
struct RayOut {
  double d, v;
  float c0, c1, c2;
};

__device__ __forceinline__ RayOut ray_fwd(const float* rr, const double* zz, int S, int nch, RaySample (&sm)[kMaxS / 64],
                                          int lane, const float* occ = nullptr) {
  float carry = 1.f;
  RayOut o{0.0, 0.0, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < kMaxS / 64; ++c) {
    if (c >= nch) break;
    sm[c] = load_sample(rr, zz, S, c * 64 + lane, lane, carry, occ);
    o.c0 += sm[c].w * sm[c].raw[0];
    o.c1 += sm[c].w * sm[c].raw[1];
    o.c2 += sm[c].w * sm[c].raw[2];
    o.d += (double)sm[c].w * sm[c].z;
  }
  o.c0 = wave_sum(o.c0);
  o.c1 = wave_sum(o.c1);
  o.c2 = wave_sum(o.c2);
  o.d = wave_sumd(o.d);
#pragma unroll
  for (int c = 0; c < kMaxS / 64; ++c) {
    if (c >= nch) break;
    const double dz = sm[c].z - o.d;
    o.v += ((double)sm[c].w * dz) * dz;  // (weights*tmp)*tmp
  }
  o.v = wave_sumd(o.v);
  return o;
}

__global__ __launch_bounds__(256) void k_composite_bwd(const float* __restrict__ raw, const double* __restrict__ zv,
                                                       int64_t n, int S, const double* __restrict__ gdep,
                                                       const double* __restrict__ gvar,
                                                       const float* __restrict__ gcol, float* __restrict__ graw) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = (int64_t)blockIdx.x * 4 + wave_id();
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
  ray_bwd(sm, nch, S, d, gd, gv, gc0, gc1, gc2, graw + ray * (int64_t)S * 4, lane);
}

// ------------------------------------------------------------------------------------------
// Rendering loss fused with compositing fwd + bwd (Mapper.py:487-503, Tracker.py:110-125)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double sgnd(double x) { return (double)((x > 0.0) - (x < 0.0)); }
__device__ __forceinline__ float sgnf(float x) { return (float)((x > 0.f) - (x < 0.f)); }

struct LossArgs {
  nslam_loss_cfg cfg;
  const float* raw;
  const double* z;
  int64_t n;
  int S;
  const float *gt, *gtc;
  const uint8_t* keep;
  double *depth, *var;
  float* color;
  double* ray_loss;
  float* g_raw;
  double* resid;      // tracker: r per ray (ws)
  const double* thr;  // tracker: 10 * median (ws), read by the backward pass
  int32_t inline_median;  // pass 2 forms the threshold itself (n <= kInlineMedian)
};

// Tracker handle_dynamic: thr = 10 * median(r over kept rays) (torch.median: lower median), by every thread
// of one workgroup: kept residuals into LDS (sv: a power of two >= n doubles); up to one per thread
// (tracking: 200 rays) the median is selected by rank, else (or with a NaN) padded with +inf to a power of
// two and bitonic-sorted.  Either way the same value for any workgroup size.
constexpr int kMedianMax = 16384;

__device__ double median_thr_block(const double* __restrict__ r, const uint8_t* __restrict__ keep, int n,
                                   double* sv) {
  __shared__ int cnt, nan_seen;
  __shared__ double thr;
  if (threadIdx.x == 0) cnt = nan_seen = 0;
  __syncthreads();
  int np2 = 1;
  while (np2 < n) np2 <<= 1;
  for (int i = threadIdx.x; i < np2; i += blockDim.x) sv[i] = INFINITY;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double v = r[i];  // (loaded beside the mask, not after it: one memory round trip, not two)
    if (!keep || keep[i]) {
      if (v != v) nan_seen = 1;
      sv[atomicAdd(&cnt, 1)] = v;
    }
  }
  __syncthreads();
  const int c = cnt;
  if (c <= (int)blockDim.x && !nan_seen) {
    // selection by rank (one value per thread, ties broken by slot): the value of rank (c-1)/2 is
    // the lower median — the element the sort below would put there, without its log^2 passes
    const int i = threadIdx.x;
    if (i < c) {
      const double x = sv[i];
      int rank = 0;
#pragma unroll 16
      for (int j = 0; j < c; ++j) {  // (unrolled: 16 broadcast LDS reads in flight, not one at a time)
        const double y = sv[j];
        rank += (y < x) || (y == x && j < i);
      }
      if (rank == (c - 1) / 2) thr = 10.0 * x;
    }
    if (c == 0 && i == 0) thr = INFINITY;
    __syncthreads();
    return thr;
  }
  for (int k = 2; k <= np2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < np2; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const double x = sv[i], y = sv[l];
          const bool up = (i & k) == 0;
          if ((x > y) == up) {
            sv[i] = y;
            sv[l] = x;
          }
        }
      }
      __syncthreads();
    }
  }
  return cnt > 0 ? 10.0 * sv[(cnt - 1) / 2] : INFINITY;
}

__global__ __launch_bounds__(1024) void k_median_thr(const double* __restrict__ r, const uint8_t* __restrict__ keep,
                                                     int n, double* __restrict__ thr) {
  extern __shared__ double sv[];
  const double t = median_thr_block(r, keep, n, sv);
  if (threadIdx.x == 0) *thr = t;
}

// up to this many rays the tracker's loss pass 2 forms the threshold itself, in every workgroup (one
// residual per thread: the rank selection), instead of a k_median_thr launch between the passes
constexpr int kInlineMedian = 256;

// PASS 0: mapper, fwd + loss + bwd in one pass.
// PASS 1: tracker fwd (outputs + residual r).  PASS 2: tracker loss + bwd (after the median).
template <int PASS>
__global__ __launch_bounds__(256) void k_render_loss(LossArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = (int64_t)blockIdx.x * 4 + wave_id();
  double thr = 0.0;
  if constexpr (PASS == 2) {
    if (a.cfg.handle_dynamic) {
      if (a.inline_median) {  // (the whole workgroup, before any wave leaves)
        __shared__ double sv[kInlineMedian];
        thr = median_thr_block(a.resid, a.keep, (int)a.n, sv);
      } else {
        thr = *a.thr;
      }
    }
  }
  if (ray >= a.n) return;
  const int S = a.S;
  const float* rr = a.raw + ray * (int64_t)S * 4;
  const double* zz = a.z + ray * (int64_t)S;
  const int nch = (S + 63) / 64;
  RaySample sm[kMaxS / 64];
  const RayOut o = ray_fwd(rr, zz, S, nch, sm, lane, a.cfg.occ_add ? a.cfg.occ_add + ray * (int64_t)S : nullptr);
  const bool kp = a.keep ? a.keep[ray] != 0 : true;
  const float gt = a.gt[ray];
  if (PASS != 2 && lane == 0) {
    a.depth[ray] = o.d;
    a.var[ray] = o.v;
    a.color[ray * 3 + 0] = o.c0;
    a.color[ray * 3 + 1] = o.c1;
    a.color[ray * 3 + 2] = o.c2;
  }
  const double x = (double)gt - o.d;  // gt (float32) - depth (float64) in float64
  double gd = 0.0, lossd = 0.0;
  bool mcol = false;
  if (PASS == 0) {
    const bool m = kp && gt > 0.f;
    gd = m ? -sgnd(x) : 0.0;
    lossd = m ? fabs(x) : 0.0;
    mcol = kp && a.cfg.use_color;
  } else {
    const double sq = sqrt(o.v + 1e-10);  // uncertainty detached (Tracker.py:110)
    const double r = fabs(x) / sq;
    if (PASS == 1) {
      if (lane == 0) a.resid[ray] = r;
      return;
    }
    const bool m = kp && gt > 0.f && (!a.cfg.handle_dynamic || r < thr);
    gd = m ? -(sgnd(x) * (1.0 / sq)) : 0.0;
    lossd = m ? r : 0.0;
    mcol = m && a.cfg.use_color;
  }
  float gc0 = 0.f, gc1 = 0.f, gc2 = 0.f;
  if (mcol) {  // d/dc of w * |gt_c - c|  (float32 branch of the loss)
    const float e0 = a.gtc[ray * 3 + 0] - o.c0, e1 = a.gtc[ray * 3 + 1] - o.c1, e2 = a.gtc[ray * 3 + 2] - o.c2;
    const float w = a.cfg.w_color;
    gc0 = -(w * sgnf(e0));
    gc1 = -(w * sgnf(e1));
    gc2 = -(w * sgnf(e2));
    lossd += (double)(w * ((fabsf(e0) + fabsf(e1)) + fabsf(e2)));
  }
  if (a.ray_loss && lane == 0) a.ray_loss[ray] = lossd;
  if (a.g_raw) ray_bwd(sm, nch, S, o.d, gd, 0.0, gc0, gc1, gc2, a.g_raw + ray * (int64_t)S * 4, lane);
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

namespace {
size_t loss_ws(const nslam_loss_cfg* cfg, int64_t n) {
  if (!cfg || cfg->mode != NSLAM_LOSS_TRACKER || n <= 0) return 0;
  return (size_t)(n + 1) * sizeof(double);
}
}  // namespace

extern "C" size_t nslam_render_loss_workspace_size(const nslam_loss_cfg* cfg, int64_t n_rays) {
  return loss_ws(cfg, n_rays);
}

extern "C" int nslam_render_loss(const nslam_loss_cfg* cfg, const float* raw, const double* z_vals, int64_t n_rays,
                                 int32_t n_samples, const float* gt_depth, const float* gt_color,
                                 const uint8_t* keep, double* depth, double* var, float* color, double* ray_loss,
                                 float* g_raw, void* ws, size_t ws_bytes, void* stream) {
  if (!cfg || (cfg->mode != NSLAM_LOSS_MAPPER && cfg->mode != NSLAM_LOSS_TRACKER)) return NSLAM_EINVAL;
  if (n_rays < 0 || n_samples <= 0) return NSLAM_EINVAL;
  if (n_samples > kMaxS) return NSLAM_EUNSUPPORTED;
  if (n_rays == 0) return NSLAM_OK;
  if (!raw || !z_vals || !gt_depth || !depth || !var || !color) return NSLAM_EINVAL;
  if (cfg->use_color && !gt_color) return NSLAM_EINVAL;
  const bool trk = cfg->mode == NSLAM_LOSS_TRACKER;
  if (trk && cfg->handle_dynamic && n_rays > kMedianMax) return NSLAM_EUNSUPPORTED;
  if (ws_bytes < loss_ws(cfg, n_rays) || (loss_ws(cfg, n_rays) && !ws)) return NSLAM_EWORKSPACE;
  const char* ml = getenv("NSLAM_MEDIAN_LAUNCH");  // "1": the separate median launch (A/B and tests)
  if (ml && strcmp(ml, "0") != 0 && strcmp(ml, "1") != 0) return NSLAM_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  LossArgs a{};
  a.cfg = *cfg;
  a.raw = raw;
  a.z = z_vals;
  a.n = n_rays;
  a.S = n_samples;
  a.gt = gt_depth;
  a.gtc = gt_color;
  a.keep = keep;
  a.depth = depth;
  a.var = var;
  a.color = color;
  a.ray_loss = ray_loss;
  a.g_raw = g_raw;
  const dim3 grid((unsigned)((n_rays + 3) / 4)), block(256);
  if (!trk) {
    hipLaunchKernelGGL(k_render_loss<0>, grid, block, 0, s, a);
    return hip_status();
  }
  double* w = reinterpret_cast<double*>(ws);
  a.resid = w;
  a.thr = w + n_rays;
  hipLaunchKernelGGL(k_render_loss<1>, grid, block, 0, s, a);  // outputs + residuals
  a.inline_median = n_rays <= kInlineMedian && !(ml && ml[0] == '1');
  if (cfg->handle_dynamic && !a.inline_median) {
    int np2 = 1;
    while (np2 < n_rays) np2 <<= 1;
    const size_t lds = (size_t)np2 * sizeof(double);
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(k_median_thr), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
      return hip_status();
    hipLaunchKernelGGL(k_median_thr, dim3(1), dim3(1024), lds, s, w, keep, (int)n_rays, w + n_rays);
  }
  hipLaunchKernelGGL(k_render_loss<2>, grid, block, 0, s, a);
  return hip_status();
}
