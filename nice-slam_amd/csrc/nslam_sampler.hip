// nslam_sampler.hip — per-ray stratified + surface sampler on gfx950.
//
// Replaces src/utils/Renderer.py:82-174 (perturb=0, N_importance=0):
//   far_bb = min_axis max_end((bound - o)/d) + 0.01                 (float64, :98-105)
//   gt given: near = gt*0.01 (f32), far = clamp(far_bb, 0, max_batch(gt*1.2))   (:94-96,107-111)
//   gt none : near = 0.01, far = far_bb, no surface samples          (:88-92)
//   z = near*(1-t) [f32] + far*t [f64]                                (:152-157)
//   surface: gt>0 → (0.95gt)*(1-u) + (1.05gt)*u ; gt<=0 → 0.001*(1-u) + max_batch(gt)*u  (:128-150)
//   z_vals = sort(cat[z, z_surface])                                  (:168-170)
// The two lists are monotone in their index, so the sort is a two-way merge (each list reversed
// first if it is descending).  Dtype promotions follow the reference exactly (no FMA contraction:
// the library is built with -ffp-contract=off).
#include "nslam_dev.h"

namespace {

constexpr int kMaxS0 = 128, kMaxS1 = 64;

__global__ void k_key_of(const float* __restrict__ gmax, uint32_t* __restrict__ ws) { *ws = fkey(*gmax); }

__global__ __launch_bounds__(256) void k_max_gt(const float* __restrict__ gt, int64_t n, uint32_t* __restrict__ ws) {
  uint32_t m = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = max(m, fkey(gt[i]));
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d, 64));
  if ((threadIdx.x & 63) == 0 && m) atomicMax(ws, m);
}

struct SamplerArgs {
  const float* o;
  const float* d;
  const float* gt;
  int64_t n;
  double lo[3], hi[3];
  const float* ts;
  int s0;
  const double* tu;
  int s1;
  int lindisp;
  double* z;
  const uint32_t* ws;    // max_batch(gt) as an order-preserving key (large batches)
  const float* gmax_ptr; // max_batch(gt) given by the caller (ray-sharded job: all-reduced)
  int local_max;         // small batch: every workgroup of k_sample_wave reduces gt itself
};

// Batches up to this many rays reduce max(gt) inside k_sample_wave (each workgroup re-reads the
// whole gt vector, <= 32 KiB from L2) instead of a memset + k_max_gt launch ahead of it.
constexpr int64_t kLocalMaxRays = 8192;

__global__ __launch_bounds__(128) void k_sample(SamplerArgs a) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.n) return;
  double tmin = 0.0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double o = (double)a.o[r * 3 + k];
    const double dd = (double)a.d[r * 3 + k];
    const double t0 = (a.lo[k] - o) / dd;
    const double t1 = (a.hi[k] - o) / dd;
    const double tm = t0 > t1 ? t0 : t1;  // max over the two ends
    tmin = (k == 0 || tm < tmin) ? tm : tmin;
  }
  const double far_bb = tmin + 0.01;
  const bool has_gt = a.gt != nullptr;
  float g = 0.f, near_f = 0.01f;
  double far = far_bb;
  float gmax = 0.f;
  if (has_gt) {
    g = a.gt[r];
    gmax = fkey_inv(*a.ws);
    near_f = g * 0.01f;
    const double hi = (double)(gmax * 1.2f);  // max(gt*1.2) == f32(max(gt)*1.2) (monotone rounding)
    far = far_bb < 0.0 ? 0.0 : far_bb;
    far = far > hi ? hi : far;
  }
  double zs[kMaxS0];
  const int s0 = a.s0;
  for (int i = 0; i < s0; ++i) {
    const float t = a.ts[i];
    if (!a.lindisp) {
      zs[i] = (double)(near_f * (1.f - t)) + far * (double)t;
    } else {
      zs[i] = 1.0 / ((double)((1.f / near_f) * (1.f - t)) + (1.0 / far) * (double)t);
    }
  }
  double* out = a.z + r * (int64_t)(s0 + (has_gt ? a.s1 : 0));
  const int s1 = has_gt ? a.s1 : 0;
  if (s1 == 0) {  // no sort in the reference when N_surface == 0 (Renderer.py:168)
    for (int i = 0; i < s0; ++i) out[i] = zs[i];
    return;
  }
  double zu[kMaxS1];
  if (g > 0.f) {
    const double lo_s = (double)(0.95f * g), hi_s = (double)(1.05f * g);
    for (int i = 0; i < s1; ++i) zu[i] = lo_s * (1.0 - a.tu[i]) + hi_s * a.tu[i];
  } else {
    for (int i = 0; i < s1; ++i) zu[i] = 0.001 * (1.0 - a.tu[i]) + (double)gmax * a.tu[i];
  }
  const bool rev0 = s0 > 1 && zs[s0 - 1] < zs[0];
  const bool rev1 = s1 > 1 && zu[s1 - 1] < zu[0];
  double m[kMaxS0 + kMaxS1];
  int i = 0, j = 0;
  for (int k = 0; k < s0 + s1; ++k) {
    const double va = i < s0 ? zs[rev0 ? s0 - 1 - i : i] : 0.0;
    const double vb = j < s1 ? zu[rev1 ? s1 - 1 - j : j] : 0.0;
    const bool take_a = (j >= s1) || (i < s0 && va <= vb);
    m[k] = take_a ? va : vb;
    i += take_a ? 1 : 0;
    j += take_a ? 0 : 1;
  }
  // rounding can leave ulp-level inversions inside a "monotone" list: finish with an insertion
  // sort (linear on nearly sorted input) so the result equals torch.sort exactly
  for (int k = 1; k < s0 + s1; ++k) {
    const double v = m[k];
    int q = k - 1;
    while (q >= 0 && m[q] > v) {
      m[q + 1] = m[q];
      --q;
    }
    m[q + 1] = v;
  }
  for (int k = 0; k < s0 + s1; ++k) out[k] = m[k];
}

// One wave per ray (S = s0 + s1 <= 64): lane k holds sample k of the stratified list (k < s0)
// or of the surface list; the final position is the rank of the value among all S values (ties
// broken by lane), i.e. exactly the ascending order torch.sort produces — no serial merge.
__global__ __launch_bounds__(256) void k_sample_wave(SamplerArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + wave_id();
  __shared__ uint32_t wmax[4];
  if (a.local_max) {  // workgroup-wide max over the batch (all threads take part before any exit)
    uint32_t m = 0;
    for (int64_t i = threadIdx.x; i < a.n; i += 256) m = max(m, fkey(a.gt[i]));
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d, 64));
    if (lane == 0) wmax[wave_id()] = m;
    __syncthreads();
  }
  if (r >= a.n) return;
  double tmin = 0.0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double o = (double)a.o[r * 3 + k];
    const double dd = (double)a.d[r * 3 + k];
    const double t0 = (a.lo[k] - o) / dd;
    const double t1 = (a.hi[k] - o) / dd;
    const double tm = t0 > t1 ? t0 : t1;
    tmin = (k == 0 || tm < tmin) ? tm : tmin;
  }
  const double far_bb = tmin + 0.01;
  const bool has_gt = a.gt != nullptr;
  const int s0 = a.s0, s1 = has_gt ? a.s1 : 0, S = s0 + s1;
  float g = 0.f, near_f = 0.01f, gmax = 0.f;
  double far = far_bb;
  if (has_gt) {
    g = a.gt[r];
    if (a.gmax_ptr)
      gmax = *a.gmax_ptr;
    else if (a.local_max)
      gmax = fkey_inv(max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3])));
    else
      gmax = fkey_inv(*a.ws);
    near_f = g * 0.01f;
    const double hi = (double)(gmax * 1.2f);
    far = far_bb < 0.0 ? 0.0 : far_bb;
    far = far > hi ? hi : far;
  }
  double v = __builtin_inf();
  if (lane < s0) {
    const float t = a.ts[lane];
    v = a.lindisp ? 1.0 / ((double)((1.f / near_f) * (1.f - t)) + (1.0 / far) * (double)t)
                  : (double)(near_f * (1.f - t)) + far * (double)t;
  } else if (lane < S) {
    const double u = a.tu[lane - s0];
    v = g > 0.f ? (double)(0.95f * g) * (1.0 - u) + (double)(1.05f * g) * u : 0.001 * (1.0 - u) + (double)gmax * u;
  }
  double* out = a.z + r * (int64_t)S;
  if (s1 == 0) {  // no sort in the reference when N_surface == 0 (Renderer.py:168)
    if (lane < S) out[lane] = v;
    return;
  }
  int rank = 0;
  const int v_lo = __double2loint(v), v_hi = __double2hiint(v);
  for (int j = 0; j < S; ++j) {  // lane j's value by v_readlane (j is uniform): no LDS round trip per step
    const double vj = __hiloint2double(__builtin_amdgcn_readlane(v_hi, j), __builtin_amdgcn_readlane(v_lo, j));
    rank += (vj < v || (vj == v && j < lane)) ? 1 : 0;
  }
  if (lane < S) out[rank] = v;
}

int hip_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? NSLAM_OK : NSLAM_EHIP - (int)e;
}

}  // namespace

extern "C" size_t nslam_workspace_size(int which, int64_t n) {
  (void)n;
  if (which == NSLAM_WS_SAMPLER) return 256;
  return 0;
}

extern "C" int nslam_sample_rays(const float* rays_o, const float* rays_d, const float* gt_depth, const float* gt_max,
                                 int64_t n_rays,
                                 const double* bound_lo, const double* bound_hi, const float* t_strat, int32_t s0,
                                 const double* t_surf, int32_t s1, int32_t lindisp, double* z_vals, void* ws,
                                 size_t ws_bytes, void* stream) {
  if (n_rays < 0 || s0 <= 0 || s1 < 0 || !bound_lo || !bound_hi) return NSLAM_EINVAL;
  if (s0 > kMaxS0 || s1 > kMaxS1) return NSLAM_EUNSUPPORTED;
  if (n_rays == 0) return NSLAM_OK;
  if (!rays_o || !rays_d || !t_strat || !z_vals) return NSLAM_EINVAL;
  if (gt_depth && s1 > 0 && !t_surf) return NSLAM_EINVAL;
  if (gt_depth && (!ws || ws_bytes < nslam_workspace_size(NSLAM_WS_SAMPLER, n_rays))) return NSLAM_EWORKSPACE;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  SamplerArgs a;
  a.o = rays_o;
  a.d = rays_d;
  a.gt = gt_depth;
  a.n = n_rays;
  for (int k = 0; k < 3; ++k) {
    a.lo[k] = bound_lo[k];
    a.hi[k] = bound_hi[k];
  }
  a.ts = t_strat;
  a.s0 = s0;
  a.tu = t_surf;
  a.s1 = s1;
  a.lindisp = lindisp;
  a.z = z_vals;
  a.ws = reinterpret_cast<const uint32_t*>(ws);
  const bool wave_form = s0 + (gt_depth ? s1 : 0) <= 64;
  a.gmax_ptr = nullptr;
  a.local_max = 0;
  if (gt_depth && gt_max && wave_form) {
    a.gmax_ptr = gt_max;
  } else if (gt_depth && wave_form && n_rays <= kLocalMaxRays) {
    a.local_max = 1;
  } else if (gt_depth && gt_max) {
    hipLaunchKernelGGL(k_key_of, dim3(1), dim3(1), 0, s, gt_max, reinterpret_cast<uint32_t*>(ws));
  } else if (gt_depth) {
    if (hipMemsetAsync(ws, 0, 4, s) != hipSuccess) return hip_status();
    const int blocks = (int)std::min<int64_t>((n_rays + 255) / 256, 1024);
    hipLaunchKernelGGL(k_max_gt, dim3(blocks), dim3(256), 0, s, gt_depth, n_rays, reinterpret_cast<uint32_t*>(ws));
  }
  if (wave_form)
    hipLaunchKernelGGL(k_sample_wave, dim3((unsigned)((n_rays + 3) / 4)), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_sample, dim3((unsigned)((n_rays + 127) / 128)), dim3(128), 0, s, a);
  return hip_status();
}

extern "C" const char* nslam_strerror(int code) {
  switch (code) {
    case NSLAM_OK: return "ok";
    case NSLAM_EINVAL: return "invalid argument (null pointer, bad size/enum or misaligned buffer)";
    case NSLAM_EUNSUPPORTED: return "configuration outside the supported NICE-SLAM path";
    case NSLAM_EWORKSPACE: return "workspace too small";
    default: return code <= NSLAM_EHIP ? "HIP launch error (NSLAM_EHIP - hipError_t)" : "unknown error";
  }
}

// v9: nslam_cam_grad / nslam_cam_pose exports (they first shipped under v8 without a bump)
extern "C" int nslam_abi_version(void) { return 23; }
