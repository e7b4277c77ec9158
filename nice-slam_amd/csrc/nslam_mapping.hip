// nslam_mapping.hip — the per-iteration glue of Mapper.optimize_map / Tracker.optimize_cam_in_batch
// as two single-launch kernels on gfx950:
//   k_gather_rays : get_samples (src/common.py:74-134) for all frames of the window at once, with
//                   the inside-mask prefilter (Mapper.py:469-481, Tracker.py:93-104) folded in;
//   k_adam        : torch.optim.Adam's update (Mapper.py:504, Tracker.py:126) over dense parameter
//                   segments and frustum-masked grid rows (Mapper.py:314-333) in one launch.
// Both are HBM/latency-bound elementwise work: no LDS, coalesced float4 rows where the layout allows.
#include <math.h>

#include "nslam_dev.h"

namespace {

int hip_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? NSLAM_OK : NSLAM_EHIP - (int)e;
}

// ------------------------------------------------------------------------------------------
// pixel sampling + rays + inside mask
// ------------------------------------------------------------------------------------------
struct GatherArgs {
  nslam_frame fr[NSLAM_MAX_FRAMES];
  int32_t nf;
  int64_t n_per, n;
  const int64_t* pix;
  int32_t W, h0, w0, ww;
  float fx, fy, cx, cy;
  int32_t use_bound;
  double lo[3], hi[3];
  float *ro, *rd, *gd, *gc;
  uint8_t* keep;
  nslam_draw draw;  // pix == NULL: in-kernel draws
  int64_t wn;       // window size (h1-h0)*(w1-w0)
  int64_t* n_kept;
};

// splitmix64 finaliser: a counter-based stream (seed, draw counter, ray) -> 64 uniform bits
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

// torch.max / torch.min propagate NaN
__device__ __forceinline__ double nanmax(double a, double b) { return (a > b || a != a) ? a : b; }
__device__ __forceinline__ double nanmin(double a, double b) { return (a < b || a != a) ? a : b; }

// get_camera_from_tensor (common.py:137-176): c2w [3][4] from the 7-vector (quad2rotation's products and
// differences, no FMA contraction); the one arithmetic of k_cam_pose, k_cam_pose_batch and the gather
__device__ __forceinline__ void cam_pose_one(const float* __restrict__ cam, float* __restrict__ c2w) {
  const float qr = cam[0], qi = cam[1], qj = cam[2], qk = cam[3];
  const float two_s = 2.0f / (((qr * qr + qi * qi) + qj * qj) + qk * qk);
  const float R[9] = {1.0f - two_s * (qj * qj + qk * qk), two_s * (qi * qj - qk * qr), two_s * (qi * qk + qj * qr),
                      two_s * (qi * qj + qk * qr), 1.0f - two_s * (qi * qi + qk * qk), two_s * (qj * qk - qi * qr),
                      two_s * (qi * qk - qj * qr), two_s * (qj * qk + qi * qr), 1.0f - two_s * (qi * qi + qj * qj)};
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) c2w[4 * i + j] = R[3 * i + j];
    c2w[4 * i + 3] = cam[4 + i];
  }
}

// One pixel of frame f at window index k: rays_o/rays_d (common.py:74-89), gt depth (0 when the
// inside mask drops the ray), the pixel offset and the mask.
struct RayAt {
  float o[3], d[3], gt;
  int64_t px;
  bool kp;
};

__device__ __forceinline__ RayAt ray_at(const GatherArgs& a, int f, int64_t k) {
  const nslam_frame& fr = a.fr[f];
  // ABI v21: a frame given by its camera 7-vector has its pose formed here (the same values as nslam_cam_pose);
  // either way the 12 entries sit in registers (no pointer that could be private or global memory)
  float P[12];
  if (fr.cam) {
    cam_pose_one(fr.cam, P);
  } else {
#pragma unroll
    for (int e = 0; e < 12; ++e) P[e] = fr.c2w[e];
  }
  RayAt r;
  // window index -> (row, col); torch.linspace(W0, W1-1, W1-W0) holds exact integers
  const int64_t row = k / a.ww, col = k - row * a.ww;
  r.px = (a.h0 + row) * a.W + (a.w0 + col);
  const float i = (float)(a.w0 + col), j = (float)(a.h0 + row);
  // dirs = ((i-cx)/fx, -(j-cy)/fy, -1); rays_d = sum(dirs * c2w[:3,:3], -1) (common.py:80-86).
  // On the GPU torch divides by a CPU scalar as a multiply by its float reciprocal
  // (BinaryDivTrueKernel), which is what the reference runs: do the same.
  const float d0 = (i - a.cx) * (1.f / a.fx);
  const float d1 = -(j - a.cy) * (1.f / a.fy);
  const float d2 = -1.f;
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const float* c2w = &P[4 * m];
    // torch's 3-element sum reduces as (p0 + p2) + p1 on this device (tools/probes/rays_order.py)
    r.d[m] = (d0 * c2w[0] + d2 * c2w[2]) + d1 * c2w[1];
    r.o[m] = c2w[3];
  }
  r.gt = fr.depth[r.px];
  r.kp = true;
  if (a.use_bound) {  // t = (bound - o) / d (float64); t_exit = min_axis max(t_lo, t_hi) >= gt
    double tex = 0.0;
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const double tl = (a.lo[m] - (double)r.o[m]) / (double)r.d[m];
      const double th = (a.hi[m] - (double)r.o[m]) / (double)r.d[m];
      const double tm = nanmax(tl, th);
      tex = m == 0 ? tm : nanmin(tex, tm);
    }
    r.kp = tex >= (double)r.gt;
  }
  if (!r.kp) r.gt = 0.f;
  return r;
}

// select_uv's draw for global ray g: Lemire's multiply-shift maps 32 uniform bits onto [0, wn)
// (bias < wn / 2^32)
__device__ __forceinline__ int64_t draw_k(const GatherArgs& a, uint64_t ctr, uint64_t g) {
  return (int64_t)(((mix64(a.draw.seed ^ mix64(ctr * 0x9e3779b97f4a7c15ull + g)) >> 32) * (uint64_t)a.wn) >> 32);
}

__global__ __launch_bounds__(256) void k_gather_rays(GatherArgs a) {
  const int64_t ray = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < NSLAM_MAX_FRAMES) {  // the poses formed from 7-vectors, for later launches
    const nslam_frame& fr = a.fr[threadIdx.x];
    if ((int)threadIdx.x < a.nf && fr.cam && fr.c2w_out) cam_pose_one(fr.cam, fr.c2w_out);
  }
  __shared__ uint64_t ctr;
  __shared__ uint32_t wred[2][4];
  const bool drawn = a.pix == nullptr;
  if (threadIdx.x == 0)  // in-kernel draws: every workgroup reads the counter before the last one bumps it
    ctr = drawn ? __hip_atomic_load(a.draw.counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  __syncthreads();
  bool kp = false;
  uint32_t mkey = 0;  // max over the global batch's kept gt (key 0: below every float)
  if (ray < a.n) {
    const int f = (int)(ray / a.n_per);
    const int64_t kk = ray - (int64_t)f * a.n_per;
    const uint64_t g0 = (uint64_t)f * (uint64_t)(a.n_per * a.draw.world) + (uint64_t)kk;  // rank 0's slot
    const int64_t k = drawn ? draw_k(a, ctr, g0 + (uint64_t)a.draw.rank * a.n_per) : a.pix[ray];
    const RayAt r = ray_at(a, f, k);
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      a.ro[ray * 3 + m] = r.o[m];
      a.rd[ray * 3 + m] = r.d[m];
      a.gc[ray * 3 + m] = a.fr[f].color[r.px * 3 + m];
    }
    a.gd[ray] = r.gt;
    if (a.keep) a.keep[ray] = r.kp ? 1 : 0;
    kp = r.kp;
    if (a.draw.gt_max) {  // the other ranks' rays of this slot, re-drawn here (no collective)
      mkey = fkey(r.gt);
      for (int j = 0; j < a.draw.world; ++j)
        if (j != a.draw.rank) mkey = max(mkey, fkey(ray_at(a, f, draw_k(a, ctr, g0 + (uint64_t)j * a.n_per)).gt));
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (a.n_kept) {  // kept-ray count: wave ballot, one atomic per workgroup
    const int cnt = __popcll(__ballot(kp));
    if (lane == 0) wred[0][wv] = (uint32_t)cnt;
  }
  if (a.draw.gt_max) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) mkey = max(mkey, (uint32_t)__shfl_xor((int)mkey, d, 64));
    if (lane == 0) wred[1][wv] = mkey;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (a.n_kept) {
      const uint32_t tot = wred[0][0] + wred[0][1] + wred[0][2] + wred[0][3];
      if (tot) atomicAdd(reinterpret_cast<unsigned long long*>(a.n_kept), (unsigned long long)tot);
    }
    if (a.draw.gt_max)
      __hip_atomic_fetch_max(a.draw.gt_max_key, max(max(wred[1][0], wred[1][1]), max(wred[1][2], wred[1][3])),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (drawn) {
      // count this workgroup in (release: its max is in); the last one (acquire: sees every max)
      // publishes the batch max, re-arms the key and ticket and advances the draw counter
      const uint32_t t = __hip_atomic_fetch_add(a.draw.ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (t == gridDim.x - 1) {
        if (a.draw.gt_max) {
          const uint32_t key = __hip_atomic_exchange(a.draw.gt_max_key, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          *a.draw.gt_max = fkey_inv(key);
        }
        __hip_atomic_store(a.draw.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(a.draw.counter, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Adam
// ------------------------------------------------------------------------------------------
struct AdamArgs {
  nslam_adam_seg seg[NSLAM_ADAM_MAX_SEGS];
  int64_t blk0[NSLAM_ADAM_MAX_SEGS + 1];  // first workgroup of each segment
  int32_t nseg;
  float b1, b2, eps;
  int32_t zero_grad;
  uint32_t* ticket;  // non-NULL: the last workgroup advances the step counts (no second launch)
};

constexpr int kAdamThreads = 256;
constexpr int kAdamItems = 4;  // float4 rows (or floats) per thread: 4 x 4 loads in flight

// A segment with a device live count (ABI v19 n_live) gets at most kLiveBlocks workgroups, which stride
// over the live rows: its launch does not scale with the capacity it is sized for.
constexpr int64_t kLiveBlocks = 512;

// the element update and its coefficients: adam_coef / adam_one (nslam_dev.h)
__global__ __launch_bounds__(kAdamThreads) void k_adam(AdamArgs a) {
  const int64_t b = blockIdx.x;
  int s = 0;
  while (s + 1 < a.nseg && b >= a.blk0[s + 1]) ++s;
  const nslam_adam_seg& sg = a.seg[s];
  const float step = *sg.step;
  const auto coef = [&] { return adam_coef(a.b1, a.b2, a.eps, sg.lr, step); };
  if (sg.n_live) {  // stride the live rows (the same per-row update as the one-pass path)
    nslam_adam_seg live = sg;
    live.n = *sg.n_live < sg.n ? *sg.n_live : sg.n;
    live.n_live = nullptr;
    const int64_t need = adam_segment_blocks<kAdamItems>(live, kAdamThreads);
    const int64_t assigned = a.blk0[s + 1] - a.blk0[s];
    for (int64_t lb = b - a.blk0[s]; lb < need; lb += assigned)
      adam_segment_block<kAdamItems>(live, coef, lb, a.zero_grad, (int)threadIdx.x, kAdamThreads);
  } else {
    adam_segment_block<kAdamItems>(sg, coef, b - a.blk0[s], a.zero_grad, (int)threadIdx.x, kAdamThreads);
  }
  if (a.ticket) {
    // Every workgroup read its segment's step count at its start (the value was consumed long
    // before this point), so once all of them have drawn a ticket no read is outstanding and the
    // last one may advance every count and re-arm the ticket for the next launch.  The next
    // launch is a later kernel: its reads see these stores across the kernel boundary.
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t tk = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tk == gridDim.x - 1) {
        for (int k = 0; k < a.nseg; ++k) *a.seg[k].step += 1.f;
        __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// Without a ticket, every segment's step advances after the update kernel in its own single-wave
// launch (stream order makes it see all reads of the old count).  The ticket path above needs no
// release fence: the last workgroup reads nothing the other workgroups wrote (only the ticket, an
// atomic), and the counts it stores are read by later kernels only, across the kernel boundary.
__global__ __launch_bounds__(64) void k_adam_steps(AdamArgs a) {
  if (threadIdx.x < (unsigned)a.nseg) *a.seg[threadIdx.x].step += 1.f;
}

// ------------------------------------------------------------------------------------------
// sparse gradient exchange (ray-sharded mapping)
// ------------------------------------------------------------------------------------------
// Only the frustum-selected rows of a grid gradient reach Adam (Mapper.py:314-333,394-401), so
// only they are summed across ranks: pack them (+ the dense decoder gradients) into one buffer,
// all-reduce it, unpack.  One float4 (rows) or float (tail) per thread; pure HBM copy.
template <bool PACK>
__global__ __launch_bounds__(256) void k_rows_xfer(float* __restrict__ grid, const int32_t* __restrict__ rows,
                                                   int64_t n_rows, int q, float* __restrict__ tail, int64_t n_tail,
                                                   float* __restrict__ buf) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nv = n_rows * q;
  if (e < nv) {
    const int64_t ri = e / q, part = e - ri * q;
    f32x4* gp = reinterpret_cast<f32x4*>(grid + ((int64_t)rows[ri] * q + part) * 4);
    f32x4* bp = reinterpret_cast<f32x4*>(buf + e * 4);
    if (PACK)
      *bp = *gp;
    else
      *gp = *bp;
  } else if (e - nv < n_tail) {
    const int64_t t = e - nv;
    if (PACK)
      buf[nv * 4 + t] = tail[t];
    else
      tail[t] = buf[nv * 4 + t];
  }
}

int rows_xfer(bool pack, float* grid, const int32_t* rows, int64_t n_rows, int32_t row_len, float* tail,
              int64_t n_tail, float* buf, void* stream) {
  if (n_rows < 0 || n_tail < 0 || row_len <= 0 || row_len % 4) return NSLAM_EINVAL;
  if ((n_rows > 0 && (!grid || !rows)) || (n_tail > 0 && !tail) || (n_rows + n_tail > 0 && !buf)) return NSLAM_EINVAL;
  if (n_rows > 0 && ((((uintptr_t)grid) | ((uintptr_t)buf)) & 15)) return NSLAM_EINVAL;
  const int64_t work = n_rows * (row_len / 4) + n_tail;
  if (work == 0) return NSLAM_OK;
  if ((work + 255) / 256 >= (int64_t(1) << 31)) return NSLAM_EUNSUPPORTED;
  const dim3 g((unsigned)((work + 255) / 256));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (pack)
    hipLaunchKernelGGL(k_rows_xfer<true>, g, dim3(256), 0, s, grid, rows, n_rows, row_len / 4, tail, n_tail, buf);
  else
    hipLaunchKernelGGL(k_rows_xfer<false>, g, dim3(256), 0, s, grid, rows, n_rows, row_len / 4, tail, n_tail, buf);
  return hip_status();
}

}  // namespace

extern "C" int nslam_rows_pack(const float* grid, const int32_t* rows, int64_t n_rows, int32_t row_len,
                               const float* tail, int64_t n_tail, float* out, void* stream) {
  return rows_xfer(true, const_cast<float*>(grid), rows, n_rows, row_len, const_cast<float*>(tail), n_tail, out,
                   stream);
}

extern "C" int nslam_rows_unpack(const float* in, const int32_t* rows, int64_t n_rows, int32_t row_len, float* grid,
                                 float* tail, int64_t n_tail, void* stream) {
  return rows_xfer(false, grid, rows, n_rows, row_len, tail, n_tail, const_cast<float*>(in), stream);
}

extern "C" int nslam_gather_rays(const nslam_frame* frames, int32_t n_frames, int64_t n_per, const int64_t* pix,
                                 int32_t H, int32_t W, int32_t h0, int32_t h1, int32_t w0, int32_t w1, float fx,
                                 float fy, float cx, float cy, const double* bound_lo, const double* bound_hi,
                                 float* rays_o, float* rays_d, float* gt_depth, float* gt_color, uint8_t* keep,
                                 const nslam_draw* draw, int64_t* n_kept, void* stream) {
  if (!frames || n_frames <= 0 || n_frames > NSLAM_MAX_FRAMES || n_per < 0) return NSLAM_EINVAL;
  if (H <= 0 || W <= 0 || h0 < 0 || w0 < 0 || h1 > H || w1 > W || h1 <= h0 || w1 <= w0) return NSLAM_EINVAL;
  if ((bound_lo == nullptr) != (bound_hi == nullptr)) return NSLAM_EINVAL;
  const int64_t n = (int64_t)n_frames * n_per;
  if (n == 0) return NSLAM_OK;
  if ((!pix && !draw) || !rays_o || !rays_d || !gt_depth || !gt_color) return NSLAM_EINVAL;
  if (!pix && (!draw->counter || !draw->ticket)) return NSLAM_EINVAL;
  if (!pix && (draw->world < 1 || draw->rank < 0 || draw->rank >= draw->world)) return NSLAM_EINVAL;
  if (!pix && draw->gt_max && !draw->gt_max_key) return NSLAM_EINVAL;
  GatherArgs a{};
  for (int f = 0; f < n_frames; ++f) {
    if (!frames[f].depth || !frames[f].color || (!frames[f].c2w && !frames[f].cam)) return NSLAM_EINVAL;
    a.fr[f] = frames[f];
  }
  a.nf = n_frames;
  a.n_per = n_per;
  a.n = n;
  a.pix = pix;
  a.W = W;
  a.h0 = h0;
  a.w0 = w0;
  a.ww = w1 - w0;
  a.fx = fx;
  a.fy = fy;
  a.cx = cx;
  a.cy = cy;
  a.use_bound = bound_lo != nullptr;
  for (int k = 0; k < 3 && a.use_bound; ++k) {
    a.lo[k] = bound_lo[k];
    a.hi[k] = bound_hi[k];
  }
  a.ro = rays_o;
  a.rd = rays_d;
  a.gd = gt_depth;
  a.gc = gt_color;
  a.keep = keep;
  if (!pix) {
    a.draw = *draw;
  } else {
    a.draw = nslam_draw{};
    a.draw.world = 1;
  }
  a.wn = (int64_t)(h1 - h0) * (w1 - w0);
  a.n_kept = n_kept;
  hipLaunchKernelGGL(k_gather_rays, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  return hip_status();
}

extern "C" int nslam_adam_step(const nslam_adam_seg* segs, int32_t n_segs, float beta1, float beta2, float eps,
                               int32_t zero_grad, uint32_t* ticket, void* stream) {
  if (!segs || n_segs <= 0 || n_segs > NSLAM_ADAM_MAX_SEGS) return NSLAM_EINVAL;
  AdamArgs a{};
  int64_t blocks = 0;
  for (int s = 0; s < n_segs; ++s) {
    const nslam_adam_seg& g = segs[s];
    if (g.n < 0 || !g.step || (g.n > 0 && (!g.param || !g.grad || !g.exp_avg || !g.exp_avg_sq))) return NSLAM_EINVAL;
    a.seg[s] = g;
    a.blk0[s] = blocks;
    if (g.rows) {
      if (g.row_len <= 0 || g.row_len % 4 || g.row_len / 4 > kAdamThreads) return NSLAM_EINVAL;
      const uintptr_t al = (uintptr_t)g.param | (uintptr_t)g.grad | (uintptr_t)g.exp_avg | (uintptr_t)g.exp_avg_sq;
      if (al & 15) return NSLAM_EINVAL;
    }
    const int64_t nb = adam_segment_blocks<kAdamItems>(g, kAdamThreads);
    blocks += g.n_live ? (nb < kLiveBlocks ? nb : kLiveBlocks) : nb;
  }
  a.blk0[n_segs] = blocks;
  a.nseg = n_segs;
  a.b1 = beta1;
  a.b2 = beta2;
  a.eps = eps;
  a.zero_grad = zero_grad;
  a.ticket = ticket;
  if (blocks == 0) return NSLAM_EINVAL;  // every segment empty: nothing would advance the steps
  if (blocks >= (int64_t(1) << 31)) return NSLAM_EUNSUPPORTED;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(kAdamThreads), 0, s, a);
  if (!ticket) hipLaunchKernelGGL(k_adam_steps, dim3(1), dim3(64), 0, s, a);
  return hip_status();
}

// ------------------------------------------------------------------------------------------
// Camera gradient of a tracking iteration (ABI v8, include/nslam.h nslam_cam_grad)
// ------------------------------------------------------------------------------------------
namespace {

constexpr int kCamThreads = 1024;

struct CamArgs {
  const float* cam;
  const float* c2w;
  const double* g_pts;
  const double* z;
  const float* rd;
  int64_t n;
  int32_t S;
  float* g_cam;
};

// The epilogue both camera-gradient kernels share (one thread): g_R = A·R, the quaternion VJP of
// quad2rotation, and the translation part.  red[k][0], k < 12: Σ g (k < 3) and A (k = 3..11).
__device__ void cam_grad_epilogue(const float* __restrict__ cam, const float* __restrict__ c2w, const double (*red)[kCamThreads / 64],
                                  float* __restrict__ g_cam, float* __restrict__ g_lds = nullptr) {
  struct Ax {
    const float* cam;
    const float* c2w;
    float* g_cam;
  } a{cam, c2w, g_cam};
  double A[9], R[9], gR[9];
  for (int k = 0; k < 9; ++k) A[k] = red[3 + k][0];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[3 * i + j] = a.c2w[4 * i + j];
  for (int i = 0; i < 3; ++i)  // g_R = A · R
    for (int j = 0; j < 3; ++j) gR[3 * i + j] = A[3 * i + 0] * R[j] + A[3 * i + 1] * R[3 + j] + A[3 * i + 2] * R[6 + j];
  // quad2rotation (common.py:150-159): R = I + s P(q), q = (w, x, y, z) = indices 0..3.
  // G[a][b] = Σ_ij gR_ij M_ij,ab with the ±1 terms of each entry of P.
  double G[4][4] = {};
  const double* g = gR;
  G[2][2] -= g[0]; G[3][3] -= g[0];
  G[1][2] += g[1]; G[3][0] -= g[1];
  G[1][3] += g[2]; G[2][0] += g[2];
  G[1][2] += g[3]; G[3][0] += g[3];
  G[1][1] -= g[4]; G[3][3] -= g[4];
  G[2][3] += g[5]; G[1][0] -= g[5];
  G[1][3] += g[6]; G[2][0] -= g[6];
  G[2][3] += g[7]; G[1][0] += g[7];
  G[1][1] -= g[8]; G[2][2] -= g[8];
  double q[4], qq = 0.0;
  for (int k = 0; k < 4; ++k) {
    q[k] = a.cam[k];
    qq += q[k] * q[k];
  }
  const double s = 2.0 / qq;
  double Hq[4], qHq = 0.0;
  for (int i = 0; i < 4; ++i) {
    double h = 0.0;
    for (int j = 0; j < 4; ++j) h += (G[i][j] + G[j][i]) * q[j];
    Hq[i] = h;
    qHq += q[i] * h;
  }
  float gc[7];
  for (int i = 0; i < 4; ++i) gc[i] = (float)(s * Hq[i] - 0.5 * s * s * qHq * q[i]);
  for (int k = 0; k < 3; ++k) gc[4 + k] = (float)red[k][0];
  for (int k = 0; k < 7; ++k) a.g_cam[k] = gc[k];
  if (g_lds)
    for (int k = 0; k < 7; ++k) g_lds[k] = gc[k];
}

__global__ __launch_bounds__(kCamThreads) void k_cam_grad(CamArgs a) {
  // One point per thread per step (coalesced g_pts rows): g_t = Σ g and A = Σ_r g_d,r d_rᵀ, which
  // is linear in the points, = Σ_p (z_p g_p) d_r(p)ᵀ; double partials, wave shuffles, then LDS.
  double acc[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) acc[k] = 0.0;
  const int np = (int)(a.n * a.S);  // 3*np < 2^31 (checked by nslam_cam_grad): 32-bit g_pts offsets
  for (int p = threadIdx.x; p < np; p += kCamThreads) {
    const int r = p / a.S;
    const double zs = a.z[p];
    double g[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      g[k] = a.g_pts[p * 3 + k];
      acc[k] += g[k];
    }
    const double d0 = a.rd[r * 3], d1 = a.rd[r * 3 + 1], d2 = a.rd[r * 3 + 2];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double gz = zs * g[i];
      acc[3 + 3 * i] += gz * d0;
      acc[4 + 3 * i] += gz * d1;
      acc[5 + 3 * i] += gz * d2;
    }
  }
#pragma unroll
  for (int k = 0; k < 12; ++k)
    for (int off = 32; off > 0; off >>= 1) acc[k] += __shfl_xor(acc[k], off, 64);
  __shared__ double red[12][kCamThreads / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 12; ++k) red[k][wave] = acc[k];
  }
  __syncthreads();
  if (threadIdx.x < 12) {  // fixed-order sum over the waves: deterministic
    double t = 0.0;
    for (int w = 0; w < kCamThreads / 64; ++w) t += red[threadIdx.x][w];
    red[threadIdx.x][0] = t;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  cam_grad_epilogue(a.cam, a.c2w, red, a.g_cam);
}

// ABI v15: the same gradient from several d/dpts buffers (the frozen decoders' shares, summed per
// point in buffer order: what the torch adds in front of nslam_cam_grad did, bit for bit) over up to
// kCamParts workgroups; each writes its 12 partial sums to ws, the last to arrive (ticket) adds them
// in workgroup order and runs the epilogue (agent-scope release / acquire around the ticket).
constexpr int kCamParts = 32;
struct CamPartsArgs {
  const float* cam;
  const float* c2w;
  const double* gp[4];
  int32_t nbuf;
  const double* z;
  const float* rd;
  int64_t n;
  int32_t S;
  float* g_cam;
  double* ws;  // [kCamParts][12]
  uint32_t* ticket;
  nslam_cam_tail tail;  // ABI v23 (nslam_cam_grad_step): the camera's Adam step, loss and best pose
  int32_t has_tail;
};

// ABI v23: what follows a tracking iteration's camera gradient, in the workgroup that formed it (all its
// threads): the loss sum (k_loss_sum_best's fixed-order tree over its first kTailSum threads: the same
// value), Adam on the 7-vector (adam_coef / adam_one, one element per thread: k_adam's element update, bit
// for bit), the step count, and the best-pose update with the stepped camera.  The camera, its Adam state,
// the step count and the best loss are loaded before the tree (their latency hides behind it); thread 0's
// epilogue left g_cam in g_lds, published by the tree's barriers.  Every read of *step / *best_loss is
// issued before those barriers, so thread 0 may replace them after.
constexpr int kTailSum = 256;
__device__ void cam_tail(const CamPartsArgs& a, const float* g_lds) {
  const nslam_cam_tail& t = a.tail;
  __shared__ double s[kTailSum];
  const int k = threadIdx.x;
  float p = 0.f, m = 0.f, v = 0.f, stp = 0.f;
  double bl = 0.0;
  if (k < 7) {
    p = t.cam[k];
    m = t.exp_avg[k];
    v = t.exp_avg_sq[k];
    stp = *t.step;
    if (t.best_loss) bl = *t.best_loss;
  }
  if (k < kTailSum) {
    double acc = 0.0;
    for (int64_t i = k; i < t.n_rays; i += kTailSum) acc += t.ray_loss[i];
    s[k] = acc;
  }
  __syncthreads();
  for (int w = kTailSum / 2; w > 0; w >>= 1) {
    if (k < w) s[k] += s[k + w];
    __syncthreads();
  }
  if (k >= 7) return;
  const double l = s[0];
  const bool better = t.best_loss && l < bl;  // (NaN: not better, as torch's comparison)
  const AdamCoef c = adam_coef(t.beta1, t.beta2, t.eps, t.lr, stp);
  adam_one(p, g_lds[k], m, v, c);
  t.cam[k] = p;
  t.exp_avg[k] = m;
  t.exp_avg_sq[k] = v;
  if (better) t.best[k] = p;
  if (k == 0) {
    *t.step = stp + 1.f;
    *t.loss_out = l;
    if (better) *t.best_loss = l;
  }
}

// workgroup wg of nwg of one camera's gradient (k_cam_grad_parts: the whole grid; k_cam_grad_batch: the
// x extent of the grid row of camera blockIdx.y)
__device__ __forceinline__ void cam_grad_parts_body(const CamPartsArgs& a, unsigned wg, unsigned nwg) {
  double acc[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) acc[k] = 0.0;
  const int np = (int)(a.n * a.S);
  for (int p = wg * kCamThreads + threadIdx.x; p < np; p += nwg * kCamThreads) {
    const int r = p / a.S;
    const double zs = a.z[p];
    double g[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      double v = a.gp[0][p * 3 + k];
      for (int b = 1; b < a.nbuf; ++b) v = v + a.gp[b][p * 3 + k];
      g[k] = v;
      acc[k] += v;
    }
    const double d0 = a.rd[r * 3], d1 = a.rd[r * 3 + 1], d2 = a.rd[r * 3 + 2];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double gz = zs * g[i];
      acc[3 + 3 * i] += gz * d0;
      acc[4 + 3 * i] += gz * d1;
      acc[5 + 3 * i] += gz * d2;
    }
  }
#pragma unroll
  for (int k = 0; k < 12; ++k)
    for (int off = 32; off > 0; off >>= 1) acc[k] += __shfl_xor(acc[k], off, 64);
  __shared__ double red[12][kCamThreads / 64];
  __shared__ float g_tail[7];
  float* const g_lds = a.has_tail ? g_tail : nullptr;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 12; ++k) red[k][wave] = acc[k];
  }
  __syncthreads();
  if (nwg == 1) {  // one workgroup: no partials to publish, no hand-over
    if (threadIdx.x < 12) {
      double t = 0.0;
      for (int w = 0; w < kCamThreads / 64; ++w) t += red[threadIdx.x][w];
      red[threadIdx.x][0] = t;
    }
    __syncthreads();
    if (threadIdx.x == 0) cam_grad_epilogue(a.cam, a.c2w, red, a.g_cam, g_lds);
    if (a.has_tail) cam_tail(a, g_lds);
    return;
  }
  if (threadIdx.x < 12) {  // fixed-order sum over the waves, published as this workgroup's partial
    double t = 0.0;
    for (int w = 0; w < kCamThreads / 64; ++w) t += red[threadIdx.x][w];
    a.ws[wg * 12 + threadIdx.x] = t;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t tk = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    red[0][0] = tk == nwg - 1 ? 1.0 : 0.0;  // "I am last", through the one LDS array
  }
  __syncthreads();
  if (red[0][0] == 0.0) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed for the next call
  }
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x < 12)  // the workgroups' partials in workgroup order: deterministic
    for (unsigned w = 0; w < nwg; ++w) t += a.ws[w * 12 + threadIdx.x];
  __syncthreads();
  if (threadIdx.x < 12) red[threadIdx.x][0] = t;
  __syncthreads();
  if (threadIdx.x == 0) cam_grad_epilogue(a.cam, a.c2w, red, a.g_cam, g_lds);
  if (a.has_tail) cam_tail(a, g_lds);
}

__global__ __launch_bounds__(kCamThreads) void k_cam_grad_parts(CamPartsArgs a) { cam_grad_parts_body(a, blockIdx.x, gridDim.x); }

// ABI v19: every bundle-adjustment camera of the window in one launch (grid row blockIdx.y = camera)
struct CamBatchArgs {
  const float* cams;
  const float* c2w;
  int64_t c2w_stride;
  int64_t r0[NSLAM_MAX_FRAMES];  // first ray of each camera's slice
  int64_t n_per;
  const double* gp[4];
  int32_t nbuf;
  const double* z;
  const float* rd;
  int32_t S;
  float* g_cam;
  double* ws;
  uint32_t* tickets;
};

__global__ __launch_bounds__(kCamThreads) void k_cam_grad_batch(CamBatchArgs b) {
  const int k = (int)blockIdx.y;
  int64_t r0 = 0;
#pragma unroll
  for (int i = 0; i < NSLAM_MAX_FRAMES; ++i)  // selects, not a dynamic index into the by-value argument
    if (i == k) r0 = b.r0[i];
  CamPartsArgs a{};
  a.cam = b.cams + 7 * k;
  a.c2w = b.c2w + b.c2w_stride * k;
  const int64_t p0 = r0 * b.S;
#pragma unroll
  for (int i = 0; i < 4; ++i) a.gp[i] = i < b.nbuf ? b.gp[i] + p0 * 3 : nullptr;
  a.nbuf = b.nbuf;
  a.z = b.z + p0;
  a.rd = b.rd + r0 * 3;
  a.n = b.n_per;
  a.S = b.S;
  a.g_cam = b.g_cam + 7 * k;
  a.ws = b.ws + (int64_t)k * kCamParts * 12;
  a.ticket = b.tickets + k;
  cam_grad_parts_body(a, blockIdx.x, gridDim.x);
}

}  // namespace

extern "C" int nslam_cam_grad(const float* cam, const float* c2w, const double* g_pts, const double* z_vals,
                              const float* rays_d, int64_t n_rays, int32_t n_samples, float* g_cam, void* stream) {
  if (!cam || !c2w || !g_cam || n_rays < 0 || n_samples <= 0) return NSLAM_EINVAL;
  if (n_rays > 0 && (!g_pts || !z_vals || !rays_d)) return NSLAM_EINVAL;
  // the kernel indexes g_pts rows as 32-bit p*3+k: the point count must satisfy 3*points < 2^31
  if (n_rays * (int64_t)n_samples * 3 >= (int64_t(1) << 31)) return NSLAM_EUNSUPPORTED;
  CamArgs a{cam, c2w, g_pts, z_vals, rays_d, n_rays, n_samples, g_cam};
  hipLaunchKernelGGL(k_cam_grad, dim3(1), dim3(kCamThreads), 0, reinterpret_cast<hipStream_t>(stream), a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? NSLAM_OK : NSLAM_EHIP - (int)e;
}

namespace {
int cam_grad_parts_launch(const float* cam, const float* c2w, const double* const* g_pts, int32_t n_parts,
                          const double* z_vals, const float* rays_d, int64_t n_rays, int32_t n_samples, float* g_cam,
                          double* ws, uint32_t* ticket, const nslam_cam_tail* tail, void* stream) {
  if (!cam || !c2w || !g_cam || !ticket || !ws || n_rays < 0 || n_samples <= 0) return NSLAM_EINVAL;
  if (n_parts < 1 || n_parts > 4 || !g_pts) return NSLAM_EINVAL;
  if (n_rays > 0 && (!z_vals || !rays_d)) return NSLAM_EINVAL;
  for (int b = 0; b < n_parts; ++b)
    if (!g_pts[b]) return NSLAM_EINVAL;
  if (n_rays * (int64_t)n_samples * 3 >= (int64_t(1) << 31)) return NSLAM_EUNSUPPORTED;
  CamPartsArgs a{};
  a.cam = cam;
  a.c2w = c2w;
  for (int b = 0; b < n_parts; ++b) a.gp[b] = g_pts[b];
  a.nbuf = n_parts;
  a.z = z_vals;
  a.rd = rays_d;
  a.n = n_rays;
  a.S = n_samples;
  a.g_cam = g_cam;
  a.ws = ws;
  a.ticket = ticket;
  if (tail) {
    a.tail = *tail;
    a.has_tail = 1;
  }
  const int64_t np = n_rays * (int64_t)n_samples;
  int64_t wg = (np + kCamThreads - 1) / kCamThreads;
  wg = wg < 1 ? 1 : (wg > kCamParts ? kCamParts : wg);
  hipLaunchKernelGGL(k_cam_grad_parts, dim3((unsigned)wg), dim3(kCamThreads), 0, reinterpret_cast<hipStream_t>(stream), a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? NSLAM_OK : NSLAM_EHIP - (int)e;
}
}  // namespace

extern "C" int nslam_cam_grad_parts(const float* cam, const float* c2w, const double* const* g_pts, int32_t n_parts,
                                    const double* z_vals, const float* rays_d, int64_t n_rays, int32_t n_samples,
                                    float* g_cam, double* ws, uint32_t* ticket, void* stream) {
  return cam_grad_parts_launch(cam, c2w, g_pts, n_parts, z_vals, rays_d, n_rays, n_samples, g_cam, ws, ticket, nullptr,
                               stream);
}

extern "C" int nslam_cam_grad_step(const nslam_cam_tail* tail, const float* c2w, const double* const* g_pts,
                                   int32_t n_parts, const double* z_vals, const float* rays_d, int64_t n_rays,
                                   int32_t n_samples, float* g_cam, double* ws, uint32_t* ticket, void* stream) {
  if (!tail || !tail->cam || !tail->exp_avg || !tail->exp_avg_sq || !tail->step || !tail->loss_out) return NSLAM_EINVAL;
  if (tail->n_rays < 0 || (tail->n_rays > 0 && !tail->ray_loss) || (tail->best_loss && !tail->best)) return NSLAM_EINVAL;
  return cam_grad_parts_launch(tail->cam, c2w, g_pts, n_parts, z_vals, rays_d, n_rays, n_samples, g_cam, ws, ticket,
                               tail, stream);
}

extern "C" int nslam_cam_grad_batch(const float* cams, const float* c2w, int64_t c2w_stride, int32_t n_cams,
                                    const int64_t* ray_begin, int64_t n_rays_per, const double* const* g_pts,
                                    int32_t n_parts, const double* z_vals, const float* rays_d, int64_t n_rays,
                                    int32_t n_samples, float* g_cam, double* ws, uint32_t* tickets, void* stream) {
  if (!cams || !c2w || !g_cam || !ws || !tickets || !ray_begin || n_cams < 1 || n_cams > NSLAM_MAX_FRAMES)
    return NSLAM_EINVAL;
  if (c2w_stride < 12 || n_rays_per < 0 || n_rays < 0 || n_samples <= 0) return NSLAM_EINVAL;
  if (n_parts < 1 || n_parts > 4 || !g_pts) return NSLAM_EINVAL;
  if (n_rays > 0 && (!z_vals || !rays_d)) return NSLAM_EINVAL;
  for (int b = 0; b < n_parts; ++b)
    if (!g_pts[b]) return NSLAM_EINVAL;
  // every slice inside the batch (the kernel reads exactly [ray_begin, ray_begin + n_rays_per) of it)
  for (int k = 0; k < n_cams; ++k)
    if (ray_begin[k] < 0 || ray_begin[k] + n_rays_per > n_rays) return NSLAM_EINVAL;
  if (n_rays * (int64_t)n_samples * 3 >= (int64_t(1) << 31)) return NSLAM_EUNSUPPORTED;
  CamBatchArgs b{};
  b.cams = cams;
  b.c2w = c2w;
  b.c2w_stride = c2w_stride;
  for (int k = 0; k < n_cams; ++k) b.r0[k] = ray_begin[k];
  b.n_per = n_rays_per;
  for (int i = 0; i < n_parts; ++i) b.gp[i] = g_pts[i];
  b.nbuf = n_parts;
  b.z = z_vals;
  b.rd = rays_d;
  b.S = n_samples;
  b.g_cam = g_cam;
  b.ws = ws;
  b.tickets = tickets;
  const int64_t np = n_rays_per * (int64_t)n_samples;
  int64_t wg = (np + kCamThreads - 1) / kCamThreads;
  wg = wg < 1 ? 1 : (wg > kCamParts ? kCamParts : wg);
  hipLaunchKernelGGL(k_cam_grad_batch, dim3((unsigned)wg, (unsigned)n_cams), dim3(kCamThreads), 0,
                     reinterpret_cast<hipStream_t>(stream), b);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? NSLAM_OK : NSLAM_EHIP - (int)e;
}

namespace {


__global__ __launch_bounds__(64) void k_cam_pose(const float* __restrict__ cam, float* __restrict__ c2w) {
  if (threadIdx.x == 0) cam_pose_one(cam, c2w);
}

__global__ __launch_bounds__(64) void k_cam_pose_batch(const float* __restrict__ cams, float* __restrict__ c2w,
                                                       int64_t stride, int n) {
  if ((int)threadIdx.x < n) cam_pose_one(cams + 7 * threadIdx.x, c2w + stride * threadIdx.x);
}

}  // namespace

extern "C" int nslam_cam_pose(const float* cam, float* c2w, void* stream) {
  if (!cam || !c2w) return NSLAM_EINVAL;
  hipLaunchKernelGGL(k_cam_pose, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), cam, c2w);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? NSLAM_OK : NSLAM_EHIP - (int)e;
}

namespace {

// One wave: lanes read the loss and the best loss before lane 0 stores (one instruction stream), so no lane
// sees a half-updated best.
__global__ __launch_bounds__(64) void k_track_best(const double* __restrict__ loss, double* __restrict__ best_loss,
                                                   const float* __restrict__ cam, float* __restrict__ best, int n) {
  const double l = *loss, b = *best_loss;
  if (!(l < b)) return;  // (NaN: not better, as torch's comparison)
  if ((int)threadIdx.x < n) best[threadIdx.x] = cam[threadIdx.x];
  if (threadIdx.x == 0) *best_loss = l;
}

}  // namespace

namespace {
// the loss of a camera iteration (fixed-order sum over one workgroup) and, optionally, the best-pose update
constexpr int kSumThreads = 256;
__global__ __launch_bounds__(kSumThreads) void k_loss_sum_best(const double* __restrict__ rl, int64_t n,
                                                              double* __restrict__ out, double* __restrict__ best_loss,
                                                              const float* __restrict__ cam, float* __restrict__ best,
                                                              int nc) {
  __shared__ double s[kSumThreads];
  double t = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += kSumThreads) t += rl[i];
  s[threadIdx.x] = t;
  __syncthreads();
  for (int w = kSumThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
    __syncthreads();
  }
  const double l = s[0];
  if (threadIdx.x == 0) *out = l;
  if (!best_loss) return;
  if (!(l < *best_loss)) return;  // (NaN: not better, as torch's comparison)
  __syncthreads();                // (every thread has read *best_loss before it is replaced)
  if ((int)threadIdx.x < nc) best[threadIdx.x] = cam[threadIdx.x];
  if (threadIdx.x == 0) *best_loss = l;
}
}  // namespace

extern "C" int nslam_loss_sum_best(const double* ray_loss, int64_t n_rays, double* loss_out, double* best_loss,
                                   const float* cam, float* best, int32_t n, void* stream) {
  if (!loss_out || n_rays < 0 || (n_rays > 0 && !ray_loss)) return NSLAM_EINVAL;
  if (best_loss && (!cam || !best || n < 1 || n > 64)) return NSLAM_EINVAL;
  hipLaunchKernelGGL(k_loss_sum_best, dim3(1), dim3(kSumThreads), 0, reinterpret_cast<hipStream_t>(stream), ray_loss,
                     n_rays, loss_out, best_loss, cam, best, (int)n);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? NSLAM_OK : NSLAM_EHIP - (int)e;
}

extern "C" int nslam_track_best(const double* loss, double* best_loss, const float* cam, float* best, int32_t n,
                                void* stream) {
  if (!loss || !best_loss || !cam || !best || n < 1 || n > 64) return NSLAM_EINVAL;
  hipLaunchKernelGGL(k_track_best, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), loss, best_loss, cam,
                     best, (int)n);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? NSLAM_OK : NSLAM_EHIP - (int)e;
}

namespace {

// get_tensor_from_camera (common.py:179-201) as common.camera_tensors restates it on the device: rotation →
// quaternion (w,x,y,z) by the trace / largest-diagonal branch rule in float64, normalised, w >= 0, then T;
// rounded to float32 once.  NaN compares false (the last branch, as torch.where's) and survives the clamp.
__device__ __forceinline__ void cam_vector_one(const float* __restrict__ M, float* __restrict__ out,
                                               float* __restrict__ out2) {
  const double r00 = M[0], r01 = M[1], r02 = M[2], r10 = M[4], r11 = M[5], r12 = M[6];
  const double r20 = M[8], r21 = M[9], r22 = M[10];
  const double tr = (r00 + r11) + r22;
  auto root = [](double x) { return 2.0 * sqrt(x < 0.0 ? 0.0 : x); };
  double q[4];
  if (tr > 0.0) {
    const double s = root(tr + 1.0);
    q[0] = 0.25 * s; q[1] = (r21 - r12) / s; q[2] = (r02 - r20) / s; q[3] = (r10 - r01) / s;
  } else if (r00 > r11 && r00 > r22) {
    const double s = root(((1.0 + r00) - r11) - r22);
    q[0] = (r21 - r12) / s; q[1] = 0.25 * s; q[2] = (r01 + r10) / s; q[3] = (r02 + r20) / s;
  } else if (r11 > r22) {
    const double s = root(((1.0 + r11) - r00) - r22);
    q[0] = (r02 - r20) / s; q[1] = (r01 + r10) / s; q[2] = 0.25 * s; q[3] = (r12 + r21) / s;
  } else {
    const double s = root(((1.0 + r22) - r00) - r11);
    q[0] = (r10 - r01) / s; q[1] = (r02 + r20) / s; q[2] = (r12 + r21) / s; q[3] = 0.25 * s;
  }
  const double nrm = sqrt(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
  for (int i = 0; i < 4; ++i) q[i] = q[i] / nrm;
  const bool flip = q[0] < 0.0;
  float v[7];
  for (int i = 0; i < 4; ++i) v[i] = (float)(flip ? -q[i] : q[i]);
  v[4] = M[3]; v[5] = M[7]; v[6] = M[11];
  for (int i = 0; i < 7; ++i) out[i] = v[i];
  if (out2)
    for (int i = 0; i < 7; ++i) out2[i] = v[i];
}

__global__ __launch_bounds__(64) void k_cam_vector_batch(const float* __restrict__ c2w, int64_t stride, int n,
                                                         float* __restrict__ cams, float* __restrict__ cams2) {
  const int k = threadIdx.x;
  if (k < n) cam_vector_one(c2w + stride * k, cams + 7 * k, cams2 ? cams2 + 7 * k : nullptr);
}

}  // namespace

extern "C" int nslam_cam_vector_batch(const float* c2w, int64_t c2w_stride, int32_t n, float* cams, float* cams_copy,
                                      void* stream) {
  if (!c2w || !cams || n < 1 || n > 64 || c2w_stride < 12) return NSLAM_EINVAL;
  hipLaunchKernelGGL(k_cam_vector_batch, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), c2w, c2w_stride,
                     (int)n, cams, cams_copy);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? NSLAM_OK : NSLAM_EHIP - (int)e;
}

extern "C" int nslam_cam_pose_batch(const float* cams, float* c2w, int64_t c2w_stride, int32_t n, void* stream) {
  if (!cams || !c2w || n < 1 || n > 64 || c2w_stride < 12) return NSLAM_EINVAL;
  hipLaunchKernelGGL(k_cam_pose_batch, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), cams, c2w,
                     c2w_stride, (int)n);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? NSLAM_OK : NSLAM_EHIP - (int)e;
}
