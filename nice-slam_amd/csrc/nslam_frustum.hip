// nslam_frustum.hip — the frustum voxel selection of Mapper.get_mask_from_c2w (src/Mapper.py:93-164)
// after its two projection GEMMs, fused with the compaction of the selection into the mapping engine's
// capacity-bound row list (ABI v20, include/nslam.h nslam_frustum_rows).
//
// The caller (mapper.frustum_rows_device) forms, with torch's own ops so the values are the
// reference's bit for bit: uvz = ((points @ w2c[:3,:3]ᵀ + w2c[:3,3]).double() * [-1,1,1]) @ Kᵀ (float64)
// and near = |points - t|² < 0.25 (the grid points within 0.5 m of the camera).  Everything after that —
// uv = (uvz[:2] / (uvz[2] + 1e-5)).float(), cv2.remap's bilinear depth lookup (INTER_BITS = 5 fixed-point
// positions, zero border; the same arithmetic as mapper._remap_bilinear), the zero-depth fill with the
// maximum over ALL grid points, the image-bounds and depth tests, the compaction — is here:
//   k_frustum_depth   per point: the remapped depth (float) into ws, and the global max (atomic max on the
//                     float bits: depths are >= 0)
//   k_frustum_mask    per voxel in channels-last order (z*Y + y)*X + x: the mask byte, per-block counts
//   k_frustum_scan    one workgroup: exclusive scan of the block counts, the live count
//   k_frustum_compact per voxel: slot (its rank among selected voxels, or -1) and rows[slot] = voxel
// Rows come out in ascending voxel order: what torch.nonzero of the channels-last mask gives
// (engine.MappingEngine.bind_masks), so the two bindings are interchangeable.  HBM/latency-bound
// elementwise work over the grid's voxel count: no LDS beyond the block scans.
#include <math.h>

#include "nslam_dev.h"

namespace {

constexpr int kFrThreads = 256;

struct FrustumArgs {
  const double* uvz;      // [N][3], reference point order i = (ix*ny + iy)*nz + iz
  const uint8_t* near;    // [N] bool, reference order
  const float* depth;     // [H][W]
  int32_t H, W;
  int32_t nx, ny, nz;
  int64_t n;
  float* dws;             // [N] remapped depth (reference order)
  uint32_t* dmax;         // float bits of the max depth
  uint8_t* mcl;           // [N] mask, channels-last order
  int32_t* counts;        // [nblocks] selected voxels per block (then exclusive offsets)
  int32_t* slot;          // [N] channels-last
  int32_t* rows;          // [N]
  int64_t* n_live;
  uint8_t* mask_ref;      // optional [N] reference-order mask
};

__device__ __forceinline__ float tap(const FrustumArgs& a, int64_t x, int64_t y) {
  return (x >= 0 && x < a.W && y >= 0 && y < a.H) ? a.depth[y * a.W + x] : 0.f;
}

// uv of point i (mapper.frustum_mask: z = uvz[:, 2] + 1e-5; uv = (uvz[:, :2] / z).float())
__device__ __forceinline__ void point_uv(const FrustumArgs& a, int64_t i, float& u, float& v, double& z) {
  const double* p = a.uvz + 3 * i;
  z = p[2] + 1e-5;
  u = (float)(p[0] / z);
  v = (float)(p[1] / z);
}

// mapper._remap_bilinear: X = round(clamp(u) * 32) (half to even), x0 = floor(X / 32), fx = (X - 32 x0) / 32
__device__ __forceinline__ float remap_depth(const FrustumArgs& a, float u, float v) {
  const float uc = fminf(fmaxf(u, -1e8f), 1e8f), vc = fminf(fmaxf(v, -1e8f), 1e8f);
  const int64_t X = (int64_t)rintf(uc * 32.f), Y = (int64_t)rintf(vc * 32.f);
  const int64_t x0 = X >> 5, y0 = Y >> 5;  // floor division by 32
  const float fx = (float)(X - x0 * 32) / 32.f, fy = (float)(Y - y0 * 32) / 32.f;
  const float w00 = (1.f - fx) * (1.f - fy), w01 = fx * (1.f - fy);
  const float w10 = (1.f - fx) * fy, w11 = fx * fy;
  return ((tap(a, x0, y0) * w00 + tap(a, x0 + 1, y0) * w01) + tap(a, x0, y0 + 1) * w10) + tap(a, x0 + 1, y0 + 1) * w11;
}

__global__ __launch_bounds__(kFrThreads) void k_frustum_depth(FrustumArgs a) {
  const int64_t i = (int64_t)blockIdx.x * kFrThreads + threadIdx.x;
  float d = 0.f;
  if (i < a.n) {
    float u, v;
    double z;
    point_uv(a, i, u, v, z);
    d = remap_depth(a, u, v);
    a.dws[i] = d;
  }
  // block max of the (non-negative) depths, one atomic per wave
  uint32_t m = __float_as_uint(fmaxf(d, 0.f));
  for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
  if ((threadIdx.x & 63) == 0 && m) atomicMax(a.dmax, m);
}

__global__ __launch_bounds__(kFrThreads) void k_frustum_mask(FrustumArgs a) {
  const int64_t v = (int64_t)blockIdx.x * kFrThreads + threadIdx.x;  // channels-last voxel
  bool sel = false;
  if (v < a.n) {
    const int64_t ix = v % a.nx, iy = (v / a.nx) % a.ny, iz = v / ((int64_t)a.nx * a.ny);
    const int64_t i = (ix * a.ny + iy) * a.nz + iz;
    float u, vv;
    double z;
    point_uv(a, i, u, vv, z);
    float d = a.dws[i];
    if (d == 0.f) d = __uint_as_float(*a.dmax);  // depths[depths == 0] = max(depths)
    const bool img = (u < (float)a.W) & (u > 0.f) & (vv < (float)a.H) & (vv > 0.f);
    sel = (img & (0.0 <= -z) & (-z <= (double)d + 0.5)) | (a.near[i] != 0);
    a.mcl[v] = sel ? 1 : 0;
    if (a.mask_ref) a.mask_ref[i] = sel ? 1 : 0;
  }
  __shared__ int wc[kFrThreads / 64];
  const int c = __popcll(__ballot(sel));
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < kFrThreads / 64; ++w) t += wc[w];
    a.counts[blockIdx.x] = t;
  }
}

// one workgroup: counts -> exclusive offsets (in place), total -> n_live (chunks of 1024 with a carry)
__global__ __launch_bounds__(1024) void k_frustum_scan(int32_t* counts, int64_t nblocks, int64_t* n_live) {
  __shared__ int32_t s[1024];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < nblocks; base += 1024) {
    const int64_t j = base + threadIdx.x;
    const int32_t x = j < nblocks ? counts[j] : 0;
    s[threadIdx.x] = x;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
      const int32_t y = threadIdx.x >= (unsigned)off ? s[threadIdx.x - off] : 0;
      __syncthreads();
      s[threadIdx.x] += y;
      __syncthreads();
    }
    if (j < nblocks) counts[j] = (int32_t)(carry + s[threadIdx.x] - x);
    __syncthreads();
    if (threadIdx.x == 1023) carry += s[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) *n_live = carry;
}

__global__ __launch_bounds__(kFrThreads) void k_frustum_compact(FrustumArgs a) {
  const int64_t v = (int64_t)blockIdx.x * kFrThreads + threadIdx.x;
  const bool sel = v < a.n && a.mcl[v];
  const uint64_t b = __ballot(sel);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ int wc[kFrThreads / 64];
  if (lane == 0) wc[wave] = __popcll(b);
  __syncthreads();
  int off = a.counts[blockIdx.x];
  for (int w = 0; w < wave; ++w) off += wc[w];
  if (v < a.n) {
    const int r = off + __popcll(b & ((1ull << lane) - 1ull));
    a.slot[v] = sel ? r : -1;
    if (sel) a.rows[r] = (int32_t)v;
  }
}

}  // namespace

extern "C" size_t nslam_frustum_rows_workspace_size(int64_t n_vox) {
  if (n_vox <= 0) return 0;
  const int64_t nb = (n_vox + kFrThreads - 1) / kFrThreads;
  const size_t al = 256;
  const size_t dws = ((size_t)n_vox * 4 + al - 1) / al * al;
  const size_t mcl = ((size_t)n_vox + al - 1) / al * al;
  const size_t cnt = ((size_t)nb * 4 + al - 1) / al * al;
  return dws + mcl + cnt + al;  // + the max word
}

extern "C" int nslam_frustum_rows(const double* uvz, const uint8_t* near, const float* depth, int32_t H, int32_t W,
                                  int32_t nx, int32_t ny, int32_t nz, int32_t* slot, int32_t* rows, int64_t* n_live,
                                  uint8_t* mask_ref, void* ws, size_t ws_bytes, void* stream) {
  if (!uvz || !near || !depth || !slot || !rows || !n_live || H <= 0 || W <= 0 || nx <= 0 || ny <= 0 || nz <= 0)
    return NSLAM_EINVAL;
  const int64_t n = (int64_t)nx * ny * nz;
  if (n >= (int64_t(1) << 31)) return NSLAM_EUNSUPPORTED;  // int32 rows
  if (!ws || ws_bytes < nslam_frustum_rows_workspace_size(n)) return NSLAM_EWORKSPACE;
  const int64_t nb = (n + kFrThreads - 1) / kFrThreads;
  const size_t al = 256;
  char* w = static_cast<char*>(ws);
  FrustumArgs a{};
  a.uvz = uvz;
  a.near = near;
  a.depth = depth;
  a.H = H;
  a.W = W;
  a.nx = nx;
  a.ny = ny;
  a.nz = nz;
  a.n = n;
  a.dws = reinterpret_cast<float*>(w);
  w += ((size_t)n * 4 + al - 1) / al * al;
  a.mcl = reinterpret_cast<uint8_t*>(w);
  w += ((size_t)n + al - 1) / al * al;
  a.counts = reinterpret_cast<int32_t*>(w);
  w += ((size_t)nb * 4 + al - 1) / al * al;
  a.dmax = reinterpret_cast<uint32_t*>(w);
  a.slot = slot;
  a.rows = rows;
  a.n_live = n_live;
  a.mask_ref = mask_ref;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(a.dmax, 0, 4, s) != hipSuccess) return NSLAM_EHIP - (int)hipGetLastError();
  const dim3 g((unsigned)nb), b(kFrThreads);
  hipLaunchKernelGGL(k_frustum_depth, g, b, 0, s, a);
  hipLaunchKernelGGL(k_frustum_mask, g, b, 0, s, a);
  hipLaunchKernelGGL(k_frustum_scan, dim3(1), dim3(1024), 0, s, a.counts, nb, n_live);
  hipLaunchKernelGGL(k_frustum_compact, g, b, 0, s, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? NSLAM_OK : NSLAM_EHIP - (int)e;
}
