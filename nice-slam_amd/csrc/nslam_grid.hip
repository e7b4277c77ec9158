// nslam_grid.hip — standalone trilinear feature lookup on a channels-last grid (gfx950).
//
// F.grid_sample(grid[1,32,D,H,W], coords[1,M,1,1,3], mode='bilinear', padding_mode='border',
// align_corners=True) as called by sample_grid_feature (src/conv_onet/models/decoder.py:168-175),
// forward and backward (grid scatter + coordinate gradient).  The fused query kernels
// (nslam_query.hip) inline the same corner math; this entry point is the unit that is
// parity-tested against F.grid_sample and measured against the HBM roofline in isolation.
//
// Forward: 8 lanes per point, each lane one float4 (16 B) of the 128-B corner row: a corner read
// is one fully used 128-B line; the 128-B output row is written by the same 8 lanes.
// Backward: 32 lanes per point, one channel each, so every atomic wave-instruction is two 128-B
// row segments (the full-rate atomic shape on MI355X).
#include "nslam_dev.h"

namespace {

__global__ __launch_bounds__(256) void k_grid_fwd(const float* __restrict__ grid, int D, int H, int W,
                                                  const float* __restrict__ coords, int64_t n,
                                                  float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t p = t >> 3;
  const int q = (int)(t & 7);  // float4 slot within the 32 channels
  if (p >= n) return;
  const float nc3[3] = {coords[p * 3 + 0], coords[p * 3 + 1], coords[p * 3 + 2]};
  const int32_t dims[3] = {D, H, W};
  Corners c;
  make_corners(c, nc3, dims);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(grid + (size_t)c.row[k] * NSLAM_C_DIM + 4 * q);
    acc += v * c.w[k];
  }
  *reinterpret_cast<f32x4*>(out + p * NSLAM_C_DIM + 4 * q) = acc;
}

__global__ __launch_bounds__(256) void k_grid_bwd(const float* __restrict__ grid, int D, int H, int W,
                                                  const float* __restrict__ coords, int64_t n,
                                                  const float* __restrict__ gout, float* __restrict__ ggrid,
                                                  float* __restrict__ gcoord) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t p = t >> 5;
  const int ch = (int)(t & 31);
  const bool valid = p < n;
  const int64_t pp = valid ? p : 0;
  const float nc3[3] = {coords[pp * 3 + 0], coords[pp * 3 + 1], coords[pp * 3 + 2]};
  const int32_t dims[3] = {D, H, W};
  Corners c;
  make_corners(c, nc3, dims);
  const float g = valid ? gout[pp * NSLAM_C_DIM + ch] : 0.f;
  float gx = 0.f, gy = 0.f, gz = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const bool ok = (c.ok >> k) & 1u;
    if (ggrid && valid && ok) unsafeAtomicAdd(ggrid + (size_t)c.row[k] * NSLAM_C_DIM + ch, c.w[k] * g);
    if (gcoord) {
      const float v = ok ? grid[(size_t)c.row[k] * NSLAM_C_DIM + ch] * g : 0.f;
      const int dx = k & 1, dy = (k >> 1) & 1, dz = k >> 2;
      const float fx = dx ? c.f1[0] : c.f0[0], fy = dy ? c.f1[1] : c.f0[1], fz = dz ? c.f1[2] : c.f0[2];
      gx += (dx ? 1.f : -1.f) * (fy * fz) * v;
      gy += (dy ? 1.f : -1.f) * (fx * fz) * v;
      gz += (dz ? 1.f : -1.f) * (fx * fy) * v;
    }
  }
  if (gcoord) {
#pragma unroll
    for (int d = 16; d >= 1; d >>= 1) {
      gx += __shfl_xor(gx, d, 64);
      gy += __shfl_xor(gy, d, 64);
      gz += __shfl_xor(gz, d, 64);
    }
    if (ch == 0 && valid) {
      gcoord[p * 3 + 0] = gx * c.gmul[0];
      gcoord[p * 3 + 1] = gy * c.gmul[1];
      gcoord[p * 3 + 2] = gz * c.gmul[2];
    }
  }
}

int hip_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? NSLAM_OK : NSLAM_EHIP - (int)e;
}

}  // namespace

extern "C" int nslam_grid_sample_fwd(const float* grid, const int32_t* dims, const float* coords, int64_t n,
                                     float* out, void* stream) {
  if (!dims || n < 0) return NSLAM_EINVAL;
  if (n == 0) return NSLAM_OK;
  if (!grid || !coords || !out || dims[0] <= 0 || dims[1] <= 0 || dims[2] <= 0) return NSLAM_EINVAL;
  if ((((uintptr_t)grid) | ((uintptr_t)out)) & 15) return NSLAM_EINVAL;
  const int64_t threads = n * 8;
  hipLaunchKernelGGL(k_grid_fwd, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), grid, dims[0], dims[1], dims[2], coords, n, out);
  return hip_status();
}

extern "C" int nslam_grid_sample_bwd(const float* grid, const int32_t* dims, const float* coords, int64_t n,
                                     const float* grad_out, float* grad_grid, float* grad_coords, void* stream) {
  if (!dims || n < 0) return NSLAM_EINVAL;
  if (n == 0) return NSLAM_OK;
  if (!grid || !coords || !grad_out || dims[0] <= 0 || dims[1] <= 0 || dims[2] <= 0) return NSLAM_EINVAL;
  const int64_t threads = n * 32;
  hipLaunchKernelGGL(k_grid_bwd, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), grid, dims[0], dims[1], dims[2], coords, n, grad_out,
                     grad_grid, grad_coords);
  return hip_status();
}
