// nslam_dev.h — device-side building blocks shared by the gfx950 kernels of libnslam.so.
//
// Conventions (CDNA4, wave64, v_mfma_f32_32x32x2_f32):
//   A "feature tile" is 32 features x 32 points held as one f32x16 accumulator in the MFMA C/D
//   layout: lane l = (h = l>>5, p = l&31) holds point p, register r holds feature
//   F(r,h) = (r&3) + 8*(r>>2) + 4*h.  Because the B operand of step s of a 32x32x2 MFMA is
//   "row k = l>>5, column j = l&31", register s of a feature tile IS the B operand of step s when
//   the K order of that step is {F(s,0), F(s,1)}.  So a layer Y = W*X chains tile -> tile with no
//   data movement: A of step s in lane l is W[l&31][F(s, l>>5)] (pre-packed "fragment", 16
//   floats per lane, 4 x dwordx4), B is X.reg[s].  The transposed product W^T*dY (backward)
//   uses the same scheme with fragments W[F(s,l>>5)][l&31].
//   Weight gradients sum over POINTS, so both operands are moved through LDS as [point][feature]
//   images (row pitch 33 floats: conflict-free ds_write_b32 of the C layout and ds_read_b32 of
//   the A/B layout).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nslam.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

#define NSLAM_FRAG 1024  // floats per packed fragment block (16 steps x 64 lanes)
#define TPITCH 33        // LDS row pitch of a transposed tile [32 points][33]
#define TILE_FLOATS (32 * TPITCH)

// ------------------------------------------------------------------------------------------
// pack layouts (single source of truth; exported to the host through nslam_pack_layout)
// ------------------------------------------------------------------------------------------
struct XyzPack {  // MLP with Fourier embedding (decoder.py:91-203); nc = feature blocks (1|2)
  int nc;
  __host__ __device__ constexpr int nf() const { return 10 + 5 * nc; }
  __host__ __device__ constexpr int L0() const { return 0; }   // 3 blocks (emb 96)
  __host__ __device__ constexpr int L1() const { return 3; }
  __host__ __device__ constexpr int L2() const { return 4; }
  __host__ __device__ constexpr int L3() const { return 5; }   // 4 blocks (emb 96 | h2 32)
  __host__ __device__ constexpr int L4() const { return 9; }
  __host__ __device__ constexpr int FC(int i, int c) const { return 10 + i * nc + c; }
  __host__ __device__ constexpr int L0T() const { return nf(); }       // 3 blocks
  __host__ __device__ constexpr int L1T() const { return nf() + 3; }
  __host__ __device__ constexpr int L2T() const { return nf() + 4; }
  __host__ __device__ constexpr int L3T() const { return nf() + 5; }   // 4 blocks
  __host__ __device__ constexpr int L4T() const { return nf() + 9; }
  __host__ __device__ constexpr int FCT(int i) const { return nf() + 10 + i; }  // feature block 0
  __host__ __device__ constexpr int nfrag() const { return nf() + 15; }
  __host__ __device__ constexpr int V() const { return nfrag() * NSLAM_FRAG; }
  __host__ __device__ constexpr int Bias(int i) const { return V() + 32 * i; }
  __host__ __device__ constexpr int BiasC(int i) const { return V() + 160 + 32 * i; }
  __host__ __device__ constexpr int Wo() const { return V() + 320; }  // [4][32]
  __host__ __device__ constexpr int Bo() const { return V() + 448; }  // [4]
  __host__ __device__ constexpr int FB() const { return V() + 452; }  // [3][96]
  __host__ __device__ constexpr int total() const { return V() + 740; }
};

struct NoXyzPack {  // MLP_no_xyz (decoder.py:206-274), coarse level
  __host__ __device__ constexpr int L0() const { return 0; }
  __host__ __device__ constexpr int L1() const { return 1; }
  __host__ __device__ constexpr int L2() const { return 2; }
  __host__ __device__ constexpr int L3() const { return 3; }  // 2 blocks (c | h2)
  __host__ __device__ constexpr int L4() const { return 5; }
  __host__ __device__ constexpr int nf() const { return 6; }
  __host__ __device__ constexpr int L0T() const { return 6; }
  __host__ __device__ constexpr int L1T() const { return 7; }
  __host__ __device__ constexpr int L2T() const { return 8; }
  __host__ __device__ constexpr int L3T() const { return 9; }  // 2 blocks
  __host__ __device__ constexpr int L4T() const { return 11; }
  __host__ __device__ constexpr int nfrag() const { return 12; }
  __host__ __device__ constexpr int V() const { return nfrag() * NSLAM_FRAG; }
  __host__ __device__ constexpr int Bias(int i) const { return V() + 32 * i; }
  __host__ __device__ constexpr int Wo() const { return V() + 160; }
  __host__ __device__ constexpr int Bo() const { return V() + 288; }
  __host__ __device__ constexpr int total() const { return V() + 292; }
};

// ------------------------------------------------------------------------------------------
// MFMA tile helpers
// ------------------------------------------------------------------------------------------
// order-preserving float <-> uint (atomicMax over a batch of floats; key 0 is below every float)
__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
// Wave index inside the workgroup as a wave-uniform (SGPR) value: LLVM's divergence analysis
// treats threadIdx.x >> 6 as divergent, which would push every tile / slab address derived from
// it into VGPRs (and buffer resources into waterfall loops).
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
__device__ __forceinline__ int fidx(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// Global-address-space view of a pointer into device memory.  A pointer read out of the kernel
// argument struct by a runtime index, or laundered through an asm constraint, is generic to the
// compiler, and a generic access is a flat_* instruction — which counts in LGKM_CNT as well as
// VM_CNT, so every LDS wait (s_waitcnt lgkmcnt(0)) also drains the loads in flight (the weight
// fragments, the activation tape), and every use of a flat-loaded value waits for all LDS traffic.
// Through this view the same accesses are global_* (VM_CNT only).
template <class T>
using gptr_t = const __attribute__((address_space(1))) T*;
template <class T>
__device__ __forceinline__ gptr_t<T> as_global(const T* p) {
  return (gptr_t<T>)p;
}
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* as_global_w(T* p) {
  return (__attribute__((address_space(1))) T*)p;
}

// acc += Wblock * X   (frag: packed [lane][16], global memory)
__device__ __forceinline__ void gemm_acc(f32x16& acc, const float* __restrict__ frag, const f32x16& x,
                                         int lane) {
  const gptr_t<f32x4> f = as_global(reinterpret_cast<const f32x4*>(frag)) + lane * 4;
  const f32x4 a0 = f[0], a1 = f[1], a2 = f[2], a3 = f[3];
  acc = mfma32(a0[0], x[0], acc);
  acc = mfma32(a0[1], x[1], acc);
  acc = mfma32(a0[2], x[2], acc);
  acc = mfma32(a0[3], x[3], acc);
  acc = mfma32(a1[0], x[4], acc);
  acc = mfma32(a1[1], x[5], acc);
  acc = mfma32(a1[2], x[6], acc);
  acc = mfma32(a1[3], x[7], acc);
  acc = mfma32(a2[0], x[8], acc);
  acc = mfma32(a2[1], x[9], acc);
  acc = mfma32(a2[2], x[10], acc);
  acc = mfma32(a2[3], x[11], acc);
  acc = mfma32(a3[0], x[12], acc);
  acc = mfma32(a3[1], x[13], acc);
  acc = mfma32(a3[2], x[14], acc);
  acc = mfma32(a3[3], x[15], acc);
}

// acc += (W^T X) TRANSPOSED: the backward fragment W[F(s,h)][k] as the B operand and the C-layout tile X
// (lane (p, h), register s = X[p][F(s, h)]) as the A operand, so D[i = point][j = k] = Σ_o X[p][o] W[o][k]
// lands as lane (k, h') register r = point F(r, h') — the MFMA with its operands swapped
__device__ __forceinline__ void gemm_acc_t(f32x16& acc, const float* __restrict__ frag, const f32x16& x, int lane) {
  const gptr_t<f32x4> f = as_global(reinterpret_cast<const f32x4*>(frag)) + lane * 4;
  const f32x4 a0 = f[0], a1 = f[1], a2 = f[2], a3 = f[3];
#pragma unroll
  for (int k = 0; k < 4; ++k) acc = mfma32(x[k], a0[k], acc);
#pragma unroll
  for (int k = 0; k < 4; ++k) acc = mfma32(x[4 + k], a1[k], acc);
#pragma unroll
  for (int k = 0; k < 4; ++k) acc = mfma32(x[8 + k], a2[k], acc);
#pragma unroll
  for (int k = 0; k < 4; ++k) acc = mfma32(x[12 + k], a3[k], acc);
}

// acc += Wblock * X in the C layout (TR false) or its transpose (TR true: gemm_acc_t)
template <bool TR>
__device__ __forceinline__ void gemm_acc_tr(f32x16& acc, const float* __restrict__ frag, const f32x16& x, int lane) {
  if (TR)
    gemm_acc_t(acc, frag, x, lane);
  else
    gemm_acc(acc, frag, x, lane);
}


// A weight fragment (16 floats per lane) held in registers, so a GEMM's fragment can be in flight
// while the previous GEMM runs
struct Frag {
  f32x4 q[4];
};
__device__ __forceinline__ Frag load_frag(const float* __restrict__ frag, int lane) {
  const gptr_t<f32x4> f = as_global(reinterpret_cast<const f32x4*>(frag)) + lane * 4;
  return Frag{{f[0], f[1], f[2], f[3]}};
}
// acc += W X from a loaded fragment (gemm_acc's MFMA chain)
__device__ __forceinline__ void gemm_frag(f32x16& acc, const Frag& f, const f32x16& x) {
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = mfma32(f.q[s >> 2][s & 3], x[s], acc);
}
// A fixed sequence of GEMMs over one decoder's packed fragments with each fragment loaded one GEMM
// ahead: gemm(acc, x, next) runs acc += W_cur X while the fragment of block `next` (< 0: none) loads.
// The fence after the load keeps the compiler from sinking it to its use (the MFMAs of the current
// GEMM wait only for the current fragment: vmcnt counts in order, the younger load stays in flight).
struct FragPipe {
  const float* pk;
  int lane;
  Frag cur;
  __device__ __forceinline__ FragPipe(const float* pk_, int first, int lane_)
      : pk(pk_), lane(lane_), cur(load_frag(pk_ + first * NSLAM_FRAG, lane_)) {}
  __device__ __forceinline__ void gemm(f32x16& acc, const f32x16& x, int next) {
    Frag n = cur;
    if (next >= 0) n = load_frag(pk + next * NSLAM_FRAG, lane);
    __builtin_amdgcn_sched_barrier(0);
    gemm_frag(acc, cur, x);
    cur = n;
  }
};

// feature-tile view of a natural [32] vector: v[F(r,h)]
__device__ __forceinline__ f32x16 vec_tile(const float* __restrict__ v, int lane) {
  const int h = lane >> 5;
  f32x16 t;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x4 q = *reinterpret_cast<const f32x4*>(v + 8 * i + 4 * h);
    t[4 * i + 0] = q[0];
    t[4 * i + 1] = q[1];
    t[4 * i + 2] = q[2];
    t[4 * i + 3] = q[3];
  }
  return t;
}
// vec_tile of a vector in global memory (global_load, not flat)
__device__ __forceinline__ f32x16 vec_tile_g(const float* __restrict__ v, int lane) {
  const int h = lane >> 5;
  f32x16 t;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x4 q = *as_global(reinterpret_cast<const f32x4*>(v + 8 * i + 4 * h));
    t[4 * i + 0] = q[0];
    t[4 * i + 1] = q[1];
    t[4 * i + 2] = q[2];
    t[4 * i + 3] = q[3];
  }
  return t;
}

// ReLU and its mask on the float's bits (both equal `a > 0 ? a : +0` and `a > 0` for every non-NaN a,
// -0 included): relu is one v_max_i32 per register, the mask bit one v_med3_i32 (clamp to [0, 1]) and
// one v_lshl_or per register.  A float compare would produce a 64-bit lane mask per register in SGPRs
// (16 per layer), which the forward's chains spilled into VGPR lanes.
__device__ __forceinline__ f32x16 relu16(const f32x16& a) {
  f32x16 o;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int v = __builtin_bit_cast(int, (float)a[r]);
    o[r] = __builtin_bit_cast(float, v > 0 ? v : 0);
  }
  return o;
}

// bit R of m = (a > 0): clamp the bits to [0, 1] and shift-or it in, in one asm statement so the bit is
// folded into m at once (as separate operations the compiler kept 16 bits live per layer)
template <int R>
__device__ __forceinline__ void mask_bit(uint32_t& m, float a) {
  int t;
  asm("v_med3_i32 %1, %2, 0, 1\n\tv_lshl_or_b32 %0, %1, %3, %0"
      : "+v"(m), "=&v"(t)
      : "v"(__builtin_bit_cast(int, a)), "n"(R));
}
__device__ __forceinline__ uint32_t mask16(const f32x16& a) {
  uint32_t m = 0;
  mask_bit<0>(m, a[0]);
  mask_bit<1>(m, a[1]);
  mask_bit<2>(m, a[2]);
  mask_bit<3>(m, a[3]);
  mask_bit<4>(m, a[4]);
  mask_bit<5>(m, a[5]);
  mask_bit<6>(m, a[6]);
  mask_bit<7>(m, a[7]);
  mask_bit<8>(m, a[8]);
  mask_bit<9>(m, a[9]);
  mask_bit<10>(m, a[10]);
  mask_bit<11>(m, a[11]);
  mask_bit<12>(m, a[12]);
  mask_bit<13>(m, a[13]);
  mask_bit<14>(m, a[14]);
  mask_bit<15>(m, a[15]);
  return m;
}

// g where bit r of m is set, else +0: a sign-extended bit field (v_bfe_i32: 0 or -1) ANDed into the bits
// (no per-register compare, i.e. no SGPR lane mask per register)
__device__ __forceinline__ f32x16 apply_mask(const f32x16& g, uint32_t m) {
  f32x16 o;
#pragma unroll
  for (int r = 0; r < 16; ++r)
    o[r] = __builtin_bit_cast(float, __builtin_bit_cast(int, (float)g[r]) & __builtin_amdgcn_sbfe((int)m, r, 1));
  return o;
}

// store a C-layout tile as a [point][feature] LDS image (pitch 33)
__device__ __forceinline__ void tstore(float* s, const f32x16& v, int lane) {
  const int p = lane & 31, h = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) s[p * TPITCH + fidx(r, h)] = v[r];
}

// read a C-layout tile back from a [point][feature] LDS image (inverse of tstore)
__device__ __forceinline__ f32x16 tload(const float* s, int lane) {
  const int p = lane & 31, h = lane >> 5;
  f32x16 v;
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = s[p * TPITCH + fidx(r, h)];
  return v;
}

// value of lane l ^ 32: one v_permlane32_swap (gfx950; swaps the upper half of its first operand
// with the lower half of its second) and a half select, instead of an LDS ds_bpermute round trip
__device__ __forceinline__ unsigned xor32u(unsigned v) {
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (threadIdx.x & 32) ? r[0] : r[1];
}
__device__ __forceinline__ float xor32(float v) {
  return __builtin_bit_cast(float, xor32u(__builtin_bit_cast(unsigned, v)));
}
__device__ __forceinline__ double xor32d(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = xor32u((unsigned)u), hi = xor32u((unsigned)(u >> 32));
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// ------------------------------------------------------------------------------------------
// trilinear corners (F.grid_sample 5-D, bilinear, padding 'border', align_corners=True)
// ------------------------------------------------------------------------------------------
struct Corners {
  int32_t row[8];  // corner row index (z*H + y)*W + x; 0 when the corner is out of range
  float w[8];      // weight ((wx*wy)*wz); exactly 0 for out-of-range corners
  float f0[3], f1[3];  // (lo-side, hi-side) linear factors per axis x,y,z
  float gmul[3];   // d(unnormalised)/d(normalised) incl. the clip gate: 0 or (n-1)/2
  uint32_t ok;     // bit k: corner k is inside the grid (torch's within_bounds_3d)
  int32_t cell;    // lower-corner voxel coordinates ix | iy << 10 | iz << 20 (dims <= 1024)
};

// normalised coordinate of axis a (decoder.py:169 → common.py:269-284), float64 then .float()
__device__ __forceinline__ float norm_coord(double p, double lo, double hi) {
  const double ext = hi - lo;
  return (float)(((p - lo) / ext) * 2.0 - 1.0);
}

// grid_sampler_compute_source_index with its gradient gate, per axis
__device__ __forceinline__ float unnorm_clip(float c, int n, float& gmul) {
  float u = ((c + 1.f) / 2.f) * (float)(n - 1);
  gmul = (float)(n - 1) / 2.f;
  if (u <= 0.f) {
    u = 0.f;
    gmul = 0.f;
  } else if (u >= (float)(n - 1)) {
    u = (float)(n - 1);
    gmul = 0.f;
  }
  return u;
}

// nc3 = normalised (x,y,z); dims = Z,Y,X
__device__ __forceinline__ void make_corners(Corners& c, const float nc3[3], const int32_t dims[3]) {
  const int n[3] = {dims[2], dims[1], dims[0]};  // x→W, y→H, z→D
  int i0[3];
  bool hi_ok[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float u = unnorm_clip(nc3[a], n[a], c.gmul[a]);
    const float fl = floorf(u);
    i0[a] = (int)fl;
    c.f1[a] = u - fl;                      // (ix - ix_tnw)
    c.f0[a] = (float)(i0[a] + 1) - u;      // (ix_bse - ix)
    hi_ok[a] = (i0[a] + 1) <= n[a] - 1;
  }
  c.cell = i0[0] | (i0[1] << 10) | (i0[2] << 20);
  c.ok = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int dx = k & 1, dy = (k >> 1) & 1, dz = k >> 2;
    const bool ok = (!dx || hi_ok[0]) && (!dy || hi_ok[1]) && (!dz || hi_ok[2]);
    c.ok |= (ok ? 1u : 0u) << k;
    const float w = ((dx ? c.f1[0] : c.f0[0]) * (dy ? c.f1[1] : c.f0[1])) * (dz ? c.f1[2] : c.f0[2]);
    c.w[k] = ok ? w : 0.f;
    c.row[k] = ok ? ((i0[2] + dz) * n[1] + (i0[1] + dy)) * n[0] + (i0[0] + dx) : 0;
  }
}

// gather this lane's 16 channels (F(r,h) layout) of the trilinear feature
__device__ __forceinline__ f32x16 gather_tile(const float* __restrict__ grid, const Corners& c, int lane) {
  const int h = lane >> 5;
  f32x16 acc = zero16();
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const gptr_t<f32x4> row = as_global(reinterpret_cast<const f32x4*>(grid + (size_t)c.row[k] * NSLAM_C_DIM + 4 * h));
    const f32x4 v0 = row[0], v1 = row[2], v2 = row[4], v3 = row[6];
    const float w = c.w[k];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[j] += v0[j] * w;
      acc[4 + j] += v1[j] * w;
      acc[8 + j] += v2[j] * w;
      acc[12 + j] += v3[j] * w;
    }
  }
  return acc;
}

// gather_tile with at most NB corners' loads in flight (a scheduling fence between batches): for a
// gather whose result is only stored, in a kernel whose register budget is set elsewhere
template <int NB>
__device__ __forceinline__ f32x16 gather_tile_batched(const float* __restrict__ grid, const Corners& c, int lane) {
  const int h = lane >> 5;
  f32x16 acc = zero16();
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (k % NB == 0) __builtin_amdgcn_sched_barrier(0);
    const gptr_t<f32x4> row = as_global(reinterpret_cast<const f32x4*>(grid + (size_t)c.row[k] * NSLAM_C_DIM + 4 * h));
    const f32x4 v0 = row[0], v1 = row[2], v2 = row[4], v3 = row[6];
    const float w = c.w[k];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[j] += v0[j] * w;
      acc[4 + j] += v1[j] * w;
      acc[8 + j] += v2[j] * w;
      acc[12 + j] += v3[j] * w;
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  return acc;
}

// d out / d (normalised coords) for cotangent tile g (this lane's 16 channels; caller adds the
// other half with xor32 and multiplies by gmul)
__device__ __forceinline__ void coord_grad_partial(const float* __restrict__ grid, const Corners& c,
                                                   const f32x16& g, int lane, float out[3]) {
  const int h = lane >> 5;
  out[0] = out[1] = out[2] = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    __builtin_amdgcn_sched_barrier(0);  // keep the 8 corner reads from being hoisted together
    const gptr_t<f32x4> row = as_global(reinterpret_cast<const f32x4*>(grid + (size_t)c.row[k] * NSLAM_C_DIM + 4 * h));
    const f32x4 v0 = row[0], v1 = row[2], v2 = row[4], v3 = row[6];
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dot += v0[j] * g[j];
      dot += v1[j] * g[4 + j];
      dot += v2[j] * g[8 + j];
      dot += v3[j] * g[12 + j];
    }
    if (!((c.ok >> k) & 1u)) dot = 0.f;  // out-of-range corner contributes nothing
    const int dx = k & 1, dy = (k >> 1) & 1, dz = k >> 2;
    const float fx = dx ? c.f1[0] : c.f0[0], fy = dy ? c.f1[1] : c.f0[1], fz = dz ? c.f1[2] : c.f0[2];
    const float sx = dx ? 1.f : -1.f, sy = dy ? 1.f : -1.f, sz = dz ? 1.f : -1.f;
    out[0] += sx * (fy * fz) * dot;
    out[1] += sy * (fx * fz) * dot;
    out[2] += sz * (fx * fy) * dot;
  }
}

// ------------------------------------------------------------------------------------------
// accurate, branch-free sin/cos for the Fourier features (args up to ~1e5 rad; decoder.py:30)
// Cody-Waite reduction x - k*pi/2 in float32 with a three-part pi/2 (P1 = float(pi/2), so
// fma(-k, P1, x) is exact for |k| < 2^24 / 2^ulp-gap and the two tails keep r to ~1 ulp), then
// float32 minimax polynomials on [-pi/4, pi/4].  Max error ~1 ulp (the reference's torch.sin is a
// <=1-ulp Sleef/libm sinf); bit-identical to the former float64 reduction on 25k sampled args.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void reduce_pio2(float x, float& r, int& q) {
  const float k = rintf(x * 0.636619746685028076171875f);
  r = fmaf(-k, 1.57079637050628662109375f, x);
  r = fmaf(-k, -4.37113882867379300296306610107421875e-8f, r);
  r = fmaf(-k, -1.7151245100058818e-15f, r);
  q = ((int)k) & 3;
}
__device__ __forceinline__ float sin_poly(float r) {
  const float r2 = r * r;
  float p = fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f);
  p = fmaf(r2, p, -1.6666654611e-1f);
  return fmaf(r * r2, p, r);
}
__device__ __forceinline__ float cos_poly(float r) {
  const float r2 = r * r;
  float p = fmaf(r2, 2.443315711809948e-5f, -1.388731625493765e-3f);
  p = fmaf(r2, p, 4.166664568298827e-2f);
  return fmaf(r2 * r2, p, fmaf(-0.5f, r2, 1.f));
}
__device__ __forceinline__ float fsin(float x) {
  float r;
  int q;
  reduce_pio2(x, r, q);
  const float s = sin_poly(r), c = cos_poly(r);
  const float v = (q & 1) ? c : s;
  return (q & 2) ? -v : v;
}
// both at once (one reduction, both polynomials): Fourier forward + its derivative
__device__ __forceinline__ void fsincos(float x, float& sv, float& cv) {
  float r;
  int q;
  reduce_pio2(x, r, q);
  const float s = sin_poly(r), c = cos_poly(r);
  const float vs = (q & 1) ? c : s, vc = (q & 1) ? s : c;
  sv = (q & 2) ? -vs : vs;
  cv = ((q + 1) & 2) ? -vc : vc;
}
__device__ __forceinline__ float fcos(float x) {
  float r;
  int q;
  reduce_pio2(x, r, q);
  const float s = sin_poly(r), c = cos_poly(r);
  const float v = (q & 1) ? s : c;
  return ((q + 1) & 2) ? -v : v;
}

// ------------------------------------------------------------------------------------------
// Adam element update (torch.optim.Adam single-tensor form, the reference's torch 1.11):
//   m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g g;  p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
// with torch's GPU division by a host scalar done as a multiply by its float reciprocal.  Shared by
// k_adam (nslam_mapping.hip) and the Adam epilogue of k_slab_reduce (nslam_query_impl.h).
// ------------------------------------------------------------------------------------------
struct AdamCoef {
  float b1, omb1, b2, omb2, eps, rbc2s, step_size;
};

__device__ __forceinline__ AdamCoef adam_coef(float b1, float b2, float eps, float lr, float step) {
  const float t = step + 1.f;
  const double bc1 = 1.0 - pow((double)b1, (double)t);
  const double bc2 = 1.0 - pow((double)b2, (double)t);
  AdamCoef c;
  c.b1 = b1;
  c.omb1 = 1.f - b1;
  c.b2 = b2;
  c.omb2 = 1.f - b2;
  c.eps = eps;
  c.rbc2s = 1.f / (float)sqrt(bc2);
  c.step_size = (float)((double)lr / bc1);
  return c;
}

__device__ __forceinline__ float adam_one(float& p, float g, float& m, float& v, const AdamCoef& c) {
  m = c.b1 * m + c.omb1 * g;
  v = c.b2 * v + c.omb2 * g * g;
  const float den = sqrtf(v) * c.rbc2s + c.eps;
  p = p - c.step_size * (m / den);
  return p;
}

// One workgroup's share of a segment's update (k_adam's body; nthreads = the workgroup's size): R
// items per thread, dense segments one element per item (element (lb R + k) nthreads + tid),
// row-masked segments row_len/4 threads per row (one float4 per item) — the same element update
// everywhere, so any launch that hands a segment's workgroups this function updates it
// bit-identically.  Every item's loads are issued before any arithmetic (R × 4 loads in flight per
// thread), and coef() (the bias corrections: two float64 pow) is evaluated while they fly.
template <int R, class CoefFn>
__device__ __forceinline__ void adam_segment_block(const nslam_adam_seg& sg, const CoefFn& coef, int64_t lb,
                                                   int zero_grad, int tid, int nthreads) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  // ABI v19: a segment sized for a capacity may carry its live row / element count on the device
  const int64_t n_seg = sg.n_live ? (*sg.n_live < sg.n ? *sg.n_live : sg.n) : sg.n;
  if (!sg.rows) {
    int64_t e[R];
    float p[R], m[R], v[R], g[R];
    bool any = false;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      e[k] = (lb * R + k) * nthreads + tid;
      if (e[k] < n_seg) {
        p[k] = sg.param[e[k]];
        m[k] = sg.exp_avg[e[k]];
        v[k] = sg.exp_avg_sq[e[k]];
        g[k] = sg.grad[e[k]];
        any = true;
      }
    }
    if (!any) return;
    __builtin_amdgcn_sched_barrier(0);  // the loads first, then the coefficients (their latency hides)
    const AdamCoef c = coef();
#pragma unroll
    for (int k = 0; k < R; ++k) {
      if (e[k] >= n_seg) continue;
      adam_one(p[k], g[k], m[k], v[k], c);
      sg.param[e[k]] = p[k];
      sg.exp_avg[e[k]] = m[k];
      sg.exp_avg_sq[e[k]] = v[k];
      if (zero_grad) sg.grad[e[k]] = 0.f;
      if (sg.mirror) {  // the packed MFMA copy of this parameter (up to two slots)
        const int i0 = sg.mirror_idx[2 * e[k]], i1 = sg.mirror_idx[2 * e[k] + 1];
        if (i0 >= 0) sg.mirror[i0] = p[k];
        if (i1 >= 0) sg.mirror[i1] = p[k];
      }
    }
  } else {
    const int q = sg.row_len / 4;  // float4 per row
    const int64_t rows_per_block = nthreads / q;
    const int part = tid % q;
    const bool lane_ok = tid < rows_per_block * q;
    int64_t ri[R], base[R], sbase[R], gbase[R];
    bool ok[R];
    bool any = false;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      ri[k] = (lb * R + k) * rows_per_block + tid / q;
      ok[k] = lane_ok && ri[k] < n_seg;
      any |= ok[k];
    }
    if (!any) return;
    int32_t row[R];
#pragma unroll
    for (int k = 0; k < R; ++k) row[k] = ok[k] ? sg.rows[ri[k]] : 0;
    f4 p[R], g[R], m[R], v[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      if (!ok[k]) continue;
      base[k] = (int64_t)row[k] * sg.row_len + part * 4;
      sbase[k] = ri[k] * sg.row_len + part * 4;
      gbase[k] = sg.grad_rows ? sbase[k] : base[k];
      p[k] = *reinterpret_cast<const f4*>(sg.param + base[k]);
      g[k] = *reinterpret_cast<const f4*>(sg.grad + gbase[k]);
      m[k] = *reinterpret_cast<const f4*>(sg.exp_avg + sbase[k]);
      v[k] = *reinterpret_cast<const f4*>(sg.exp_avg_sq + sbase[k]);
    }
    __builtin_amdgcn_sched_barrier(0);
    const AdamCoef c = coef();
#pragma unroll
    for (int k = 0; k < R; ++k) {
      if (!ok[k]) continue;
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        float pk = p[k][l], mk = m[k][l], vk = v[k][l];
        adam_one(pk, g[k][l], mk, vk, c);
        p[k][l] = pk;
        m[k][l] = mk;
        v[k][l] = vk;
      }
      *reinterpret_cast<f4*>(sg.param + base[k]) = p[k];
      *reinterpret_cast<f4*>(sg.exp_avg + sbase[k]) = m[k];
      *reinterpret_cast<f4*>(sg.exp_avg_sq + sbase[k]) = v[k];
      if (zero_grad) *reinterpret_cast<f4*>(sg.grad + gbase[k]) = f4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

// workgroups of `nthreads` threads (R items each) a segment's update takes (adam_segment_block)
template <int R>
__host__ __device__ inline int64_t adam_segment_blocks(const nslam_adam_seg& sg, int nthreads) {
  if (sg.rows) {
    const int64_t rpb = (int64_t)(nthreads / (sg.row_len / 4)) * R;
    return (sg.n + rpb - 1) / rpb;
  }
  const int64_t per = (int64_t)nthreads * R;
  return (sg.n + per - 1) / per;
}
