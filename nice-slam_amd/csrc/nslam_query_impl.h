#pragma once
// nslam_query_impl.h — fused point query for gfx950: normalise → trilinear gather (channels-last
// grids) → Fourier embedding → tiny MLP decoders on MFMA (v_mfma_f32_32x32x2_f32) → stage
// combiner → OOB logit, and its recompute-backward.
//
// Replaces, per point: Renderer.eval_points (src/utils/Renderer.py:23-61), NICE.forward
// (src/conv_onet/models/decoder.py:312-342), MLP / MLP_no_xyz forward (decoder.py:177-203,
// 262-274), sample_grid_feature (decoder.py:168-175, F.grid_sample) and the autograd backward of
// all of them (Tracker.py:125, Mapper.py:503).
//
// Work decomposition: one wave = one tile of 32 points.  Each lane pair (l, l+32) owns one point;
// the half h = l>>5 gathers/holds the 16 feature channels F(r,h) of that point (nslam_dev.h).
#include <type_traits>

#include "nslam_dev.h"

// Everything lives in a named namespace: the per-decoder backward launchers are explicitly
// instantiated in their own translation units (nslam_query_dec.hip, built once per decoder) so the
// library compiles in parallel; the API translation unit (nslam_query.hip) only declares them.
namespace nslamq {

struct QueryKArgs {
  nslam_query_cfg c;
  const double* pts;
  int64_t n;
  float* raw;          // fwd output [n][4]
  const float* g_raw;  // bwd input  [n][4]
  double* g_pts;       // bwd output [n][3]
};

// ------------------------------------------------------------------------------------------
// per-point context
// ------------------------------------------------------------------------------------------
struct Pt {
  double p[3];
  float x[3];  // p.float() (decoder.py:189)
  bool valid;
  bool inside;
};

__device__ __forceinline__ Pt load_point(const QueryKArgs& a, int64_t idx) {
  Pt q;
  q.valid = idx < a.n;
  const int64_t i = q.valid ? idx : 0;  // invalid tail lanes compute on a real point, write nothing
  if (a.c.rays_o) {  // pts = rays_o + rays_d * z (float64, Renderer.py:172-174); host checks n < 2^31
    const uint32_t r = (uint32_t)i / (uint32_t)a.c.n_samples;
    const double z = a.c.z_vals[i];
#pragma unroll
    for (int k = 0; k < 3; ++k) q.p[k] = (double)a.c.rays_o[r * 3 + k] + (double)a.c.rays_d[r * 3 + k] * z;
  } else {
    q.p[0] = a.pts[i * 3 + 0];
    q.p[1] = a.pts[i * 3 + 1];
    q.p[2] = a.pts[i * 3 + 2];
  }
  bool in = true;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    q.x[k] = (float)q.p[k];
    in = in && (q.p[k] < a.c.bound_hi[k]) && (q.p[k] > a.c.bound_lo[k]);  // Renderer.py:43-46
  }
  q.inside = in;
  return q;
}

__device__ __forceinline__ void grid_corners(Corners& cr, const nslam_grid& g, const Pt& q) {
  float nc3[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) nc3[k] = norm_coord(q.p[k], g.lo[k], g.hi[k]);
  make_corners(cr, nc3, g.dims);
}

// The trilinear cell of a point in one grid, corners formed on demand (make_corners' rows and weights,
// the same arithmetic): 10 values per lane instead of a Corners struct's 8 rows + 8 weights.
struct LazyCell {
  int row0, nx, nxy;
  float f0[3], f1[3];
  bool hi_ok[3];
  __device__ __forceinline__ LazyCell(const nslam_grid& g, const Pt& q) {
    const int n[3] = {g.dims[2], g.dims[1], g.dims[0]};  // x→W, y→H, z→D
    int i0[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      float gm;
      const float u = unnorm_clip(norm_coord(q.p[a], g.lo[a], g.hi[a]), n[a], gm);
      const float fl = floorf(u);
      i0[a] = (int)fl;
      f1[a] = u - fl;
      f0[a] = (float)(i0[a] + 1) - u;
      hi_ok[a] = (i0[a] + 1) <= n[a] - 1;
    }
    nx = n[0];
    nxy = n[1] * n[0];
    row0 = (i0[2] * n[1] + i0[1]) * n[0] + i0[0];
  }
  // corner k's row (0 when out of range) and weight (exactly 0 when out of range)
  __device__ __forceinline__ int row(int k, float& w) const {
    const int dx = k & 1, dy = (k >> 1) & 1, dz = k >> 2;
    const bool ok = (!dx || hi_ok[0]) && (!dy || hi_ok[1]) && (!dz || hi_ok[2]);
    const float wr = ((dx ? f1[0] : f0[0]) * (dy ? f1[1] : f0[1])) * (dz ? f1[2] : f0[2]);
    w = ok ? wr : 0.f;
    return (row0 + dz * nxy + dy * nx + dx) & -(int)ok;  // (a select, not a branch)
  }
};

// Two trilinear gathers (the fine decoder's fine and middle features, decoder.py:184-187) software-
// pipelined corner by corner: corner k + 1's rows of both grids are loaded while corner k is summed, so
// 16 row loads per lane are in flight and no corner waits for a full round trip after the previous one.
// Each feature sums its corners in gather_tile's order (the same values).
__device__ __forceinline__ void gather_pair(const nslam_grid& gA, const nslam_grid& gB, const Pt& q, int lane,
                                            f32x16& accA, f32x16& accB) {
  const int h = lane >> 5;
  const LazyCell A(gA, q), B(gB, q);
  accA = zero16();
  accB = zero16();
  auto load = [&](const LazyCell& L, const float* data, int k, f32x4 (&v)[4], float& w) {
    const gptr_t<f32x4> rp =
        as_global(reinterpret_cast<const f32x4*>(data + (size_t)(uint32_t)L.row(k, w) * NSLAM_C_DIM + 4 * h));
    v[0] = rp[0];
    v[1] = rp[2];
    v[2] = rp[4];
    v[3] = rp[6];
  };
  f32x4 va[4], vb[4];
  float wa, wb;
  load(A, gA.data, 0, va, wa);
  load(B, gB.data, 0, vb, wb);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    f32x4 na[4], nb[4];
    float nwa = 0.f, nwb = 0.f;
    if (k < 7) {
      load(A, gA.data, k + 1, na, nwa);
      load(B, gB.data, k + 1, nb, nwb);
    }
    __builtin_amdgcn_sched_barrier(0);  // the next corner's loads are issued before this one is summed
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      accA[j] += va[0][j] * wa;
      accA[4 + j] += va[1][j] * wa;
      accA[8 + j] += va[2][j] * wa;
      accA[12 + j] += va[3][j] * wa;
      accB[j] += vb[0][j] * wb;
      accB[4 + j] += vb[1][j] * wb;
      accB[8 + j] += vb[2][j] * wb;
      accB[12 + j] += vb[3][j] * wb;
    }
    if (k < 7) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        va[i] = na[i];
        vb[i] = nb[i];
      }
      wa = nwa;
      wb = nwb;
    }
  }
}

// gather_tile's trilinear feature software-pipelined like gather_pair (corner k + 1's row loads in flight
// while corner k is summed; the same sum order, so the same values) with its corners formed lazily
__device__ __forceinline__ f32x16 gather_one(const nslam_grid& g, const Pt& q, int lane) {
  const int h = lane >> 5;
  const LazyCell A(g, q);
  f32x16 acc = zero16();
  auto load = [&](int k, f32x4 (&v)[4], float& w) {
    const gptr_t<f32x4> rp =
        as_global(reinterpret_cast<const f32x4*>(g.data + (size_t)(uint32_t)A.row(k, w) * NSLAM_C_DIM + 4 * h));
    v[0] = rp[0];
    v[1] = rp[2];
    v[2] = rp[4];
    v[3] = rp[6];
  };
  f32x4 va[4];
  float wa;
  load(0, va, wa);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    f32x4 na[4];
    float nwa = 0.f;
    if (k < 7) load(k + 1, na, nwa);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[j] += va[0][j] * wa;
      acc[4 + j] += va[1][j] * wa;
      acc[8 + j] += va[2][j] * wa;
      acc[12 + j] += va[3][j] * wa;
    }
    if (k < 7) {
#pragma unroll
      for (int i = 0; i < 4; ++i) va[i] = na[i];
      wa = nwa;
    }
  }
  return acc;
}

// gather_tile's trilinear feature with NB corners' row loads issued together (8 / NB round trips of
// memory latency instead of gather_one's 8 pipelined ones), summed in gather_tile's corner order (the
// same values).  For a wave with nothing else in registers (the producer of k_query_fwd_pc).
template <int NB>
__device__ __forceinline__ f32x16 gather_nb(const nslam_grid& g, const Pt& q, int lane) {
  const int h = lane >> 5;
  const LazyCell A(g, q);
  f32x16 acc = zero16();
#pragma unroll
  for (int k0 = 0; k0 < 8; k0 += NB) {
    f32x4 v[NB][4];
    float w[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const gptr_t<f32x4> rp = as_global(
          reinterpret_cast<const f32x4*>(g.data + (size_t)(uint32_t)A.row(k0 + k, w[k]) * NSLAM_C_DIM + 4 * h));
      v[k][0] = rp[0];
      v[k][1] = rp[2];
      v[k][2] = rp[4];
      v[k][3] = rp[6];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < NB; ++k) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[j] += v[k][0][j] * w[k];
        acc[4 + j] += v[k][1][j] * w[k];
        acc[8 + j] += v[k][2][j] * w[k];
        acc[12 + j] += v[k][3][j] * w[k];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  return acc;
}

// ------------------------------------------------------------------------------------------
// Fourier embedding (decoder.py:26-30): block b, reg r of lane (h,p) is dim k = 32b + F(r,h)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float fourier_arg(const float x[3], float b0, float b1, float b2) {
  return fmaf(x[2], b2, fmaf(x[1], b1, x[0] * b0));
}

// G: B is in global memory (else LDS or generic); see as_global
template <bool COS, bool G = false>
__device__ __forceinline__ f32x16 emb_tile(const float* __restrict__ B, const float x[3], int b, int lane) {
  const int h = lane >> 5;
  f32x16 e;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = 32 * b + 8 * i + 4 * h;
    const f32x4 B0 = G ? *as_global(reinterpret_cast<const f32x4*>(B + k)) : *reinterpret_cast<const f32x4*>(B + k);
    const f32x4 B1 = G ? *as_global(reinterpret_cast<const f32x4*>(B + 96 + k))
                       : *reinterpret_cast<const f32x4*>(B + 96 + k);
    const f32x4 B2 = G ? *as_global(reinterpret_cast<const f32x4*>(B + 192 + k))
                       : *reinterpret_cast<const f32x4*>(B + 192 + k);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float t = fourier_arg(x, B0[j], B1[j], B2[j]);
      e[4 * i + j] = COS ? fcos(t) : fsin(t);
    }
  }
  return e;
}

// ------------------------------------------------------------------------------------------
// LDS helpers for weight gradients (wave-private scratch, WG = 1 wave in the backward kernel)
// ------------------------------------------------------------------------------------------
struct Scratch {
  float* sA;    // [32][33] transposed cotangent tile
  float* sX;    // [32][33] transposed input tile
  float* gtab;  // [32][4]  per-point output cotangents
  float* xtab;  // [32][3]  per-point x (float)
  int* crow;    // [32][8]  corner rows (grad slots when the grid gradient is frustum-compacted)
  float* cw;    // [32][8]
  int* ccell;   // [32]     cell of each point (packed lower-corner coordinates): the run-merge key
};

// Scratch is wave-private: ordering LDS writes before other lanes' reads of the same wave needs
// only the wave's own LDS counter drained (and a compiler memory barrier), not a workgroup barrier.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Phase timing (debug build only, make phases): lane 0 of each backward wave records s_memtime
// at marks 0..15 of its tile into g_phase[decoder][wave][16].
#ifdef NSLAM_PHASES
constexpr int kPhaseWaves = 1 << 15;
// slots: 0 forward, 1..3 decoder backward, 4 k_color_wgrad (per wave: cycles in prod / cons / hand-over)
__device__ unsigned long long g_phase[5 * kPhaseWaves * 16];  // one-TU phases build only
#define PHASE(dec, k)                                                                                     \
  do {                                                                                                    \
    const int64_t w_ = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);                     \
    if ((threadIdx.x & 63) == 0 && w_ < kPhaseWaves)                                                      \
      g_phase[((size_t)(dec) * kPhaseWaves + w_) * 16 + (k)] = __builtin_amdgcn_s_memtime();              \
  } while (0)
#else
#define PHASE(dec, k) \
  do {                \
  } while (0)
#endif
// Timeline (make phases, or make timeline: the marks below only, so the kernels keep their production
// register allocation — the phase marks cost the forward 88 VGPRs and its third wave per SIMD): per
// wave of kernel slot k (0 forward, 1 mask-only backward, 2 k_color_wgrad) {start, end} of
// s_memrealtime (100 MHz, one clock for all XCDs), HW_ID | XCC_ID << 32, and a tag
#if defined(NSLAM_PHASES) || defined(NSLAM_TIMELINE)
constexpr int kTlWaves = 1 << 15;
__device__ unsigned long long g_tl[3 * kTlWaves * 4];
__device__ __forceinline__ void tl_mark(int slot, int end, long long tag) {
  const int64_t w_ = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) != 0 || w_ >= kTlWaves) return;
  unsigned long long* o = g_tl + ((size_t)slot * kTlWaves + w_) * 4;
  o[end] = __builtin_amdgcn_s_memrealtime();
  if (!end) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
    o[2] = (unsigned long long)hw | ((unsigned long long)(xcc & 15) << 32);
    o[3] = (unsigned long long)tag;
  }
}
#define TL(slot, end, tag) tl_mark(slot, end, tag)
// add v << 8 into this wave's tag (after its start mark): e.g. the 10-ns ticks a wave spent waiting
// (field f = 0: bits 8-31, f = 1: bits 32-55 — e.g. a producer's gather time)
__device__ __forceinline__ void tl_add(int slot, unsigned long long v, int f = 0) {
  const int64_t w_ = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && w_ < kTlWaves) g_tl[((size_t)slot * kTlWaves + w_) * 4 + 3] += v << (8 + 24 * f);
}
#define TL_ADD(slot, v) tl_add(slot, v)
#define TL_ADD1(slot, v) tl_add(slot, v, 1)
#define TL_NOW() __builtin_amdgcn_s_memrealtime()
#else
#define TL_ADD(slot, v) \
  do {                  \
  } while (0)
#define TL_ADD1(slot, v) \
  do {                   \
  } while (0)
#define TL_NOW() 0ull
#define TL(slot, end, tag) \
  do {                     \
  } while (0)
#endif

// ReLU masks saved by the forward: [decoder][tile][layer][64 lanes] uint16 (one 128-B row per layer)
__device__ __forceinline__ uint16_t* mask_slot(const QueryKArgs& a, int dec, int64_t tile) {
  const int64_t ntiles = (a.n + 31) / 32;
  return a.c.saved_masks + ((size_t)dec * ntiles + tile) * 5 * 64;
}
__device__ __forceinline__ void save_masks(const QueryKArgs& a, int dec, int64_t tile, const uint32_t m[5],
                                           int lane) {
  if (!a.c.saved_masks) return;
  uint16_t* s = mask_slot(a, dec, tile);
#pragma unroll
  for (int i = 0; i < 5; ++i) s[i * 64 + lane] = (uint16_t)m[i];
}
__device__ __forceinline__ void load_masks(const QueryKArgs& a, int dec, int64_t tile, uint32_t m[5], int lane) {
  const uint16_t* s = mask_slot(a, dec, tile);
#pragma unroll
  for (int i = 0; i < 5; ++i) m[i] = s[i * 64 + lane];
}

// Activation tape of the colour decoder (ABI v9 nslam_query_cfg.act_tape): the forward stores the
// post-ReLU hidden tiles h0..h4 of every tile (C layout) and the weight-gradient backward reads them
// instead of recomputing the decoder (it needs them as the inputs of dW; Mapper.py:503).
constexpr int kTapeFloats = 5 * 16 * 64;  // per tile: h0..h4
// Layout [tile][layer][register r][64 lanes] float: every store / load instruction moves 256 B
// contiguous, and no 4-register grouping of the tile is needed (a float4 layout cost the forward
// ~30 VGPRs of copies).
// Point-major: layer i of a tile is [32 points][32 features], the layout of the weight-gradient
// MFMA's B operand (K = points), so the backward streams it from global memory with no LDS
// transpose.  The forward stores registers 4k..4k+3 of lane (p, h) — features 8k+4h..+3, i.e.
// F(r, h) — as one 16-B store at [p][8k+4h].
__device__ __forceinline__ void tape_store(float* __restrict__ t, int i, const f32x16& v, int lane) {
  const int p = lane & 31, h = lane >> 5;
  __attribute__((address_space(1))) f32x4* q =
      reinterpret_cast<__attribute__((address_space(1))) f32x4*>(as_global_w(t) + i * 1024 + p * 32 + 4 * h);
#pragma unroll
  for (int k = 0; k < 4; ++k) q[2 * k] = f32x4{v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]};
}
// Parameter-gradient slab of one wave, addressed as a raw buffer: every update is a buffer store
// (or load + store) with the lane-dependent part of the offset in a VGPR and the uniform part
// (parameter block, row) in soffset, so the ~350 updates per tile cost one address VGPR per block.
// A slab address is owned by one lane of one wave, so no atomics: WG == 1 (a wave's only tile)
// stores, WG == 2 (waves walking several tiles over a zeroed slab) read-modify-writes; both are
// per-lane program-ordered.
struct Slab {
  __amdgpu_buffer_rsrc_t r;
};

__device__ __forceinline__ Slab make_slab(float* base, int floats) {
  return Slab{__builtin_amdgcn_make_buffer_rsrc(base, 0, floats * 4, 0x00020000)};
}

template <int WG>
__device__ __forceinline__ void put(const Slab& A, int lane_off, int uni_off, float v) {
  // the b32 intrinsics move raw bits (unsigned): bit-cast, never convert
  if (WG == 2) v += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(A.r, lane_off * 4, uni_off * 4, 0));
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), A.r, lane_off * 4, uni_off * 4, 0);
}

// dW[o][kofs + k] += sum_p sa[p][o] * sx[p][k]   for k < kvalid   (dW at slab offset base)
template <int WG>
__device__ __forceinline__ void dw_block_img(const Slab& A, int base, int ldk, int kofs, int kvalid,
                                             const float* __restrict__ sa, const float* __restrict__ sx, int lane) {
  const int h = lane >> 5, j = lane & 31;
  f32x16 acc = zero16();
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = mfma32(sa[(2 * s + h) * TPITCH + j], sx[(2 * s + h) * TPITCH + j], acc);
  if (j < kvalid) {
    const int lo = 4 * h * ldk + j;  // fidx(r, h) = (r & 3) + 8 (r >> 2) + 4 h
#pragma unroll
    for (int r = 0; r < 16; ++r) put<WG>(A, lo, base + ((r & 3) + 8 * (r >> 2)) * ldk + kofs, acc[r]);
  }
}
// the same with the input side as a B-operand stream in registers (tape_bop): no sx image
template <int WG>
__device__ __forceinline__ void dw_block_bop(const Slab& A, int base, int ldk, int kofs, int kvalid,
                                             const float* __restrict__ sa, const f32x16& bx, int lane) {
  const int h = lane >> 5, j = lane & 31;
  f32x16 acc = zero16();
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = mfma32(sa[(2 * s + h) * TPITCH + j], bx[s], acc);
  if (j < kvalid) {
    const int lo = 4 * h * ldk + j;
#pragma unroll
    for (int r = 0; r < 16; ++r) put<WG>(A, lo, base + ((r & 3) + 8 * (r >> 2)) * ldk + kofs, acc[r]);
  }
}
template <int WG>
__device__ __forceinline__ void dw_block(const Slab& A, int base, int ldk, int kofs, int kvalid, const Scratch& S,
                                         int lane) {
  dw_block_img<WG>(A, base, ldk, kofs, kvalid, S.sA, S.sX, lane);
}

// db[o] += sum_p sa[p][o]
template <int WG>
__device__ __forceinline__ void db_vec_img(const Slab& A, int base, const float* __restrict__ sa, int lane) {
  const int h = lane >> 5, o = lane & 31;
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 16; ++t) s += sa[(2 * t + h) * TPITCH + o];
  s += xor32(s);
  if (h == 0) put<WG>(A, o, base, s);
}
template <int WG>
__device__ __forceinline__ void db_vec(const Slab& A, int base, const Scratch& S, int lane) {
  db_vec_img<WG>(A, base, S.sA, lane);
}

// sA <- d ; then per input tile: sX <- x ; dW += ...
__device__ __forceinline__ void wg_begin(const f32x16& d, const Scratch& S, int lane) { tstore(S.sA, d, lane); }
template <int WG>
__device__ __forceinline__ void wg_block(const Slab& A, int base, int ldk, int kofs, int kvalid, const f32x16& x,
                                         const Scratch& S, int lane) {
  tstore(S.sX, x, lane);
  lds_sync();
  dw_block<WG>(A, base, ldk, kofs, kvalid, S, lane);
  lds_sync();
}
template <int WG>
__device__ __forceinline__ void wg_end(const Slab& A, int base, const Scratch& S, int lane) {
  lds_sync();
  db_vec<WG>(A, base, S, lane);
  lds_sync();
}

// ------------------------------------------------------------------------------------------
// MLP with Fourier embedding (decoder.py:177-203): forward
//   layer-3's embedding product is formed right after layer 0, so the 48-register embedding
//   dies early (the MFMA work is unchanged).
// ------------------------------------------------------------------------------------------
// vector-section tile: LDS copy (vec_tile) or global (vec_tile_g)
template <bool VLDS>
__device__ __forceinline__ f32x16 vtile(const float* __restrict__ v, int lane) {
  return VLDS ? vec_tile(v, lane) : vec_tile_g(v, lane);
}

template <int NC, bool VLDS>
__device__ __forceinline__ f32x16 fc_branch(const float* __restrict__ pk, const XyzPack& L, int i,
                                            const f32x16 (&cin)[NC], int lane, const float* vec) {
  // vec: the decoder's vector section (biases, output row, Fourier B) — an LDS copy in the
  // decoder-parallel forward, else pk + L.V()
  f32x16 z = vtile<VLDS>(vec + (L.BiasC(i) - L.V()), lane);
#pragma unroll
  for (int c = 0; c < NC; ++c) gemm_acc(z, pk + L.FC(i, c) * NSLAM_FRAG, cin[c], lane);
  return z;
}

template <int NC, bool KEEP, bool PHF = false, bool TAPE = false, bool VLDS = false>
__device__ __forceinline__ f32x16 xyz_forward(const float* __restrict__ pk, const f32x16 (&cin)[NC],
                                              const float x[3], int lane, uint32_t m[5], f32x16* hs,
                                              float* __restrict__ tape = nullptr, const float* vec = nullptr) {
  const XyzPack L{NC};
  // vector section: the workgroup's LDS copy (VLDS) or global.  A compile-time choice: a runtime
  // select of an LDS and a global pointer is a generic pointer, i.e. flat loads.
  const float* vs = VLDS ? vec : pk + L.V();
#define PHF_(k) \
  if (PHF) PHASE(0, k)
  f32x16 a = vtile<VLDS>(vs + (L.Bias(0) - L.V()), lane);
  f32x16 a3 = vtile<VLDS>(vs + (L.Bias(3) - L.V()), lane);
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const f32x16 e = emb_tile<false, !VLDS>(vs + (L.FB() - L.V()), x, b, lane);
    gemm_acc(a, pk + (L.L0() + b) * NSLAM_FRAG, e, lane);
    gemm_acc(a3, pk + (L.L3() + b) * NSLAM_FRAG, e, lane);
  }
  PHF_(5);
  m[0] = mask16(a);
  f32x16 h = relu16(a) + fc_branch<NC, VLDS>(pk, L, 0, cin, lane, vs);
  if (KEEP) hs[0] = h;
  if (TAPE) tape_store(tape, 0, h, lane);
  a = vtile<VLDS>(vs + (L.Bias(1) - L.V()), lane);
  gemm_acc(a, pk + L.L1() * NSLAM_FRAG, h, lane);
  m[1] = mask16(a);
  h = relu16(a) + fc_branch<NC, VLDS>(pk, L, 1, cin, lane, vs);
  if (KEEP) hs[1] = h;
  if (TAPE) tape_store(tape, 1, h, lane);
  PHF_(6);
  a = vtile<VLDS>(vs + (L.Bias(2) - L.V()), lane);
  gemm_acc(a, pk + L.L2() * NSLAM_FRAG, h, lane);
  m[2] = mask16(a);
  h = relu16(a) + fc_branch<NC, VLDS>(pk, L, 2, cin, lane, vs);
  if (KEEP) hs[2] = h;
  if (TAPE) tape_store(tape, 2, h, lane);
  gemm_acc(a3, pk + (L.L3() + 3) * NSLAM_FRAG, h, lane);
  m[3] = mask16(a3);
  h = relu16(a3) + fc_branch<NC, VLDS>(pk, L, 3, cin, lane, vs);
  if (KEEP) hs[3] = h;
  if (TAPE) tape_store(tape, 3, h, lane);
  PHF_(7);
  a = vtile<VLDS>(vs + (L.Bias(4) - L.V()), lane);
  gemm_acc(a, pk + L.L4() * NSLAM_FRAG, h, lane);
  m[4] = mask16(a);
  h = relu16(a) + fc_branch<NC, VLDS>(pk, L, 4, cin, lane, vs);
  if (TAPE) tape_store(tape, 4, h, lane);
  PHF_(8);
  return h;
#undef PHF_
}

// xyz_forward of the decoder-parallel forward (VLDS: the vector section in LDS), its 15 (NC = 1) or 20
// (NC = 2) GEMMs as a FragPipe: each weight fragment is loaded while the previous GEMM runs, so no GEMM
// waits for its fragment's L2 round trip.  The same products in the same order as xyz_forward.
// (phases build: marks MK .. MK + 3 after the embedding GEMMs, layers 1-2, layer 3 and layer 4)
// The weight-fragment blocks of xyz_forward_pf_e's GEMMs in issue order: L0_b / L3_b for b = 0..2, then
// per layer i = 0..4 the NC fc_c.i blocks followed by the next layer's block (L1, L2, L3's h2 block, L4)
template <int NC>
__device__ __forceinline__ constexpr int frag_seq(int i) {
  const XyzPack L{NC};
  if (i < 6) return (i & 1) ? L.L3() + (i >> 1) : L.L0() + (i >> 1);
  i -= 6;
  const int layer = i / (NC + 1), j = i % (NC + 1);
  if (j < NC) return L.FC(layer, j);
  return layer == 0 ? L.L1() : layer == 1 ? L.L2() : layer == 2 ? L.L3() + 3 : L.L4();
}
// FragPipe with D fragments in flight: GEMM i runs while the fragments of GEMMs i+1 .. i+D load (the
// block order is frag_seq's, so the call sites' `next` is not needed)
template <int NC, int D>
struct SeqPipe {
  static constexpr int kN = 10 + 5 * NC;
  const float* pk;
  int lane, i;
  Frag f[D];
  __device__ __forceinline__ SeqPipe(const float* pk_, int, int lane_) : pk(pk_), lane(lane_), i(0) {
#pragma unroll
    for (int d = 0; d < D; ++d) f[d] = load_frag(pk + frag_seq<NC>(d) * NSLAM_FRAG, lane);
  }
  __device__ __forceinline__ void gemm(f32x16& acc, const f32x16& x, int) {
    const Frag cur = f[0];
#pragma unroll
    for (int d = 0; d + 1 < D; ++d) f[d] = f[d + 1];
    if (i + D < kN) f[D - 1] = load_frag(pk + frag_seq<NC>(i + D) * NSLAM_FRAG, lane);
    __builtin_amdgcn_sched_barrier(0);
    gemm_frag(acc, cur, x);
    ++i;
  }
};

// no fragment pipeline: each GEMM loads its own fragment (gemm_acc), in frag_seq order
template <int NC>
struct NoPipe {
  const float* pk;
  int lane, i;
  __device__ __forceinline__ NoPipe(const float* pk_, int, int lane_) : pk(pk_), lane(lane_), i(0) {}
  __device__ __forceinline__ void gemm(f32x16& acc, const f32x16& x, int) {
    gemm_acc(acc, pk + frag_seq<NC>(i) * NSLAM_FRAG, x, lane);
    ++i;
  }
};

// (E(b): embedding block b — sin(x B_b) formed here, or handed over by a producer wave, k_query_fwd_pc;
//  FD: weight fragments in flight, 1 = FragPipe, 0 = none)
template <int NC, bool TAPE, int MK = 5, int FD = 1, class EmbFn>
__device__ __forceinline__ f32x16 xyz_forward_pf_e(const float* __restrict__ pk, const f32x16 (&cin)[NC],
                                                   const EmbFn& E, int lane, uint32_t m[5],
                                                   float* __restrict__ tape, const float* vs) {
  const XyzPack L{NC};
  typename std::conditional<FD == 1, FragPipe,
                            typename std::conditional<FD == 0, NoPipe<NC>, SeqPipe<NC, FD>>::type>::type fp(
      pk, L.L0(), lane);
  f32x16 a = vec_tile(vs + (L.Bias(0) - L.V()), lane);
  f32x16 a3 = vec_tile(vs + (L.Bias(3) - L.V()), lane);
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const f32x16 e = E(b);
    fp.gemm(a, e, L.L3() + b);
    fp.gemm(a3, e, b < 2 ? L.L0() + b + 1 : L.FC(0, 0));
  }
  PHASE(0, MK);
  // fc_c.i (cin) with the next layer's first fragment after it
  auto fc = [&](int i, int next) {
    f32x16 z = vec_tile(vs + (L.BiasC(i) - L.V()), lane);
#pragma unroll
    for (int c = 0; c < NC; ++c) fp.gemm(z, cin[c], c + 1 < NC ? L.FC(i, c + 1) : next);
    return z;
  };
  m[0] = mask16(a);
  f32x16 h = relu16(a) + fc(0, L.L1());
  if (TAPE) tape_store(tape, 0, h, lane);
  a = vec_tile(vs + (L.Bias(1) - L.V()), lane);
  fp.gemm(a, h, L.FC(1, 0));
  m[1] = mask16(a);
  h = relu16(a) + fc(1, L.L2());
  if (TAPE) tape_store(tape, 1, h, lane);
  a = vec_tile(vs + (L.Bias(2) - L.V()), lane);
  fp.gemm(a, h, L.FC(2, 0));
  m[2] = mask16(a);
  h = relu16(a) + fc(2, L.L3() + 3);
  if (TAPE) tape_store(tape, 2, h, lane);
  PHASE(0, MK + 1);
  fp.gemm(a3, h, L.FC(3, 0));
  m[3] = mask16(a3);
  h = relu16(a3) + fc(3, L.L4());
  if (TAPE) tape_store(tape, 3, h, lane);
  PHASE(0, MK + 2);
  a = vec_tile(vs + (L.Bias(4) - L.V()), lane);
  fp.gemm(a, h, L.FC(4, 0));
  m[4] = mask16(a);
  h = relu16(a) + fc(4, -1);
  if (TAPE) tape_store(tape, 4, h, lane);
  PHASE(0, MK + 3);
  return h;
}
#ifndef NSLAM_UNITS_PAIR
#define NSLAM_UNITS_PAIR 1  // the fine unit's two gathers software-pipelined together (0: one after the other)
#endif
#ifndef NSLAM_UNITS_FD
#define NSLAM_UNITS_FD 1  // weight fragments in flight in the units / parts forward (0: none, 1: FragPipe)
#endif
template <int NC, bool TAPE, int MK = 5>
__device__ __forceinline__ f32x16 xyz_forward_pf(const float* __restrict__ pk, const f32x16 (&cin)[NC],
                                                 const float x[3], int lane, uint32_t m[5],
                                                 float* __restrict__ tape, const float* vs) {
  const XyzPack L{NC};
  return xyz_forward_pf_e<NC, TAPE, MK, NSLAM_UNITS_FD>(
      pk, cin, [&](int b) { return emb_tile<false, false>(vs + (L.FB() - L.V()), x, b, lane); }, lane, m, tape, vs);
}

// output_linear row j: sum_f Wo[j][f] h4[f] + bo[j]  (complete in both halves)
__device__ __forceinline__ float out_row(const float* __restrict__ Wo, const float* __restrict__ bo, int j,
                                         const f32x16& h4, int lane) {
  const f32x16 w = vec_tile(Wo + 32 * j, lane);
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += w[r] * h4[r];
  return (s + xor32(s)) + bo[j];
}

// dh += the caller's cotangent of h4 (ABI v17 nslam_query_cfg.g_h4; row = this lane's point, [32] floats,
// NULL: none): feature F(r, h) of register r = 4i + j is float 8i + 4h + j of the row
__device__ __forceinline__ void add_gh4(f32x16& dh, const float* __restrict__ row, int lane) {
  if (!row) return;
  const gptr_t<f32x4> p = as_global(reinterpret_cast<const f32x4*>(row + 4 * (lane >> 5)));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x4 v = p[2 * i];
#pragma unroll
    for (int j = 0; j < 4; ++j) dh[4 * i + j] += v[j];
  }
}

// ------------------------------------------------------------------------------------------
// MLP with Fourier embedding: backward (forward recomputed first).
//   gall[GOFS + j], j < NOUT : cotangents of the decoder outputs (per point, both halves)
//   dc : out, d/d(feature block 0) (C layout);  gx : out, d/dx through the embedding (if EMBG)
// Parameter gradients (WG) go through LDS transposes + MFMA over the 32 points and are added
// with atomics shaped as two 128-B row segments.
// ------------------------------------------------------------------------------------------
template <int NC, int WG>
__device__ __forceinline__ void fc_bwd(const float* __restrict__ pk, const XyzPack& L, int i,
                                       const f32x16 (&cin)[NC], const f32x16& dh, const nslam_dec_grad& dg,
                                       const Slab& A, const Scratch& S, int lane, f32x16& dc) {
  gemm_acc(dc, pk + L.FCT(i) * NSLAM_FRAG, dh, lane);  // dz_i = dh_i
  if (WG) {
    wg_begin(dh, S, lane);
#pragma unroll
    for (int c = 0; c < NC; ++c) wg_block<WG>(A, dg.wc[i], 32 * NC, 32 * c, 32, cin[c], S, lane);
    wg_end<WG>(A, dg.bc[i], S, lane);
  }
}

template <int NC, int NOUT, int GOFS, int WG, bool EMBG>
__device__ __forceinline__ void xyz_backward(const float* __restrict__ pk, const f32x16 (&cin)[NC],
                                             const float x[3], const float (&gall)[4], const nslam_dec_grad& dg,
                                             const Slab& A, const Scratch& S, int lane, f32x16& dc, float gx[3],
                                             const float* gh4 = nullptr) {
  const XyzPack L{NC};
  [[maybe_unused]] constexpr int DEC_ = NOUT == 3 ? 3 : (NC == 2 ? 2 : 1);
  const int h = lane >> 5;
  uint32_t m[5];
  f32x16 hs[4];
  const f32x16 h4 = xyz_forward<NC, WG != 0>(pk, cin, x, lane, m, hs);
  PHASE(DEC_, 4);

  // output layer: dh4 = Wo^T g
  f32x16 dh = zero16();
#pragma unroll
  for (int j = 0; j < NOUT; ++j) {
    const f32x16 w = vec_tile_g(pk + L.Wo() + 32 * j, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) dh[r] += w[r] * gall[GOFS + j];
  }
  add_gh4(dh, gh4, lane);
  if (WG) {
    tstore(S.sX, h4, lane);
    lds_sync();
    const int f = lane & 31;
#pragma unroll
    for (int j = 0; j < NOUT; ++j) {
      float s = 0.f;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int p = 2 * t + h;
        s += S.gtab[p * 4 + GOFS + j] * S.sX[p * TPITCH + f];
      }
      s += xor32(s);
      if (h == 0) put<WG>(A, f, dg.wo + 32 * j, s);
      if (lane == 0) {
        float sb = 0.f;
        for (int p = 0; p < 32; ++p) sb += S.gtab[p * 4 + GOFS + j];
        put<WG>(A, 0, dg.bo + j, sb);
      }
    }
    if (WG == 1 && GOFS + NOUT < 4 && GOFS == 0) {  // colour: output row 3 is never used, store zeros
#pragma unroll
      for (int j = NOUT; j < 4; ++j) {
        if (h == 0) put<1>(A, f, dg.wo + 32 * j, 0.f);
        if (lane == 0) put<1>(A, 0, dg.bo + j, 0.f);
      }
    }
    lds_sync();
  }
  dc = zero16();
  const float* FB = pk + L.FB();
  PHASE(DEC_, 5);

  // layer 4
  fc_bwd<NC, WG>(pk, L, 4, cin, dh, dg, A, S, lane, dc);
  f32x16 da = apply_mask(dh, m[4]);
  if (WG) {
    wg_begin(da, S, lane);
    wg_block<WG>(A, dg.w[4], 32, 0, 32, hs[3], S, lane);
    wg_end<WG>(A, dg.b[4], S, lane);
  }
  dh = zero16();
  gemm_acc(dh, pk + L.L4T() * NSLAM_FRAG, da, lane);
  PHASE(DEC_, 6);
  // layer 3 (input = [emb | h2])
  fc_bwd<NC, WG>(pk, L, 3, cin, dh, dg, A, S, lane, dc);
  const f32x16 da3 = apply_mask(dh, m[3]);
  if (WG) {
    wg_begin(da3, S, lane);
#pragma unroll
    for (int b = 0; b < 3; ++b)
      wg_block<WG>(A, dg.w[3], 125, 32 * b, b < 2 ? 32 : 29, emb_tile<false, true>(FB, x, b, lane), S, lane);
    wg_block<WG>(A, dg.w[3], 125, 93, 32, hs[2], S, lane);
    wg_end<WG>(A, dg.b[3], S, lane);
  }
  dh = zero16();
  gemm_acc(dh, pk + (L.L3T() + 3) * NSLAM_FRAG, da3, lane);
  PHASE(DEC_, 7);
  // layer 2
  fc_bwd<NC, WG>(pk, L, 2, cin, dh, dg, A, S, lane, dc);
  da = apply_mask(dh, m[2]);
  if (WG) {
    wg_begin(da, S, lane);
    wg_block<WG>(A, dg.w[2], 32, 0, 32, hs[1], S, lane);
    wg_end<WG>(A, dg.b[2], S, lane);
  }
  dh = zero16();
  gemm_acc(dh, pk + L.L2T() * NSLAM_FRAG, da, lane);
  PHASE(DEC_, 8);
  // layer 1
  fc_bwd<NC, WG>(pk, L, 1, cin, dh, dg, A, S, lane, dc);
  da = apply_mask(dh, m[1]);
  if (WG) {
    wg_begin(da, S, lane);
    wg_block<WG>(A, dg.w[1], 32, 0, 32, hs[0], S, lane);
    wg_end<WG>(A, dg.b[1], S, lane);
  }
  dh = zero16();
  gemm_acc(dh, pk + L.L1T() * NSLAM_FRAG, da, lane);
  PHASE(DEC_, 9);
  // layer 0 (input = emb)
  fc_bwd<NC, WG>(pk, L, 0, cin, dh, dg, A, S, lane, dc);
  da = apply_mask(dh, m[0]);
  if (WG) {
    wg_begin(da, S, lane);
#pragma unroll
    for (int b = 0; b < 3; ++b)
      wg_block<WG>(A, dg.w[0], 93, 32 * b, b < 2 ? 32 : 29, emb_tile<false, true>(FB, x, b, lane), S, lane);
    wg_end<WG>(A, dg.b[0], S, lane);
  }

  PHASE(DEC_, 10);
  // Fourier features: de_b = L3T_b da3 + L0T_b da0 ; G = de * cos(theta)
  gx[0] = gx[1] = gx[2] = 0.f;
  if (EMBG) {
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      f32x16 de = zero16();
      gemm_acc(de, pk + (L.L3T() + b) * NSLAM_FRAG, da3, lane);
      gemm_acc(de, pk + (L.L0T() + b) * NSLAM_FRAG, da, lane);
      const f32x16 cs = emb_tile<true, true>(FB, x, b, lane);
      f32x16 G;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 32 * b + 8 * i + 4 * h;
        const f32x4 B0 = *as_global(reinterpret_cast<const f32x4*>(FB + k));
        const f32x4 B1 = *as_global(reinterpret_cast<const f32x4*>(FB + 96 + k));
        const f32x4 B2 = *as_global(reinterpret_cast<const f32x4*>(FB + 192 + k));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float gk = de[4 * i + j] * cs[4 * i + j];
          G[4 * i + j] = gk;
          gx[0] += gk * B0[j];
          gx[1] += gk * B1[j];
          gx[2] += gk * B2[j];
        }
      }
      if (WG) {  // dB[j][k] += sum_p x_j[p] G[k][p]
        tstore(S.sA, G, lane);
        lds_sync();
        const int jj = lane & 31;
        const int jc = jj < 3 ? jj : 0;
        f32x16 acc = zero16();
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const int p = 2 * s + h;
          const float xv = jj < 3 ? S.xtab[p * 3 + jc] : 0.f;
          acc = mfma32(S.sA[p * TPITCH + jj], xv, acc);
        }
        if (jj < 3) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int k = 32 * b + fidx(r, h);
            if (k < NSLAM_EMB) put<WG>(A, jj * NSLAM_EMB + 4 * h, dg.B + 32 * b + (r & 3) + 8 * (r >> 2), acc[r]);
          }
        }
        lds_sync();
      }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) gx[k] += xor32(gx[k]);
  }
  PHASE(DEC_, 11);
}

// ------------------------------------------------------------------------------------------
// MLP_no_xyz (coarse, decoder.py:262-274): forward / backward
// ------------------------------------------------------------------------------------------
template <bool KEEP>
__device__ __forceinline__ f32x16 noxyz_forward(const float* __restrict__ pk, const f32x16& c, int lane,
                                                uint32_t m[5], f32x16* hs) {
  const NoXyzPack L;
  f32x16 a = vec_tile_g(pk + L.Bias(0), lane);
  gemm_acc(a, pk + L.L0() * NSLAM_FRAG, c, lane);
  f32x16 a3 = vec_tile_g(pk + L.Bias(3), lane);
  gemm_acc(a3, pk + L.L3() * NSLAM_FRAG, c, lane);
  m[0] = mask16(a);
  f32x16 h = relu16(a);
  if (KEEP) hs[0] = h;
  a = vec_tile_g(pk + L.Bias(1), lane);
  gemm_acc(a, pk + L.L1() * NSLAM_FRAG, h, lane);
  m[1] = mask16(a);
  h = relu16(a);
  if (KEEP) hs[1] = h;
  a = vec_tile_g(pk + L.Bias(2), lane);
  gemm_acc(a, pk + L.L2() * NSLAM_FRAG, h, lane);
  m[2] = mask16(a);
  h = relu16(a);
  if (KEEP) hs[2] = h;
  gemm_acc(a3, pk + (L.L3() + 1) * NSLAM_FRAG, h, lane);
  m[3] = mask16(a3);
  h = relu16(a3);
  if (KEEP) hs[3] = h;
  a = vec_tile_g(pk + L.Bias(4), lane);
  gemm_acc(a, pk + L.L4() * NSLAM_FRAG, h, lane);
  m[4] = mask16(a);
  return relu16(a);
}

template <int WG>
__device__ __forceinline__ void noxyz_backward(const float* __restrict__ pk, const f32x16& c, float g,
                                               const nslam_dec_grad& dg, const Slab& A, const Scratch& S, int lane,
                                               f32x16& dc) {
  const NoXyzPack L;
  const int h = lane >> 5;
  uint32_t m[5];
  f32x16 hs[4];
  const f32x16 h4 = noxyz_forward<WG != 0>(pk, c, lane, m, hs);
  f32x16 dh;
  {
    const f32x16 w = vec_tile_g(pk + L.Wo(), lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) dh[r] = w[r] * g;
  }
  if (WG) {
    tstore(S.sX, h4, lane);
    lds_sync();
    const int f = lane & 31;
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int p = 2 * t + h;
      s += S.gtab[p * 4 + 3] * S.sX[p * TPITCH + f];
    }
    s += xor32(s);
    if (h == 0) put<WG>(A, f, dg.wo, s);
    if (lane == 0) {
      float sb = 0.f;
      for (int p = 0; p < 32; ++p) sb += S.gtab[p * 4 + 3];
      put<WG>(A, 0, dg.bo, sb);
    }
    lds_sync();
  }
  dc = zero16();
  // layer 4
  f32x16 da = apply_mask(dh, m[4]);
  if (WG) {
    wg_begin(da, S, lane);
    wg_block<WG>(A, dg.w[4], 32, 0, 32, hs[3], S, lane);
    wg_end<WG>(A, dg.b[4], S, lane);
  }
  dh = zero16();
  gemm_acc(dh, pk + L.L4T() * NSLAM_FRAG, da, lane);
  // layer 3 (input = [c | h2])
  da = apply_mask(dh, m[3]);
  if (WG) {
    wg_begin(da, S, lane);
    wg_block<WG>(A, dg.w[3], 64, 0, 32, c, S, lane);
    wg_block<WG>(A, dg.w[3], 64, 32, 32, hs[2], S, lane);
    wg_end<WG>(A, dg.b[3], S, lane);
  }
  gemm_acc(dc, pk + L.L3T() * NSLAM_FRAG, da, lane);
  dh = zero16();
  gemm_acc(dh, pk + (L.L3T() + 1) * NSLAM_FRAG, da, lane);
  // layer 2
  da = apply_mask(dh, m[2]);
  if (WG) {
    wg_begin(da, S, lane);
    wg_block<WG>(A, dg.w[2], 32, 0, 32, hs[1], S, lane);
    wg_end<WG>(A, dg.b[2], S, lane);
  }
  dh = zero16();
  gemm_acc(dh, pk + L.L2T() * NSLAM_FRAG, da, lane);
  // layer 1
  da = apply_mask(dh, m[1]);
  if (WG) {
    wg_begin(da, S, lane);
    wg_block<WG>(A, dg.w[1], 32, 0, 32, hs[0], S, lane);
    wg_end<WG>(A, dg.b[1], S, lane);
  }
  dh = zero16();
  gemm_acc(dh, pk + L.L1T() * NSLAM_FRAG, da, lane);
  // layer 0 (input = c)
  da = apply_mask(dh, m[0]);
  if (WG) {
    wg_begin(da, S, lane);
    wg_block<WG>(A, dg.w[0], 32, 0, 32, c, S, lane);
    wg_end<WG>(A, dg.b[0], S, lane);
  }
  gemm_acc(dc, pk + L.L0T() * NSLAM_FRAG, da, lane);
}

// ------------------------------------------------------------------------------------------
// Backward from saved ReLU masks (decoders without parameter gradients): no forward recompute,
// no embedding sin, no feature gather.  dh_4 = Wo^T g; for i = 4..0: dc += FCT_i dh_i and
// dh_{i-1} = L_iT mask_i(dh_i) (layer 3 through its hidden block); EMBG adds d/dx through the
// Fourier features from mask_3(dh_3) and mask_0(dh_0).
// ------------------------------------------------------------------------------------------
// TR: dc is formed transposed (lane (c, h) register r = channel c of point F(r, h); gemm_acc_t), the
// layout the lean scatter walk consumes without an LDS transpose (only without EMBG: coord_grad
// reads the C layout)
// img (EMBG; the d/dpts mask-only kernels): the caller's scatter image — dc, complete before the Fourier
// backward, is stored there (tstore layout) and does not hold 16 registers through it (the caller's
// scatter reads it there; its coordinate gradient reads it back: tload)
template <int NC, int NOUT, int GOFS, bool EMBG, bool TR = false>
__device__ __forceinline__ void xyz_backward_saved(const float* __restrict__ pk, const uint32_t m[5],
                                                   const float x[3], const float (&gall)[4], int lane, f32x16& dc,
                                                   float gx[3], const float* gh4 = nullptr,
                                                   float* __restrict__ img = nullptr) {
  static_assert(!(TR && EMBG), "d/dpts needs dc in the C layout");
  const XyzPack L{NC};
  const int h = lane >> 5;
  f32x16 dh = zero16();
#pragma unroll
  for (int j = 0; j < NOUT; ++j) {
    const f32x16 w = vec_tile_g(pk + L.Wo() + 32 * j, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) dh[r] += w[r] * gall[GOFS + j];
  }
  add_gh4(dh, gh4, lane);
  dc = zero16();
  gemm_acc_tr<TR>(dc, pk + L.FCT(4) * NSLAM_FRAG, dh, lane);
  f32x16 da = apply_mask(dh, m[4]);
  dh = zero16();
  gemm_acc(dh, pk + L.L4T() * NSLAM_FRAG, da, lane);
  gemm_acc_tr<TR>(dc, pk + L.FCT(3) * NSLAM_FRAG, dh, lane);
  const f32x16 da3 = apply_mask(dh, m[3]);
  dh = zero16();
  gemm_acc(dh, pk + (L.L3T() + 3) * NSLAM_FRAG, da3, lane);
  gemm_acc_tr<TR>(dc, pk + L.FCT(2) * NSLAM_FRAG, dh, lane);
  da = apply_mask(dh, m[2]);
  dh = zero16();
  gemm_acc(dh, pk + L.L2T() * NSLAM_FRAG, da, lane);
  gemm_acc_tr<TR>(dc, pk + L.FCT(1) * NSLAM_FRAG, dh, lane);
  da = apply_mask(dh, m[1]);
  dh = zero16();
  gemm_acc(dh, pk + L.L1T() * NSLAM_FRAG, da, lane);
  gemm_acc_tr<TR>(dc, pk + L.FCT(0) * NSLAM_FRAG, dh, lane);
  gx[0] = gx[1] = gx[2] = 0.f;
  if (EMBG) {
    da = apply_mask(dh, m[0]);
    if (img) {
      tstore(img, dc, lane);
      asm volatile("" ::: "memory");  // (read back after the scatter, not kept in registers meanwhile)
    }
    const float* FB = pk + L.FB();
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      f32x16 de = zero16();
      gemm_acc(de, pk + (L.L3T() + b) * NSLAM_FRAG, da3, lane);
      gemm_acc(de, pk + (L.L0T() + b) * NSLAM_FRAG, da, lane);
      const f32x16 cs = emb_tile<true, true>(FB, x, b, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 32 * b + 8 * i + 4 * h;
        const f32x4 B0 = *as_global(reinterpret_cast<const f32x4*>(FB + k));
        const f32x4 B1 = *as_global(reinterpret_cast<const f32x4*>(FB + 96 + k));
        const f32x4 B2 = *as_global(reinterpret_cast<const f32x4*>(FB + 192 + k));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float gk = de[4 * i + j] * cs[4 * i + j];
          gx[0] += gk * B0[j];
          gx[1] += gk * B1[j];
          gx[2] += gk * B2[j];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) gx[k] += xor32(gx[k]);
  }
}

template <bool TR = false>
__device__ __forceinline__ void noxyz_backward_saved(const float* __restrict__ pk, const uint32_t m[5], float g,
                                                     int lane, f32x16& dc) {
  const NoXyzPack L;
  f32x16 dh;
  {
    const f32x16 w = vec_tile_g(pk + L.Wo(), lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) dh[r] = w[r] * g;
  }
  dc = zero16();
  f32x16 da = apply_mask(dh, m[4]);
  dh = zero16();
  gemm_acc(dh, pk + L.L4T() * NSLAM_FRAG, da, lane);
  da = apply_mask(dh, m[3]);
  gemm_acc_tr<TR>(dc, pk + L.L3T() * NSLAM_FRAG, da, lane);
  dh = zero16();
  gemm_acc(dh, pk + (L.L3T() + 1) * NSLAM_FRAG, da, lane);
  da = apply_mask(dh, m[2]);
  dh = zero16();
  gemm_acc(dh, pk + L.L2T() * NSLAM_FRAG, da, lane);
  da = apply_mask(dh, m[1]);
  dh = zero16();
  gemm_acc(dh, pk + L.L1T() * NSLAM_FRAG, da, lane);
  da = apply_mask(dh, m[0]);
  gemm_acc_tr<TR>(dc, pk + L.L0T() * NSLAM_FRAG, da, lane);
}

// ------------------------------------------------------------------------------------------
// grid gradient scatter (atomics shaped as two 128-B row segments per wave-instruction) and
// coordinate gradient through the trilinear weights
// ------------------------------------------------------------------------------------------
// Stage a tile's corner rows / weights for the scatter.  With a slot map (ABI v6: frustum-
// compacted grid gradient, Mapper.py:314-333) corner row r accumulates into compact row slot[r];
// corners outside the frustum selection (slot -1) get weight 0, i.e. no atomic: the reference
// never forms their gradient (its optimised tensor is the masked vector, Mapper.py:394-401).
__device__ __forceinline__ void stage_corners(const Corners& cr, const int32_t* __restrict__ slot, bool valid,
                                              const Scratch& S, int lane) {
  if (lane < 32) {
    const int p = lane;
    S.ccell[p] = cr.cell;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      int r = cr.row[k];
      float w = valid ? cr.w[k] : 0.f;
      if (slot) {
        r = slot[r];
        if (r < 0) {
          r = 0;
          w = 0.f;
        }
      }
      S.crow[p * 8 + k] = r;
      S.cw[p * 8 + k] = w;
    }
  }
}


// grid-gradient add of one lane's channel
__device__ __forceinline__ void grid_add(float* p, float v) { unsafeAtomicAdd(p, v); }

__device__ __forceinline__ float rdlane(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// Corners 4h..4h+3 of this lane's point, frustum-slot mapped (slot -1: weight 0, no atomic).
// Issued right after the corners are known, so the slot gathers' latency hides behind the
// decoder backward instead of stalling the scatter.
struct ScatterCorners {
  int rk[4];
  float wk[4];
};
__device__ __forceinline__ ScatterCorners resolve_corners(const int32_t* __restrict__ slot, const Corners& cr,
                                                          bool valid, int lane) {
  const int h = lane >> 5;
  ScatterCorners sc;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int r = h ? cr.row[4 + i] : cr.row[i];
    float w = valid ? (h ? cr.w[4 + i] : cr.w[i]) : 0.f;
    if (slot) {
      r = slot[r];
      if (r < 0) {
        r = 0;
        w = 0.f;
      }
    }
    sc.rk[i] = r;
    sc.wk[i] = w;
  }
  return sc;
}

// The walk keeps each corner voxel of the current cell in a register chosen by the voxel's own
// coordinate parities, not by its position in the cell: lane half h holds the corners with
// x & 1 == h, register j those with (y & 1) + 2 (z & 1) == j.  Stepping to a neighbouring cell then
// leaves every shared voxel where it is (its running sum simply continues), and only the voxels
// that leave the cell are flushed and their registers cleared — no data moves between registers.
// Walk table of one tile (per wave, kWalkFloats): entry (p, h) holds point p's weights (then its
// frustum rows) of the four corners in lane half h, register order j, so one ds_read_b128 with a
// half-uniform address (an LDS broadcast) fetches them.
constexpr int kWalkFloats = 2 * 32 * 8;
__device__ __forceinline__ void stage_walk_table(float* __restrict__ tab, const ScatterCorners& sc, int cellk,
                                                 int lane) {
  // lane (hz, p) resolved corners 4 hz + i, i = dx + 2 dy, of the cell with lower corner cellk
  const int hz = lane >> 5, p = lane & 31;
  const int px = cellk & 1, py = (cellk >> 10) & 1, pz = (cellk >> 20) & 1;
  float* w = tab + p * 8;
  int* r = reinterpret_cast<int*>(tab + 256) + p * 8;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = (((i & 1) ^ px) << 2) | ((i >> 1) ^ py) | ((hz ^ pz) << 1);
    w[e] = sc.wk[i];
    r[e] = sc.rk[i];
  }
}

// Step codes of the walk: every lane evaluates, in parallel before the
// walk, what the step from point p-1's cell to point p's does — bit 8: the cell changes; bit 4 hh + j:
// voxel (hh, j) of the previous cell is kept (a neighbouring-cell step).  The walk itself then
// reads one code per point (v_readlane) instead of deriving the steps' axis deltas and parities on the
// scalar unit point after point (~3k SALU instructions per tile, shared by the CU's waves).
__device__ __forceinline__ int walk_code(int cellk, int lane) {
  const int p = lane & 31;
  const int prev = __shfl(cellk, (lane & 32) | ((p + 31) & 31), 64);  // point p - 1 (same half)
  if (p == 0) return 0x100;        // the first point: nothing accumulated, nothing kept
  if (prev == cellk) return 0;     // the same cell: no step
  const int ax = (cellk & 1023) - (prev & 1023);
  const int ay = ((cellk >> 10) & 1023) - ((prev >> 10) & 1023);
  const int az = (cellk >> 20) - (prev >> 20);
  const int px = prev & 1, py = (prev >> 10) & 1, pz = (prev >> 20) & 1;
  int code = 0x100;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const bool kx = ax == 0 || (ax == 1 && (hh ^ px) == 1) || (ax == -1 && (hh ^ px) == 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int dy = (j & 1) ^ py, dz = (j >> 1) ^ pz;
      const bool ky = ay == 0 || (ay == 1 && dy == 1) || (ay == -1 && dy == 0);
      const bool kz = az == 0 || (az == 1 && dz == 1) || (az == -1 && dz == 0);
      if (kx && ky && kz) code |= 1 << (4 * hh + j);
    }
  }
  return code;
}

// STAGED: the caller wrote the walk table already.  TR: dc arrives transposed (xyz_backward_saved<..., TR>):
// lane (ch, h) holds channel ch of points F(r, h), and one v_permlane32_swap per register hands every
// lane both halves' points — the walk's cotangent columns straight from registers, no LDS image.
template <bool STAGED = false, bool TR = false, bool IMG_READY = false>
__device__ __forceinline__ void scatter_grid_grad_uniform(float* __restrict__ grad, const ScatterCorners& sc,
                                                          int cellk, const f32x16& dc, float* __restrict__ img,
                                                          float* __restrict__ tab, int lane) {
  // Points of a tile are consecutive samples of (mostly) one ray: a voxel's contributions from a
  // run of cells touching it are summed in one register and flushed once (one atomic per voxel per
  // run).  The whole wave walks the tile's 32 points in step (fully unrolled, uniform control
  // flow); lane (h, ch) owns channel ch of its half's four corners, and the two halves hold x-
  // neighbours, i.e. adjacent rows of the channels-last grid, so every flush wave-instruction adds
  // one contiguous 256-B segment (the full-rate shape of a float atomic).  Per point: the cell by
  // v_readlane (it steers the uniform branch), weights and rows by broadcast LDS reads of the walk
  // table, and the cotangent column of channel ch from one LDS transpose of dc.
  const int h = lane >> 5, ch = lane & 31;
  float vlo[16], vhi[16];  // TR: channel ch of point F(r, 0) / F(r, 1)
  if (TR) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      // (through a scalar: clang's __builtin_bit_cast of a vector-element lvalue reads element 0)
      const float d = dc[r];
      const unsigned u = __builtin_bit_cast(unsigned, d);
      const auto sw = __builtin_amdgcn_permlane32_swap(u, u, false, false);  // {lower half's, upper half's}
      vlo[r] = __builtin_bit_cast(float, (unsigned)sw[0]);
      vhi[r] = __builtin_bit_cast(float, (unsigned)sw[1]);
    }
  } else if (!IMG_READY) {  // (IMG_READY: the caller's chain left dc in img already)
    tstore(img, dc, lane);
  }
  if (!STAGED) stage_walk_table(tab, sc, cellk, lane);
  lds_sync();
  const f32x4* wt = reinterpret_cast<const f32x4*>(tab) + h;        // (t, h) at wt[2 t]
  const i32x4* rt = reinterpret_cast<const i32x4*>(tab + 256) + h;  // (t, h) at rt[2 t]
  float acc[4], wsum[4];
  int rows[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    acc[j] = 0.f;
    wsum[j] = 0.f;
    rows[j] = 0;
  }
  const int codes = walk_code(cellk, lane);
#pragma unroll
  for (int t = 0; t < 32; ++t) {
    const int code = __builtin_amdgcn_readlane(codes, t);
    // point t = F(r, hh): r = (t & 3) + 4 (t >> 3), hh = (t >> 2) & 1
    const float vc = TR ? (((t >> 2) & 1) ? vhi[(t & 3) + 4 * (t >> 3)] : vlo[(t & 3) + 4 * (t >> 3)])
                        : img[t * TPITCH + ch];
    const f32x4 w = wt[2 * t];
    const i32x4 nr = rt[2 * t];
    if (code & 0x100) {  // wave-uniform: the walk steps to another cell
      const int kb = code >> (4 * h);  // this half's voxels of the previous cell that stay
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool keep = (kb >> j) & 1;
        // one exec-masked flush (both conditions evaluated: no nested branch)
        if ((!keep) & (wsum[j] != 0.f)) grid_add(grad + (size_t)rows[j] * NSLAM_C_DIM + ch, acc[j]);
        acc[j] = keep ? acc[j] : 0.f;
        wsum[j] = keep ? wsum[j] : 0.f;
        rows[j] = nr[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[j] += w[j] * vc;
      wsum[j] += w[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (wsum[j] != 0.f) grid_add(grad + (size_t)rows[j] * NSLAM_C_DIM + ch, acc[j]);
  lds_sync();
}

// Per-half variant (weight-gradient kernels): half h walks points 16h..16h+15 on its own, every
// flush wave-instruction is one 128-B row segment.  Kept for the register-starved weight-gradient
// kernels, where the uniform variant above coincided with an illegal-address fault in the fine
// decoder's kernel (both runs of tests/test_gpu_parity.py eval fine, r1k and r1l).
__device__ __forceinline__ void scatter_grid_grad_halves(float* __restrict__ grad, const int32_t* __restrict__ slot,
                                                         const Corners& cr, const f32x16& dc, bool valid,
                                                         const Scratch& S, int lane) {
  const int h = lane >> 5, ch = lane & 31;
  tstore(S.sA, dc, lane);
  stage_corners(cr, slot, valid, S, lane);
  lds_sync();
  float acc[8], wsum[8];
  int rows[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    acc[k] = 0.f;
    wsum[k] = 0.f;
    rows[k] = 0;
  }
  int cur = -1;
  for (int t = 0; t < 16; ++t) {
    const int pp = 16 * h + t;
    const int cell = S.ccell[pp];
    if (cell != cur) {
      if (cur >= 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (wsum[k] != 0.f) grid_add(grad + (size_t)rows[k] * NSLAM_C_DIM + ch, acc[k]);
      }
      cur = cell;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        acc[k] = 0.f;
        wsum[k] = 0.f;
        rows[k] = S.crow[pp * 8 + k];
      }
    }
    const float v = S.sA[pp * TPITCH + ch];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float w = S.cw[pp * 8 + k];
      acc[k] += w * v;
      wsum[k] += w;
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (wsum[k] != 0.f) grid_add(grad + (size_t)rows[k] * NSLAM_C_DIM + ch, acc[k]);
  lds_sync();
}

__device__ __forceinline__ void coord_grad(const nslam_grid& g, const Corners& cr, const f32x16& dc, int lane,
                                           double gp[3]) {
  float part[3];
  coord_grad_partial(g.data, cr, dc, lane, part);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float gn = (part[k] + xor32(part[k])) * cr.gmul[k];
    gp[k] += ((double)gn * 2.0) / (g.hi[k] - g.lo[k]);
  }
}

// ------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------
template <int STAGE>
__global__ __launch_bounds__(256, 2) void k_query_fwd(QueryKArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t tile = (int64_t)blockIdx.x * 4 + wave_id();
  if (tile * 32 >= a.n) return;  // wave-uniform
  const int h = lane >> 5;
  const Pt q = load_point(a, tile * 32 + (lane & 31));
  float out[4] = {0.f, 0.f, 0.f, 0.f};
  uint32_t m[5];
  if (STAGE == NSLAM_STAGE_COARSE) {
    Corners cr;
    grid_corners(cr, a.c.grid[NSLAM_DEC_COARSE], q);
    const f32x16 c = gather_tile(a.c.grid[NSLAM_DEC_COARSE].data, cr, lane);
    const float* pk = a.c.packed[NSLAM_DEC_COARSE];
    const NoXyzPack L;
    const f32x16 h4 = noxyz_forward<false>(pk, c, lane, m, nullptr);
    save_masks(a, NSLAM_DEC_COARSE, tile, m, lane);
    out[3] = out_row(pk + L.Wo(), pk + L.Bo(), 0, h4, lane);
  } else {
    Corners cr;
    grid_corners(cr, a.c.grid[NSLAM_DEC_MIDDLE], q);
    const f32x16 cm[1] = {gather_tile(a.c.grid[NSLAM_DEC_MIDDLE].data, cr, lane)};
    {
      const float* pk = a.c.packed[NSLAM_DEC_MIDDLE];
      const XyzPack L{1};
      const f32x16 h4 = xyz_forward<1, false>(pk, cm, q.x, lane, m, nullptr);
      save_masks(a, NSLAM_DEC_MIDDLE, tile, m, lane);
      out[3] = out_row(pk + L.Wo(), pk + L.Bo(), 0, h4, lane);
    }
    if (STAGE >= NSLAM_STAGE_FINE) {
      grid_corners(cr, a.c.grid[NSLAM_DEC_FINE], q);
      const f32x16 cf[2] = {gather_tile(a.c.grid[NSLAM_DEC_FINE].data, cr, lane), cm[0]};
      const float* pk = a.c.packed[NSLAM_DEC_FINE];
      const XyzPack L{2};
      const f32x16 h4 = xyz_forward<2, false>(pk, cf, q.x, lane, m, nullptr);
      save_masks(a, NSLAM_DEC_FINE, tile, m, lane);
      out[3] = out_row(pk + L.Wo(), pk + L.Bo(), 0, h4, lane) + out[3];  // fine_occ + middle_occ
    }
    if (STAGE == NSLAM_STAGE_COLOR) {
      grid_corners(cr, a.c.grid[NSLAM_DEC_COLOR], q);
      const f32x16 cc[1] = {gather_tile(a.c.grid[NSLAM_DEC_COLOR].data, cr, lane)};
      const float* pk = a.c.packed[NSLAM_DEC_COLOR];
      const XyzPack L{1};
      f32x16 h4;
      if (a.c.act_tape)
        h4 = xyz_forward<1, false, false, true>(pk, cc, q.x, lane, m, nullptr, a.c.act_tape + tile * kTapeFloats);
      else
        h4 = xyz_forward<1, false>(pk, cc, q.x, lane, m, nullptr);
      save_masks(a, NSLAM_DEC_COLOR, tile, m, lane);
#pragma unroll
      for (int j = 0; j < 3; ++j) out[j] = out_row(pk + L.Wo(), pk + L.Bo(), j, h4, lane);
    }
  }
  if (!q.inside) out[3] = 100.f;  // Renderer.py:57
  if (h == 0 && q.valid) {
    f32x4 v;
    v[0] = out[0];
    v[1] = out[1];
    v[2] = out[2];
    v[3] = out[3];
    *reinterpret_cast<f32x4*>(a.raw + (tile * 32 + (lane & 31)) * 4) = v;
  }
}

// Decoder-parallel forward (fine and colour stages): each workgroup evaluates ONE decoder for its
// 4 tiles, so a launch has 2-3x the waves of k_query_fwd (room0 mapping: 4500 instead of 1500 on
// 1024 SIMDs) and every wave a third of the serial MFMA/gather chain.  Parts are interleaved
// over blockIdx (heavy fine and light middle/colour workgroups mix on every CU):
//   part 0  middle: occ_mid[p] = inside ? middle_occ : 100
//   part 1  fine:   raw[p][3]  = inside ? fine_occ : 0     (fine stage: the whole row)
//   part 2  colour: raw[p][0..2]
// and k_occ_combine then forms raw[p][3] = fine_occ + middle_occ (decoder.py:331-334, the
// reference's operand order) — exactly 100 outside the bound (0 + 100; Renderer.py:57).
// One decoder of the decoder-parallel forward for this wave's tile.
// the middle decoder's chain and output for this wave's tile from its gathered feature cm
__device__ __forceinline__ void fwd_middle_chain(const QueryKArgs& a, const Pt& q, int64_t tile, int64_t idx,
                                                 int lane, float* __restrict__ occ_mid, const float* vec,
                                                 const f32x16& cm) {
  const int h = lane >> 5;
  uint32_t m[5];
  const float* pk = a.c.packed[NSLAM_DEC_MIDDLE];
  const XyzPack L{1};
  const f32x16 cms[1] = {cm};
  const f32x16 h4 = xyz_forward_pf<1, false>(pk, cms, q.x, lane, m, nullptr, vec);
  save_masks(a, NSLAM_DEC_MIDDLE, tile, m, lane);
  float o = out_row(vec + (L.Wo() - L.V()), vec + (L.Bo() - L.V()), 0, h4, lane);
  if (!q.inside) o = 100.f;
  if (h == 0 && q.valid) occ_mid[idx] = o;
}
__device__ __forceinline__ void fwd_part_middle(const QueryKArgs& a, const Pt& q, int64_t tile, int64_t idx, int lane,
                                                float* __restrict__ occ_mid, const float* vec) {
  Corners cr;
  grid_corners(cr, a.c.grid[NSLAM_DEC_MIDDLE], q);
  PHASE(0, 2);
  const f32x16 cm = gather_tile(a.c.grid[NSLAM_DEC_MIDDLE].data, cr, lane);
  PHASE(0, 3);
  fwd_middle_chain(a, q, tile, idx, lane, occ_mid, vec, cm);
}

template <int STAGE>
__device__ __forceinline__ void fwd_part_fine(const QueryKArgs& a, const Pt& q, int64_t tile, int64_t idx, int lane,
                                              const float* vec) {
  // the fine decoder also reads the middle feature (decoder.py:184-187)
  const int h = lane >> 5;
  uint32_t m[5];
  PHASE(0, 2);
  f32x16 cf[2];
#if NSLAM_UNITS_PAIR
  gather_pair(a.c.grid[NSLAM_DEC_FINE], a.c.grid[NSLAM_DEC_MIDDLE], q, lane, cf[0], cf[1]);
#else
  cf[0] = gather_one(a.c.grid[NSLAM_DEC_FINE], q, lane);
  cf[1] = gather_one(a.c.grid[NSLAM_DEC_MIDDLE], q, lane);
#endif
  PHASE(0, 3);
  const float* pk = a.c.packed[NSLAM_DEC_FINE];
  const XyzPack L{2};
  const f32x16 h4 = xyz_forward_pf<2, false>(pk, cf, q.x, lane, m, nullptr, vec);
  save_masks(a, NSLAM_DEC_FINE, tile, m, lane);
  float o = out_row(vec + (L.Wo() - L.V()), vec + (L.Bo() - L.V()), 0, h4, lane);
  if (!q.inside) o = 0.f;
  if (h == 0 && q.valid) {
    if (STAGE == NSLAM_STAGE_COLOR) {
      a.raw[idx * 4 + 3] = o;
    } else {
      f32x4 v = {0.f, 0.f, 0.f, o};
      *reinterpret_cast<f32x4*>(a.raw + idx * 4) = v;
    }
  }
}

// the colour decoder's chain (+ activation tape) and outputs for this wave's tile from its feature cc
template <bool TAPE>
__device__ __forceinline__ void fwd_color_chain(const QueryKArgs& a, const Pt& q, int64_t tile, int64_t idx,
                                                int lane, const float* vec, const f32x16& cc) {
  const int h = lane >> 5;
  uint32_t m[5];
  const float* pk = a.c.packed[NSLAM_DEC_COLOR];
  const XyzPack L{1};
  float* tp = TAPE ? a.c.act_tape + tile * kTapeFloats : nullptr;
  const f32x16 ccs[1] = {cc};
  const f32x16 h4 = xyz_forward_pf<1, TAPE, 12>(pk, ccs, q.x, lane, m, tp, vec);
  save_masks(a, NSLAM_DEC_COLOR, tile, m, lane);
  float o[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) o[j] = out_row(vec + (L.Wo() - L.V()), vec + (L.Bo() - L.V()), j, h4, lane);
  if (h == 0 && q.valid) {
#pragma unroll
    for (int j = 0; j < 3; ++j) a.raw[idx * 4 + j] = o[j];
  }
}
template <bool TAPE>
__device__ __forceinline__ void fwd_part_color(const QueryKArgs& a, const Pt& q, int64_t tile, int64_t idx, int lane,
                                               const float* vec) {
  Corners cr;
  grid_corners(cr, a.c.grid[NSLAM_DEC_COLOR], q);
  PHASE(0, 10);
  const f32x16 cc = gather_tile(a.c.grid[NSLAM_DEC_COLOR].data, cr, lane);
  PHASE(0, 11);
  fwd_color_chain<TAPE>(a, q, tile, idx, lane, vec, cc);
}

// Decoder-parallel forward (fine and colour stages): each workgroup evaluates ONE part for its 4
// tiles, so a launch has 2-3x the waves of k_query_fwd and every wave a fraction of the serial
// MFMA/gather chain.  Parts are interleaved over blockIdx (heavy and light workgroups mix on
// every CU).  NPARTS = 3 (colour stage): middle | fine | colour; NPARTS = 2: fine stage middle |
// fine, or colour stage (middle then colour) | fine — fewer, balanced waves (3000 at room0) that
// fit the chip's wave slots in one round.
//   middle: occ_mid[p] = inside ? middle_occ : 100
//   fine:   raw[p][3]  = inside ? fine_occ : 0     (fine stage: the whole row)
//   colour: raw[p][0..2]
// and k_occ_combine (or the loss kernel, defer_occ) then forms raw[p][3] = fine_occ + middle_occ
// (decoder.py:331-334, the reference's operand order) — exactly 100 outside the bound (0 + 100;
// Renderer.py:57).
#ifndef NSLAM_FWD_LB
#define NSLAM_FWD_LB 2  // min waves per SIMD (experiments: 3..5 trade VGPRs for occupancy)
#endif
// register cap of the forward (experiments: a SIMD's wave slots are shared with the ray prefetch's
// sampler / gather waves of the next iteration, which run beside this launch)
#ifdef NSLAM_FWD_NUMVGPR
#define NSLAM_FWD_ATTR __attribute__((amdgpu_num_vgpr(NSLAM_FWD_NUMVGPR)))
#else
#define NSLAM_FWD_ATTR
#endif
constexpr int kVecFloats = 744;  // XyzPack vector section (740) rounded to float4s
template <int STAGE, int NPARTS, bool TAPE>
NSLAM_FWD_ATTR __global__ __launch_bounds__(256, NSLAM_FWD_LB) void k_query_fwd_parts(QueryKArgs a,
                                                                                     float* __restrict__ occ_mid) {
  const int part = (int)(blockIdx.x % NPARTS);
  const int lane = threadIdx.x & 63;
  TL(0, 0, part);
  // The part's decoder vector sections (biases, output rows, Fourier B: ~3 KiB each) are read by
  // every layer of every wave: an LDS copy per workgroup turns ~90 global loads per wave into
  // ds_reads.  Part 0 of the 2-part colour forward evaluates middle then colour: two copies.
  __shared__ __attribute__((aligned(16))) float vsec[2][kVecFloats];
  {
    const int d0 = part == 0 ? NSLAM_DEC_MIDDLE : part == 1 ? NSLAM_DEC_FINE : NSLAM_DEC_COLOR;
    const int nc0 = d0 == NSLAM_DEC_FINE ? 2 : 1;
    const float* src0 = a.c.packed[d0] + XyzPack{nc0}.V();
    const bool two = NPARTS == 2 && STAGE == NSLAM_STAGE_COLOR && part == 0;
    const float* src1 = two ? a.c.packed[NSLAM_DEC_COLOR] + XyzPack{1}.V() : nullptr;
    for (int i = threadIdx.x; i < 740; i += 256) {
      vsec[0][i] = src0[i];
      if (two) vsec[1][i] = src1[i];
    }
    __syncthreads();
  }
  const int64_t tile = (int64_t)(blockIdx.x / NPARTS) * 4 + wave_id();
  if (tile * 32 >= a.n) return;  // wave-uniform
  const int64_t idx = tile * 32 + (lane & 31);
  PHASE(0, 0);
  const Pt q = load_point(a, idx);
  PHASE(0, 1);
  if (NPARTS == 2 && STAGE == NSLAM_STAGE_COLOR) {
    if (part == 0) {
      fwd_part_middle(a, q, tile, idx, lane, occ_mid, vsec[0]);
      fwd_part_color<TAPE>(a, q, tile, idx, lane, vsec[1]);
    } else {
      fwd_part_fine<STAGE>(a, q, tile, idx, lane, vsec[0]);
    }
  } else if (part == 0) {
    fwd_part_middle(a, q, tile, idx, lane, occ_mid, vsec[0]);
  } else if (part == 1) {
    fwd_part_fine<STAGE>(a, q, tile, idx, lane, vsec[0]);
  } else if (STAGE == NSLAM_STAGE_COLOR) {
    fwd_part_color<TAPE>(a, q, tile, idx, lane, vsec[0]);
  }
  PHASE(0, 9);
  TL(0, 1, 0);
}

// Decoder-parallel forward with DYNAMIC work distribution: the same per-decoder units (one decoder of one
// 32-point tile: fwd_part_fine / fwd_part_middle / fwd_part_color, the same arithmetic and outputs as
// k_query_fwd_parts), but a launch of at most one wave per wave slot whose waves take units off a
// device counter until none is left — the heaviest (fine: two gathers, 20 GEMMs) first.  A SIMD whose
// waves drew light units takes more of them, so the launch ends when the chip's work does, not when the
// unluckiest SIMD's statically assigned mix does.  ctr: 2 uint32 zeroed before the launch.
template <int STAGE, bool TAPE>
__global__ __launch_bounds__(256, 3) void k_query_fwd_dyn(QueryKArgs a, float* __restrict__ occ_mid,
                                                                      unsigned* __restrict__ ctr) {
  constexpr int NP = STAGE == NSLAM_STAGE_COLOR ? 3 : 2;
  // every part's vector section (biases, output rows, Fourier B) once per workgroup
  __shared__ __attribute__((aligned(16))) float vsec[NP][kVecFloats];
  {
    const float* s0 = a.c.packed[NSLAM_DEC_MIDDLE] + XyzPack{1}.V();
    const float* s1 = a.c.packed[NSLAM_DEC_FINE] + XyzPack{2}.V();
    const float* s2 = NP == 3 ? a.c.packed[NSLAM_DEC_COLOR] + XyzPack{1}.V() : nullptr;
    for (int i = threadIdx.x; i < 740; i += 256) {
      vsec[0][i] = s0[i];
      vsec[1][i] = s1[i];
      if (NP == 3) vsec[NP - 1][i] = s2[i];
    }
    __syncthreads();
  }
  const int lane0 = threadIdx.x & 63;
  const int64_t ntiles = (a.n + 31) / 32;
  const int64_t nunits = ntiles * NP;
  TL(0, 0, 0);
  for (;;) {
    unsigned u = 0;
    if (lane0 == 0) u = atomicAdd(ctr, 1u);
    u = __builtin_amdgcn_readfirstlane(u);
    if ((int64_t)u >= nunits) break;  // wave-uniform
    // units [0, T): fine; [T, 2T): middle; [2T, 3T): colour
    const int part = (int64_t)u < ntiles ? 1 : (int64_t)u < 2 * ntiles ? 0 : 2;
    const int64_t tile = (int64_t)u - (part == 1 ? 0 : part == 0 ? ntiles : 2 * ntiles);
    // every lane-dependent address (weight fragments, vector tiles) is loop-invariant: laundered per unit,
    // so none of their loads is hoisted out of the loop to pin registers for all of it
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const int64_t idx = tile * 32 + (lane & 31);
    const Pt q = load_point(a, idx);
    if (part == 1) {
      fwd_part_fine<STAGE>(a, q, tile, idx, lane, vsec[1]);
    } else if (part == 0) {
      fwd_part_middle(a, q, tile, idx, lane, occ_mid, vsec[0]);
    } else if (NP == 3) {
      fwd_part_color<TAPE>(a, q, tile, idx, lane, vsec[NP - 1]);
    }
  }
  TL(0, 1, 0);
}

// Decoder-parallel forward, one wave per workgroup: unit u = blockIdx is one decoder of one 32-point
// tile — [0, T) fine (two gathers, 20 GEMMs: the heaviest, dispatched first), [T, 2T) middle, [2T, 3T)
// colour — with the same per-decoder code and outputs as k_query_fwd_parts.  With one-wave workgroups
// the dispatcher refills every wave slot the moment its wave exits, so the launch balances itself over
// the SIMDs (k_query_fwd_parts' 4-wave workgroups of middle-then-colour waves left the SIMDs that drew
// two of them running ~25 us after the others: tools/probes/wave_timeline.py, profiles/r05_*).
template <int STAGE, bool TAPE>
#ifndef NSLAM_UNITS_ORDER
#define NSLAM_UNITS_ORDER 0  // dispatch order of the colour stage's units: 0 fine, middle, colour; 1 fine, colour, middle
#endif
#ifndef NSLAM_UNITS_LB
#define NSLAM_UNITS_LB 3  // waves per SIMD the units kernel's register budget allows (4: <= 128 VGPRs)
#endif
__global__ __launch_bounds__(64, NSLAM_UNITS_LB) void k_query_fwd_units(QueryKArgs a, float* __restrict__ occ_mid) {
  const int64_t ntiles = (a.n + 31) / 32;
  const int64_t u = blockIdx.x;
  const int j = u < ntiles ? 0 : u < 2 * ntiles ? 1 : 2;  // dispatch slot
  const int part = j == 0 ? 1 : (NSLAM_UNITS_ORDER == 1 && STAGE == NSLAM_STAGE_COLOR) ? (j == 1 ? 2 : 0) : (j == 1 ? 0 : 2);
  const int64_t tile = u - j * ntiles;
  TL(0, 0, part);
  // this unit's decoder vector section (biases, output rows, Fourier B), read by every layer
  __shared__ __attribute__((aligned(16))) float vsec[kVecFloats];
  {
    const int d = part == 0 ? NSLAM_DEC_MIDDLE : part == 1 ? NSLAM_DEC_FINE : NSLAM_DEC_COLOR;
    const float* src = a.c.packed[d] + XyzPack{d == NSLAM_DEC_FINE ? 2 : 1}.V();
    for (int i = threadIdx.x; i < 740; i += 64) vsec[i] = src[i];
    __syncthreads();
  }
  const int lane = threadIdx.x;
  const int64_t idx = tile * 32 + (lane & 31);
  const Pt q = load_point(a, idx);
  if (part == 1) {
    fwd_part_fine<STAGE>(a, q, tile, idx, lane, vsec);
  } else if (part == 0) {
    fwd_part_middle(a, q, tile, idx, lane, occ_mid, vsec);
  } else if (STAGE == NSLAM_STAGE_COLOR) {
    fwd_part_color<TAPE>(a, q, tile, idx, lane, vsec);
  }
  TL(0, 1, 0);
}

// ------------------------------------------------------------------------------------------
// Producer / consumer forward (round 5): the decoder-tile units of k_query_fwd_units, but each unit's
// work split between two kinds of wave of one persistent workgroup per CU, so every SIMD holds both at
// once and its MFMA pipe (consumers) and VALU / memory pipes (producers) run side by side:
//   producer waves (4, one per SIMD): the unit's points, trilinear gathers (gather_pair / gather_tile)
//     and Fourier embedding sin(x B_b) — exactly the units kernel's arithmetic — into an LDS slot, in
//     the register layout (16 floats per lane per tile: one conflict-free ds_write_b128 per quad);
//   consumer waves (8, two per SIMD): read a full slot into registers (3 embedding tiles + NC feature
//     tiles), hand the slot back at once, then run the decoder's GEMM chain (xyz_forward_pf_e: the same
//     products in the same order), masks, activation tape and outputs.
// Slots form a ring of kPcSlots: position k (the CU's k-th unit) lives in slot k % kPcSlots; its
// producer waits until position k - kPcSlots was read (pc_free), fills the slot and publishes k
// (pc_full); its consumer waits for k, reads, releases.  Producers and consumers take positions from
// two LDS counters in order, so the CU's waves balance among themselves; CU g owns the global units
// g, g + G, g + 2G, ... (fine units first: the heaviest).  Every wave leaves when the counter passes
// the CU's unit count, and every position below it is produced and consumed exactly once, so the
// grid drains.  Flags are LDS words written after an explicit lgkmcnt(0) (the slot's data is in LDS
// before the flag is) and polled with s_sleep.
#ifndef NSLAM_PC_CONS
#define NSLAM_PC_CONS 8  // consumer waves per workgroup (2 per SIMD)
#endif
constexpr int kPcCons = NSLAM_PC_CONS, kPcProd = 4, kPcWaves = kPcCons + kPcProd;
#ifndef NSLAM_PC_NB
#define NSLAM_PC_NB 8  // corners whose row loads the producer issues together
#endif
#ifndef NSLAM_PC_FD
#define NSLAM_PC_FD 1  // weight fragments the consumers keep in flight
#endif
constexpr int kPcSlots = 7;
constexpr int kPcTileF = 1024;                   // one register tile: 16 floats x 64 lanes
constexpr int kPcSlotF = 5 * kPcTileF + 4;       // emb 0-2, features 3-4, header {unit, inside lo, hi}
static_assert((kPcSlotF * 4) % 16 == 0, "slots stay 16-B aligned");

__device__ __forceinline__ void pc_put(float* __restrict__ t, const f32x16& v, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    *reinterpret_cast<f32x4*>(t + i * 256 + lane * 4) = f32x4{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
}
__device__ __forceinline__ f32x16 pc_get(const float* __restrict__ t, int lane) {
  f32x16 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x4 q = *reinterpret_cast<const f32x4*>(t + i * 256 + lane * 4);
    v[4 * i] = q[0];
    v[4 * i + 1] = q[1];
    v[4 * i + 2] = q[2];
    v[4 * i + 3] = q[3];
  }
  return v;
}
// LDS flag words (workgroup-visible): a store after every earlier LDS access of this wave has completed;
// a poll whose value orders every later LDS access of this wave after it
__device__ __forceinline__ void pc_flag_store(int* p, int v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// (bounded: a wait that never ends — a broken invariant; one unit's hand-over takes microseconds — traps
// after ~2^24 polls (~0.5 s) instead of letting the wave go on with a slot it does not own: the launch
// fails loudly, the caller's next HIP call reports the error, and nothing is silently corrupted)
__device__ __forceinline__ void pc_flag_wait(const int* p, int v) {
  [[maybe_unused]] const unsigned long long t0 = TL_NOW();
  for (int it = 0;; ++it) {
    const int x = __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    if (x == v) break;
    if (it == (1 << 24)) __builtin_trap();
    __builtin_amdgcn_s_sleep(1);
  }
  TL_ADD(0, TL_NOW() - t0);  // (timeline build: the wave's waiting time)
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ int pc_take(int* ctr, int lane) {
  int k = 0;
  if (lane == 0) k = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return __builtin_amdgcn_readfirstlane(k);
}

// The producer's share of unit (part, tile) into slot sl: features (part 1: fine and middle), the
// embedding of the part's decoder and the inside ballot — the units kernel's arithmetic
template <int STAGE>
__device__ __forceinline__ void pc_produce(const QueryKArgs& a, int part, int64_t tile, int64_t unit, int lane,
                                           const float* vs, float* __restrict__ sl, int* full, int* freed, int k,
                                           int s) {
  const int64_t idx = tile * 32 + (lane & 31);
  const Pt q = load_point(a, idx);
  // the grids by opaque indices: their constants (extents, scales; float64) are formed per unit —
  // hoisted out of the producer loop they would pin (and spill) registers for all of it
  int gi = part == 1 ? NSLAM_DEC_FINE : part == 0 ? NSLAM_DEC_MIDDLE : NSLAM_DEC_COLOR, gm = NSLAM_DEC_MIDDLE;
  asm volatile("" : "+s"(gi), "+s"(gm));
  // the slot first (position k - kPcSlots has been read out of it); then every tile is stored as soon as
  // it is formed — the features, then the embedding blocks one at a time — so at most one tile and the
  // loads of one gather are in registers
  pc_flag_wait(freed + s, k - kPcSlots);
  [[maybe_unused]] const unsigned long long tg0 = TL_NOW();
  pc_put(sl + 3 * kPcTileF, gather_nb<NSLAM_PC_NB>(a.c.grid[gi], q, lane), lane);
  if (part == 1) {
    __builtin_amdgcn_sched_barrier(0);
    pc_put(sl + 4 * kPcTileF, gather_nb<NSLAM_PC_NB>(a.c.grid[gm], q, lane), lane);
  }
  TL_ADD1(0, TL_NOW() - tg0);  // (timeline build: the producer's gather time)
  const uint64_t in = __ballot(q.inside);
  const float* B = vs + (XyzPack{1}.FB() - XyzPack{1}.V());  // (the same offset for NC = 2)
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    __builtin_amdgcn_sched_barrier(0);
    pc_put(sl + b * kPcTileF, emb_tile<false, false>(B, q.x, b, lane), lane);
  }
  if (lane == 0) {
    int* hd = reinterpret_cast<int*>(sl + 5 * kPcTileF);
    hd[0] = (int)unit;
    hd[1] = (int)(uint32_t)in;
    hd[2] = (int)(uint32_t)(in >> 32);
  }
  pc_flag_store(full + s, k);
}

template <int STAGE, bool TAPE>
__global__ __launch_bounds__(64 * kPcWaves, 1) void k_query_fwd_pc(QueryKArgs a, float* __restrict__ occ_mid) {
  constexpr int NP = STAGE == NSLAM_STAGE_COLOR ? 3 : 2;
  __shared__ __attribute__((aligned(16))) float vsec[3][kVecFloats];
  __shared__ __attribute__((aligned(16))) float slots[kPcSlots * kPcSlotF];
  __shared__ int full[kPcSlots], freed[kPcSlots], ctr[2];
  {
    const float* s0 = a.c.packed[NSLAM_DEC_MIDDLE] + XyzPack{1}.V();
    const float* s1 = a.c.packed[NSLAM_DEC_FINE] + XyzPack{2}.V();
    const float* s2 = NP == 3 ? a.c.packed[NSLAM_DEC_COLOR] + XyzPack{1}.V() : nullptr;
    for (int i = threadIdx.x; i < 740; i += 64 * kPcWaves) {
      vsec[0][i] = s0[i];
      vsec[1][i] = s1[i];
      if (NP == 3) vsec[2][i] = s2[i];
    }
    if (threadIdx.x < kPcSlots) {
      full[threadIdx.x] = -1;
      freed[threadIdx.x] = (int)threadIdx.x - kPcSlots;
    }
    if (threadIdx.x < 2) ctr[threadIdx.x] = 0;
    __syncthreads();
  }
  const int64_t ntiles = (a.n + 31) / 32;
  const int64_t U = ntiles * NP, G = gridDim.x, g = blockIdx.x;
  const int K = (int)((U - g + G - 1) / G);  // this CU's units (the launch has G <= U)
  const int w = wave_id(), lane0 = threadIdx.x & 63;
  TL(0, 0, w >= kPcCons);
  if (w >= kPcCons) {  // producer
    for (;;) {
      const int k = pc_take(&ctr[0], lane0);
      if (k >= K) break;  // wave-uniform
      // lane-derived addresses re-formed per unit (no hoisting)
      int lane = lane0;
      asm volatile("" : "+v"(lane));
      const int64_t u = g + (int64_t)k * G;
      const int part = u < ntiles ? 1 : u < 2 * ntiles ? 0 : 2;
      const int64_t tile = u - (part == 1 ? 0 : part == 0 ? ntiles : 2 * ntiles);
      const int s = k % kPcSlots;
      pc_produce<STAGE>(a, part, tile, u, lane, vsec[part == 0 ? 0 : part == 1 ? 1 : 2], slots + s * kPcSlotF,
                        full, freed, k, s);
    }
  } else {  // consumer
    for (;;) {
      const int k = pc_take(&ctr[1], lane0);
      if (k >= K) break;  // wave-uniform
      int lane = lane0;
      asm volatile("" : "+v"(lane));
      const int s = k % kPcSlots;
      const float* sl = slots + s * kPcSlotF;
      pc_flag_wait(full + s, k);
      const int* hd = reinterpret_cast<const int*>(sl + 5 * kPcTileF);
      const int64_t u = __builtin_amdgcn_readfirstlane(hd[0]);
      const uint32_t inw = (uint32_t)hd[1 + (lane >> 5)];
      const bool inside = (inw >> (lane & 31)) & 1u;
      const int part = u < ntiles ? 1 : u < 2 * ntiles ? 0 : 2;
      const int64_t tile = u - (part == 1 ? 0 : part == 0 ? ntiles : 2 * ntiles);
      const int64_t idx = tile * 32 + (lane & 31);
      const bool valid = idx < a.n;
      const int h = lane >> 5;
      // the embedding tiles are read where the chain uses them (one at a time in registers); the slot is
      // handed back once the last one is in registers (the features are read into registers first)
      const auto E = [&](int b) {
        const f32x16 v = pc_get(sl + b * kPcTileF, lane);
        if (b == 2) pc_flag_store(freed + s, k);
        return v;
      };
      uint32_t m[5];
      if (part == 1) {
        const f32x16 cf[2] = {pc_get(sl + 3 * kPcTileF, lane), pc_get(sl + 4 * kPcTileF, lane)};
        const XyzPack L{2};
        const float* vs = vsec[1];
        const f32x16 h4 = xyz_forward_pf_e<2, false, 5, NSLAM_PC_FD>(a.c.packed[NSLAM_DEC_FINE], cf, E, lane, m, nullptr, vs);
        save_masks(a, NSLAM_DEC_FINE, tile, m, lane);
        float o = out_row(vs + (L.Wo() - L.V()), vs + (L.Bo() - L.V()), 0, h4, lane);
        if (!inside) o = 0.f;
        if (h == 0 && valid) {
          if (STAGE == NSLAM_STAGE_COLOR) {
            a.raw[idx * 4 + 3] = o;
          } else {
            f32x4 v = {0.f, 0.f, 0.f, o};
            *reinterpret_cast<f32x4*>(a.raw + idx * 4) = v;
          }
        }
      } else if (part == 0) {
        const f32x16 cm[1] = {pc_get(sl + 3 * kPcTileF, lane)};
        const XyzPack L{1};
        const float* vs = vsec[0];
        const f32x16 h4 = xyz_forward_pf_e<1, false, 5, NSLAM_PC_FD>(a.c.packed[NSLAM_DEC_MIDDLE], cm, E, lane, m, nullptr, vs);
        save_masks(a, NSLAM_DEC_MIDDLE, tile, m, lane);
        float o = out_row(vs + (L.Wo() - L.V()), vs + (L.Bo() - L.V()), 0, h4, lane);
        if (!inside) o = 100.f;
        if (h == 0 && valid) occ_mid[idx] = o;
      } else if (STAGE == NSLAM_STAGE_COLOR) {
        const f32x16 cc[1] = {pc_get(sl + 3 * kPcTileF, lane)};
        const XyzPack L{1};
        const float* vs = vsec[2];
        float* tp = TAPE ? a.c.act_tape + tile * kTapeFloats : nullptr;
        const f32x16 h4 = xyz_forward_pf_e<1, TAPE, 12, NSLAM_PC_FD>(a.c.packed[NSLAM_DEC_COLOR], cc, E, lane, m, tp, vs);
        save_masks(a, NSLAM_DEC_COLOR, tile, m, lane);
        float o[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) o[j] = out_row(vs + (L.Wo() - L.V()), vs + (L.Bo() - L.V()), j, h4, lane);
        if (h == 0 && valid) {
#pragma unroll
          for (int j = 0; j < 3; ++j) a.raw[idx * 4 + j] = o[j];
        }
      }
    }
  }
  TL(0, 1, 0);
}

static __global__ __launch_bounds__(256) void k_occ_combine(float* __restrict__ raw, const float* __restrict__ occ_mid,
                                                     int64_t n) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p < n) raw[p * 4 + 3] = raw[p * 4 + 3] + occ_mid[p];
}

// One backward launch per decoder: the decoder's forward is recomputed, its grid gradient is
// scattered, its parameter gradients are accumulated and its share of d/dpts is added into g_pts
// (launches on one stream are ordered and each point is owned by one lane pair: plain
// read-modify-write, no atomics).  With parameter gradients every wave owns a slab of the
// workspace (WG == 1: one tile per wave, slab = tile; WG == 2: a fixed number of waves walk the
// tiles over pre-zeroed slabs) and k_slab_reduce sums the slabs in a fixed order
// (deterministic).  LDS holds only each wave's transpose scratch: LDS float atomics
// (ds_add_f32, one RMW per lane) were the bottleneck of the previous shared-accumulator design.
constexpr int kScratchFloats = 2 * TILE_FLOATS + 32 * 4 + 32 * 3 + 32 * 8 * 2 + 32;
constexpr int kWavesBwd = 4;
constexpr int kMaxSlabs = 4096;  // WG == 2 above this many tiles

// lean mapping tile (saved masks, no weight or point gradients): dc transposed, walk without LDS image
constexpr bool lean_tr(int WG, bool PG, bool SAVED) { return SAVED && WG == 0 && !PG; }
// per-wave LDS floats of a backward kernel variant
// per-wave LDS floats of a backward kernel variant
constexpr int bwd_scratch_floats(int WG, bool PG, bool SAVED) {
  return WG ? kScratchFloats : lean_tr(WG, PG, SAVED) ? kWalkFloats : TILE_FLOATS + kWalkFloats;
}

template <int DEC, int WG, bool PG, bool FIRST, bool SAVED>
__device__ __forceinline__ void dec_bwd_tile(const QueryKArgs& a, int64_t tile, const Slab& A, const Scratch& S,
                                             int lane, double* __restrict__ gpts, int64_t gbase = 0) {
  // gpts: d/dpts of point idx at gpts[(idx - gbase) * 3 + k] (gbase: a tile's LDS staging rows)
  // Every scratch / slab address is a function of the lane only, i.e. invariant across the tile
  // loop; letting LICM hoist the ~300 of them pins (and spills) the register file.  Re-derive
  // them per tile.
  asm volatile("" : "+v"(lane));
  PHASE(DEC, 0);
  const int h = lane >> 5, p = lane & 31;
  const int64_t idx = tile * 32 + p;
  const Pt q = load_point(a, idx);
  float g[4] = {0.f, 0.f, 0.f, 0.f};
  if (q.valid) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(a.g_raw + idx * 4);
    g[0] = v[0];
    g[1] = v[1];
    g[2] = v[2];
    g[3] = q.inside ? v[3] : 0.f;  // ret[~mask,3]=100 blocks the occupancy gradient
  }
  if (WG) {
    if (h == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) S.gtab[p * 4 + j] = g[j];
#pragma unroll
      for (int j = 0; j < 3; ++j) S.xtab[p * 3 + j] = q.x[j];
    }
    lds_sync();
  }
  const nslam_grid& gr = a.c.grid[DEC];
  const nslam_dec_grad& dg = a.c.dgrad[DEC];
  const float* pk = a.c.packed[DEC];
  // the colour decoder's h4 cotangent of a direct MLP(color=True) caller (ABI v17), none for tail lanes
  const float* gh4 = (DEC == NSLAM_DEC_COLOR && a.c.g_h4 && q.valid) ? a.c.g_h4 + idx * 32 : nullptr;
  // The weight fragments are loop-invariant across the tile loop; hoisting their ~100 loads out of
  // the loop would pin hundreds of registers.  Launder the base pointer per tile so they stay put.
  asm volatile("" : "+s"(pk));
  PHASE(DEC, 1);
  Corners cr;
  grid_corners(cr, gr, q);
  ScatterCorners scn{};
  if (WG == 0 && gr.grad) scn = resolve_corners(gr.slot, cr, q.valid, lane);
  PHASE(DEC, 2);
  f32x16 dc;
  float gx[3] = {0.f, 0.f, 0.f};
  static_assert(!(SAVED && WG), "weight gradients from saved masks run as k_color_wgrad");
  // the lean mapping chain forms dc transposed for the register-only scatter walk (lean_tr)
  constexpr bool TR = lean_tr(WG, PG, SAVED);
  float* const tab = TR ? S.sA : S.sA + TILE_FLOATS;  // the walk table (after the transpose image if any)
  // d/dpts mask-only tiles (not the coarse decoder's: its chain keeps dc in registers): dc waits in the
  // scatter image while the Fourier backward runs
  constexpr bool IMGDC = SAVED && WG == 0 && PG && DEC != NSLAM_DEC_COARSE;
  float* const img = IMGDC ? S.sA : nullptr;
  if (SAVED) {  // masks from the forward: no recompute (the mask-only chain)
    uint32_t m[5];
    load_masks(a, DEC, tile, m, lane);
    // the walk table goes to LDS before the chain (its corner rows and weights need no registers
    // through it); the slot loads were issued before the masks, so this waits for nothing extra
    if (WG == 0 && gr.grad) stage_walk_table(tab, scn, cr.cell, lane);
    if (DEC == NSLAM_DEC_COARSE) {
      noxyz_backward_saved<TR>(pk, m, g[3], lane, dc);
    } else if (DEC == NSLAM_DEC_FINE) {
      xyz_backward_saved<2, 1, 3, PG, TR>(pk, m, q.x, g, lane, dc, gx, nullptr, img);
    } else if (DEC == NSLAM_DEC_COLOR) {
      xyz_backward_saved<1, 3, 0, PG, TR>(pk, m, q.x, g, lane, dc, gx, gh4, img);
    } else {
      xyz_backward_saved<1, 1, 3, PG, TR>(pk, m, q.x, g, lane, dc, gx, nullptr, img);
    }
  } else if (DEC == NSLAM_DEC_COARSE) {
    const f32x16 c = gather_tile(gr.data, cr, lane);
    noxyz_backward<WG>(pk, c, g[3], dg, A, S, lane, dc);
  } else if (DEC == NSLAM_DEC_FINE) {
    Corners cm;
    grid_corners(cm, a.c.grid[NSLAM_DEC_MIDDLE], q);
    // the middle feature enters the fine decoder under torch.no_grad (decoder.py:184-187)
    const f32x16 cf[2] = {gather_tile(gr.data, cr, lane), gather_tile(a.c.grid[NSLAM_DEC_MIDDLE].data, cm, lane)};
    xyz_backward<2, 1, 3, WG, PG || WG>(pk, cf, q.x, g, dg, A, S, lane, dc, gx);
  } else {
    const f32x16 c[1] = {gather_tile(gr.data, cr, lane)};
    PHASE(DEC, 3);
    if (DEC == NSLAM_DEC_COLOR)  // the colour decoder's 4th output is overwritten by the combiner
      xyz_backward<1, 3, 0, WG, PG || WG>(pk, c, q.x, g, dg, A, S, lane, dc, gx, gh4);
    else
      xyz_backward<1, 1, 3, WG, PG || WG>(pk, c, q.x, g, dg, A, S, lane, dc, gx);
  }
  PHASE(DEC, 12);
  if (gr.grad) {
    if (WG) {
      scatter_grid_grad_halves(gr.grad, gr.slot, cr, dc, q.valid, S, lane);
    } else {  // walk table: the lean kernels' slot after the transpose image
      scatter_grid_grad_uniform<SAVED, TR, IMGDC>(gr.grad, scn, cr.cell, dc, S.sA, tab, lane);
    }
  }
  PHASE(DEC, 13);
  if (PG) {
    double gp[3] = {(double)gx[0], (double)gx[1], (double)gx[2]};
    if (SAVED && WG == 0) {
      // the corners again (the same arithmetic, so the same values) instead of 27 registers held across
      // the chain; the laundered coordinates keep the compiler from merging the two computations
      Pt q2 = q;
#pragma unroll
      for (int k = 0; k < 3; ++k) asm volatile("" : "+v"(q2.p[k]));
      grid_corners(cr, gr, q2);
    }
    if (IMGDC) {
      lds_sync();  // (the scatter read the image; the reads below are this wave's own stores)
      dc = tload(S.sA, lane);
    }
    coord_grad(gr, cr, dc, lane, gp);
    if (h == 0 && q.valid) {
#pragma unroll
      for (int k = 0; k < 3; ++k)
        gpts[(idx - gbase) * 3 + k] = FIRST ? gp[k] : gpts[(idx - gbase) * 3 + k] + gp[k];
    }
  }
  PHASE(DEC, 14);
}

#ifndef NSLAM_LEAN_LB
#define NSLAM_LEAN_LB 2  // min waves per SIMD of the mask-only kernels (experiments: 3..5)
#endif
template <int DEC, int WG, bool PG, bool FIRST, bool SAVED>
__global__ __launch_bounds__(64 * kWavesBwd, (WG || PG || !SAVED) ? 2 : NSLAM_LEAN_LB) void k_dec_bwd(QueryKArgs a, float* __restrict__ slab,
                                                                 int acc_floats) {
  // per-wave scratch: the scatter needs sA + corner rows/weights; weight gradients add sX and
  // the per-point tables (sizing LDS per variant keeps the lean kernels at 5+ waves/SIMD)
  // (the lean kernels' scatter walk needs only the sA transpose image and its walk table)
  constexpr int kScr = bwd_scratch_floats(WG, PG, SAVED);
  __shared__ __attribute__((aligned(16))) float lds[kWavesBwd * kScr];
  const int lane = threadIdx.x & 63, wave = wave_id();
  float* sc = lds + wave * kScr;
  Scratch S;
  S.sA = sc;
  if (WG) {
    S.sX = sc + TILE_FLOATS;
    S.gtab = sc + 2 * TILE_FLOATS;
    S.xtab = S.gtab + 32 * 4;
    S.crow = reinterpret_cast<int*>(S.xtab + 32 * 3);
    S.cw = reinterpret_cast<float*>(S.crow + 32 * 8);
    S.ccell = reinterpret_cast<int*>(S.cw + 32 * 8);
  } else {
    S.sX = S.gtab = S.xtab = S.cw = nullptr;
    S.crow = S.ccell = nullptr;
  }
  const int64_t ntiles = (a.n + 31) / 32;
  const int64_t w = (int64_t)blockIdx.x * kWavesBwd + wave;
  const Slab A = make_slab(WG ? slab + (size_t)w * acc_floats : slab, WG ? acc_floats : 0);
  if (WG == 0) {  // one tile per wave (grid covers all tiles)
    if (w < ntiles) dec_bwd_tile<DEC, WG, PG, FIRST, SAVED>(a, w, A, S, lane, a.g_pts);
    return;
  }
  if (WG == 1) {  // one tile per wave, then the workgroup folds its waves' slabs into its first one
    if (w < ntiles) dec_bwd_tile<DEC, WG, PG, FIRST, SAVED>(a, w, A, S, lane, a.g_pts);
    // the slabs were just written by this CU (L2-resident): summing them here in wave order (a
    // fixed order: deterministic) leaves k_slab_reduce a quarter of the bytes to read
    __syncthreads();
    const int64_t w0 = (int64_t)blockIdx.x * kWavesBwd;
    const int nv = (int)(ntiles - w0 < kWavesBwd ? ntiles - w0 : kWavesBwd);
    f32x4* s0 = reinterpret_cast<f32x4*>(slab + (size_t)w0 * acc_floats);
    const int q = acc_floats / 4;
    for (int i = threadIdx.x; i < q; i += blockDim.x) {
      f32x4 t = s0[i];
      for (int v = 1; v < nv; ++v) t += s0[(size_t)v * q + i];
      s0[i] = t;
    }
    return;
  }
#pragma nounroll
  for (int64_t tile = w; tile < ntiles; tile += (int64_t)gridDim.x * kWavesBwd)
    dec_bwd_tile<DEC, WG, PG, FIRST, SAVED>(a, tile, A, S, lane, a.g_pts);
}

// Mask-only backward of several decoders in ONE launch (ABI v10 nslam_query_bwd_decoders): the
// decoders' workgroups are interleaved over blockIdx (part = blockIdx % ndec), so frozen decoders
// that would otherwise run as concurrent launches on separate streams (tracking: middle, fine and
// colour; mapping: middle and fine) need no fork / join between streams.  Each part writes its own
// d/dpts buffer gp[part] (no cross-decoder accumulation, no atomics on points).
struct MultiDecArgs {
  int ndec;
  int dec[4];
  double* gp[4];
};
// (a colour decoder with weight gradients runs here as its lean chain too: grid gradient, d/dpts;
// its parameter gradients come from k_color_wgrad, nslam_color_wgrad.hip)
// Register bound of the mapping (no d/dpts) variant: 4 waves/SIMD -> 106 VGPRs (the walk table staged
// before the chain frees its corner registers).  A/B on one box, 3 alternating rounds (r4t): 0.2287 ms
// per iteration at the old 2-wave bound (115 VGPRs), 0.2208 ms at 4, 0.2260 ms at 5 (96 VGPRs: one
// resident round for room0's 4500 waves, but the standalone launch only 1 % shorter than at 4).
#ifndef NSLAM_MULTI_LB
#define NSLAM_MULTI_LB 4
#endif
#ifndef NSLAM_MULTI_PG_LB
#define NSLAM_MULTI_PG_LB 3  // the d/dpts (tracking, bundle adjustment) variant: 163 VGPRs with dc in the
                             // scatter image through the Fourier backward (218 before: 2 waves/SIMD)
#endif
template <bool PG>
__global__ __launch_bounds__(64 * kWavesBwd, PG ? NSLAM_MULTI_PG_LB : NSLAM_MULTI_LB) void k_dec_bwd_multi(QueryKArgs a, MultiDecArgs m) {
  constexpr int kScr = bwd_scratch_floats(0, PG, true);
  __shared__ __attribute__((aligned(16))) float lds[kWavesBwd * kScr];
  const int lane = threadIdx.x & 63, wave = wave_id();
  Scratch S;
  S.sA = lds + wave * kScr;
  S.sX = S.gtab = S.xtab = S.cw = nullptr;
  S.crow = S.ccell = nullptr;
  const int part = (int)(blockIdx.x % (unsigned)m.ndec);
  // selects, not a dynamic index into the by-value argument (that would copy it to scratch)
  const int dec = part == 0 ? m.dec[0] : part == 1 ? m.dec[1] : part == 2 ? m.dec[2] : m.dec[3];
  double* gp = part == 0 ? m.gp[0] : part == 1 ? m.gp[1] : part == 2 ? m.gp[2] : m.gp[3];
  const int64_t w = (int64_t)(blockIdx.x / (unsigned)m.ndec) * kWavesBwd + wave;
  const int64_t ntiles = (a.n + 31) / 32;
  if (w >= ntiles) return;
  TL(1, 0, part);
  const Slab A = make_slab(nullptr, 0);
  switch (dec) {
    case NSLAM_DEC_COARSE: dec_bwd_tile<NSLAM_DEC_COARSE, 0, PG, true, true>(a, w, A, S, lane, gp); break;
    case NSLAM_DEC_MIDDLE: dec_bwd_tile<NSLAM_DEC_MIDDLE, 0, PG, true, true>(a, w, A, S, lane, gp); break;
    case NSLAM_DEC_FINE: dec_bwd_tile<NSLAM_DEC_FINE, 0, PG, true, true>(a, w, A, S, lane, gp); break;
    default: dec_bwd_tile<NSLAM_DEC_COLOR, 0, PG, true, true>(a, w, A, S, lane, gp); break;
  }
  TL(1, 1, 0);
}

// base[j] += sum_b slab[b][j].  A workgroup owns 64 parameters; lane (r, c) of a wave reads the
// float4 c of slab r of every 64th slab group, so the 16 waves x 4 lane rows keep 64 slab streams
// in flight per workgroup (~count/64 workgroups fill the chip; a wave load is 4 x 256-B
// segments).  The 64 partials are combined in LDS in a fixed order: deterministic.
constexpr int kReduceWaves = 16;
static __global__ __launch_bounds__(64 * kReduceWaves) void k_slab_reduce(const float* __restrict__ slab, int64_t nslab,
                                                                   int acc_floats, int count,
                                                                   float* __restrict__ base) {
  __shared__ f32x4 part[kReduceWaves * 4][16];
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int c = lane & 15, r = wave * 4 + (lane >> 4);  // r: slab stream 0..63
  const int j = (blockIdx.x * 16 + c) * 4;
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
  if (j < count) {
    const float* p = slab + j;
    int64_t b = r;
    for (; b + 64 < nslab; b += 128) {
      s0 += *reinterpret_cast<const f32x4*>(p + b * acc_floats);
      s1 += *reinterpret_cast<const f32x4*>(p + (b + 64) * acc_floats);
    }
    if (b < nslab) s0 += *reinterpret_cast<const f32x4*>(p + b * acc_floats);
  }
  part[r][c] = s0 + s1;
  __syncthreads();
  if (threadIdx.x < 16 && j < count) {
    f32x4 t = part[0][c];
#pragma unroll 8
    for (int k = 1; k < kReduceWaves * 4; ++k) t += part[k][c];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (j + e < count) base[j + e] += t[e];
  }
}

inline bool grid_ok(const nslam_grid& g) {
  // every axis <= 1024: the scatter packs a cell's coordinates into 10 bits each (Corners::cell)
  return g.data && g.dims[0] > 0 && g.dims[1] > 0 && g.dims[2] > 0 && g.dims[0] <= 1024 && g.dims[1] <= 1024 &&
         g.dims[2] <= 1024 && (((uintptr_t)g.data) & 15) == 0;
}

inline int check_cfg(const nslam_query_cfg* c, bool bwd) {
  if (!c || c->stage < 0 || c->stage > 3) return NSLAM_EINVAL;
  const int st = c->stage;
  bool need[4] = {st == NSLAM_STAGE_COARSE, st != NSLAM_STAGE_COARSE, st >= NSLAM_STAGE_FINE,
                  st == NSLAM_STAGE_COLOR};
  for (int d = 0; d < 4; ++d) {
    if (!need[d]) continue;
    if (!grid_ok(c->grid[d]) || !c->packed[d]) return NSLAM_EINVAL;
    if ((((uintptr_t)c->packed[d]) & 15) != 0) return NSLAM_EINVAL;
  }
  if (c->rays_o) {
    if (!c->rays_d || !c->z_vals || c->n_samples <= 0) return NSLAM_EINVAL;
  }
  // the h4 cotangent is read as float4 rows (add_gh4, k_color_wgrad): 16-byte aligned
  if (c->g_h4 && (((uintptr_t)c->g_h4) & 15) != 0) return NSLAM_EINVAL;
  return NSLAM_OK;
}

inline int hip_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? NSLAM_OK : NSLAM_EHIP - (int)e;
}


inline int acc_floats_of(const nslam_dec_grad& dg) { return (int)((dg.count + 3) & ~int64_t(3)); }

// ---- the colour decoder's weight gradients (k_color_wgrad, nslam_color_wgrad.hip) ----------------
// With the forward's activation tape and ReLU masks, the colour decoder's backward is two launches that
// need not wait for each other: the lean mask-only chain (grid gradient, d/dpts) and k_color_wgrad, a
// split-K reduction over tile chunks of every weight block (one 8-wave workgroup per chunk; each
// chunk's partial sums fill one slab), then k_slab_reduce over the chunks.  Workspace: the chunk slabs.
#ifndef NSLAM_CW_CHUNKS
#define NSLAM_CW_CHUNKS 256
#endif
constexpr int kCwTargetChunks = NSLAM_CW_CHUNKS;  // one workgroup per CU
struct CwPlan {
  int64_t chunk_tiles;
  int nchunks;
  size_t slab_bytes;
};
inline CwPlan cw_plan(const nslam_dec_grad& dg, int64_t n_pts) {
  CwPlan p;
  const int64_t tiles = (n_pts + 31) / 32;
  p.chunk_tiles = (tiles + kCwTargetChunks - 1) / kCwTargetChunks;
  p.nchunks = (int)((tiles + p.chunk_tiles - 1) / p.chunk_tiles);
  p.slab_bytes = (size_t)p.nchunks * acc_floats_of(dg) * sizeof(float);
  return p;
}
inline bool cw_tape_path(const nslam_query_cfg* c) { return c->act_tape != nullptr && c->saved_masks != nullptr; }
// k_color_wgrad + k_slab_reduce into a.c.dgrad[COLOR] (a.g_raw: the cotangent; ws: the chunk slabs)
int launch_color_wgrad(const QueryKArgs& a, float* ws, hipStream_t s);

// Slab cap: kMaxSlabs, or NSLAM_MAX_SLABS from the environment (tests use it to reach the
// multi-tile read-modify-write mode at small sizes).
inline int64_t max_slabs() {
  const char* e = getenv("NSLAM_MAX_SLABS");
  const long v = e ? strtol(e, nullptr, 10) : 0;
  return v > 0 ? v : kMaxSlabs;
}

// parameter-gradient slabs for a decoder: one per tile up to the cap, else one per launched wave
// (the cap rounded up to whole workgroups), each wave walking tiles with grid stride
inline int64_t n_slabs(int64_t tiles) {
  const int64_t cap = max_slabs();
  return tiles <= cap ? tiles : (cap + kWavesBwd - 1) / kWavesBwd * kWavesBwd;
}

template <int DEC, int WG, bool PG, bool FIRST, bool SAVED = false>
int launch_one(const QueryKArgs& a, float* slab, int acc, int64_t blocks, hipStream_t s) {
  hipLaunchKernelGGL((k_dec_bwd<DEC, WG, PG, FIRST, SAVED>), dim3((unsigned)blocks), dim3(64 * kWavesBwd), 0, s, a,
                     slab, acc);
  return hip_status();
}

// WG == 1 launches leave one folded slab per workgroup (stride kWavesBwd slabs); WG == 2 one per wave
inline int slab_reduce(const nslam_dec_grad& dg, float* slab, bool folded, int64_t nslab, int64_t blocks, int acc,
                       hipStream_t s) {
  const int64_t n = folded ? blocks : nslab;
  const int stride = folded ? acc * kWavesBwd : acc;
  const int64_t nblk = (dg.count + 63) / 64;
  hipLaunchKernelGGL(k_slab_reduce, dim3((unsigned)nblk), dim3(64 * kReduceWaves), 0, s, slab, n, stride,
                     (int)dg.count, dg.base);
  return hip_status();
}

template <int DEC, int WG, bool PG>
int launch_dec_bwd(const QueryKArgs& a, bool first, float* slab, hipStream_t s) {
  const int64_t tiles = (a.n + 31) / 32;
  if (WG == 0) {
    const int64_t blocks = (tiles + kWavesBwd - 1) / kWavesBwd;
    if (a.c.saved_masks)
      return first ? launch_one<DEC, 0, PG, true, true>(a, nullptr, 0, blocks, s)
                   : launch_one<DEC, 0, PG, false, true>(a, nullptr, 0, blocks, s);
    return first ? launch_one<DEC, 0, PG, true>(a, nullptr, 0, blocks, s)
                 : launch_one<DEC, 0, PG, false>(a, nullptr, 0, blocks, s);
  }
  const nslam_dec_grad& dg = a.c.dgrad[DEC];
  const int acc = acc_floats_of(dg);
  const int64_t nslab = n_slabs(tiles);
  const int64_t blocks = (nslab + kWavesBwd - 1) / kWavesBwd;
  // the colour decoder's weight gradients from the forward's activation tape when it is there: the
  // lean chain (grid gradient), then k_color_wgrad (which does not read anything the chain wrote)
  constexpr bool kTapeable = DEC == NSLAM_DEC_COLOR && !PG;
  int rc;
  if constexpr (kTapeable) {
    if (cw_tape_path(&a.c)) {
      rc = launch_one<DEC, 0, false, true, true>(a, nullptr, 0, (tiles + kWavesBwd - 1) / kWavesBwd, s);
      return rc ? rc : launch_color_wgrad(a, slab, s);
    }
  }
  if (tiles > max_slabs() && hipMemsetAsync(slab, 0, (size_t)nslab * acc * sizeof(float), s) != hipSuccess)
    return hip_status();
  if (tiles <= max_slabs()) {
    rc = first ? launch_one<DEC, 1, PG, true>(a, slab, acc, blocks, s)
               : launch_one<DEC, 1, PG, false>(a, slab, acc, blocks, s);
  } else {
    rc = first ? launch_one<DEC, 2, PG, true>(a, slab, acc, blocks, s)
               : launch_one<DEC, 2, PG, false>(a, slab, acc, blocks, s);
  }
  if (rc) return rc;
  return slab_reduce(dg, slab, tiles <= max_slabs(), nslab, blocks, acc, s);
}

template <int DEC>
int dispatch_dec_bwd(const QueryKArgs& a, bool first, float* slab, hipStream_t s) {
  const bool wg = a.c.dgrad[DEC].base != nullptr;
  const bool pg = a.c.need_pts_grad != 0;
  if (wg && pg && a.c.saved_masks) {
    // Split instead of the combined kernel (which spills ~100 VGPRs): parameter + grid gradients
    // first, then d/dpts from the saved masks with the grid scatter switched off.
    int rc = launch_dec_bwd<DEC, 1, false>(a, first, slab, s);
    if (rc) return rc;
    QueryKArgs b = a;
    b.c.grid[DEC].grad = nullptr;
    b.c.dgrad[DEC].base = nullptr;
    return launch_dec_bwd<DEC, 0, true>(b, first, nullptr, s);
  }
  if (wg && pg) return launch_dec_bwd<DEC, 1, true>(a, first, slab, s);
  if (wg) return launch_dec_bwd<DEC, 1, false>(a, first, slab, s);
  if (pg) return launch_dec_bwd<DEC, 0, true>(a, first, slab, s);
  return launch_dec_bwd<DEC, 0, false>(a, first, slab, s);
}

inline size_t dec_ws_bytes(const nslam_query_cfg* cfg, int dec, int64_t n_pts) {
  const nslam_dec_grad& dg = cfg->dgrad[dec];
  if (!dg.base || dg.count <= 0) return 0;
  if (dec == NSLAM_DEC_COLOR && cw_tape_path(cfg)) {
    return cw_plan(dg, n_pts).slab_bytes;
  }
  return (size_t)n_slabs((n_pts + 31) / 32) * acc_floats_of(dg) * sizeof(float);
}

inline size_t bwd_ws_bytes(const nslam_query_cfg* cfg, int64_t n_pts) {
  size_t need = 0;
  for (int d = 0; d < 4; ++d) {
    const size_t b = dec_ws_bytes(cfg, d, n_pts);
    need = b > need ? b : need;  // decoders run one after the other on the stream: one region
  }
  return need;
}

inline bool stage_uses(int stage, int dec) {
  switch (stage) {
    case NSLAM_STAGE_COARSE: return dec == NSLAM_DEC_COARSE;
    case NSLAM_STAGE_MIDDLE: return dec == NSLAM_DEC_MIDDLE;
    case NSLAM_STAGE_FINE: return dec == NSLAM_DEC_MIDDLE || dec == NSLAM_DEC_FINE;
    default: return dec != NSLAM_DEC_COARSE;
  }
}


#ifndef NSLAM_QUERY_ONE_TU
extern template int dispatch_dec_bwd<NSLAM_DEC_COARSE>(const QueryKArgs&, bool, float*, hipStream_t);
extern template int dispatch_dec_bwd<NSLAM_DEC_MIDDLE>(const QueryKArgs&, bool, float*, hipStream_t);
extern template int dispatch_dec_bwd<NSLAM_DEC_FINE>(const QueryKArgs&, bool, float*, hipStream_t);
extern template int dispatch_dec_bwd<NSLAM_DEC_COLOR>(const QueryKArgs&, bool, float*, hipStream_t);
#endif

}  // namespace nslamq
