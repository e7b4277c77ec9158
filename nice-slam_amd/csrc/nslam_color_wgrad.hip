// nslam_color_wgrad.hip — the colour decoder's parameter gradients of a mapping iteration
// (Mapper.py:503 reaching color_decoder.parameters(), fix_color False; decoder.py:177-203 backward)
// as a split-K reduction over the points (ABI v16).
//
// Inputs: the forward's activation tape (h0..h4 of every 32-point tile) and ReLU masks, the loss
// cotangent g_raw and the points (ray form or pts).  Everything else is recomputed here, so the
// kernel depends on the forward and the loss only — not on the lean backward chain that scatters the
// colour grid's gradient — and the two run side by side:
//   the cotangent chain  dh4 = Woᵀ g, dh_{i-1} = L_iᵀ mask_i(dh_i)     (4 GEMM tiles per tile)
//   the colour feature   c = trilinear(colour grid)                     (decoder.py:168-175)
//   the embedding        S_b = sin(x B_b)                               (decoder.py:26-30)
//   the Fourier backward de_b = L3_bᵀ da3 + L0_bᵀ da0, formed TRANSPOSED (lane = embedding dim,
//                        registers = points: the MFMA with its operands swapped), so
//                        dB[c][d] = Σ_p x_c de cos(x B) needs no LDS transpose.
// One workgroup (8 waves) owns a chunk of consecutive tiles, software-pipelined over two LDS buffers:
// while waves 0-6 form the weight gradients of tile t from buffer t&1, wave 7 produces tile t+1 into
// the other buffer (cotangent chain, colour feature, masks, x | g table) and waves 0-6 stage its
// activation tape by LDS-DMA.  Every weight block dW = Σ_points (cotangent ⊗ input) is an MFMA chain
// over point-major LDS image streams (element s of lane (j, h) = point 2s + h, column j), accumulated
// in registers over the whole chunk and written once into the chunk's slab; k_slab_reduce sums the
// slabs in a fixed order (deterministic).
//
// Roles ("waves" 0-7; which hardware wave takes which role: the permutation in k_color_wgrad):
//   wave b = 0..2  dW_3[:, 32b..] = Σ da3 ⊗ S_b, dW_0[:, 32b..] = Σ da0 ⊗ S_b (+ db_0, b = 0)
//   wave 3         dW_3[:, 93:125] = Σ da3 ⊗ h2, dW_2 = Σ da2 ⊗ h1 (+ db_3, db_2)
//   wave 4, 5      fc_c.k, fc_c.(k+3) = Σ dh ⊗ c (k = wave - 4), and dB[:, 32k..]
//   wave 6         fc_c.2, dW_4 = Σ da4 ⊗ h3, and dB[:, 64..93]
//   wave 7         the producer of the next tile; dW_1 = Σ da1 ⊗ h0 (+ db_1), dWo = Σ g ⊗ h4 (rows 0-2;
//                  row 3 is replaced by the stage combiner, decoder.py:341), dbo
// Every role holds at most two weight blocks (the compiler keeps every role's loop-carried values live
// in every wave, so the register budget is the union's).
#include "nslam_query_impl.h"

// k_color_wgrad asks for 4 waves per SIMD (launch bounds) to cap itself at 128 VGPRs, so two waves of
// the lean backward fit beside its two on each SIMD; its 95 KiB of LDS keeps it at one workgroup per
// CU, which the compiler reports as a missed occupancy target.
#pragma clang diagnostic ignored "-Wpass-failed"

namespace nslamq {

namespace {

constexpr int kCwWaves = 8;
constexpr int kStagers = kCwWaves - 1;         // waves 0-6 stage the activation tape
constexpr int kImg32 = 1024;                   // activation image [32 points][32] (LDS-DMA, pitch 32)
constexpr int kImg33 = 32 * TPITCH;            // cotangent / colour-feature image (pitch 33)
constexpr int kBA = 0;                         // h0..h4
constexpr int kBD = kBA + 5 * kImg32;          // dh0..dh4
constexpr int kBC = kBD + 5 * kImg33;          // colour feature
constexpr int kBM = kBC + kImg33;              // masks, uint16 [layer 5][64 lanes]
constexpr int kBX = kBM + 5 * 64 / 2;          // [32 points][8]: x (3 + pad), g (3 + pad)
constexpr int kBuf = kBX + 32 * 8;             // floats per buffer
constexpr int kWoOff = 2 * kBuf;               // the output layer's rows 0-2 (both buffers' chains)
constexpr int kActPieces = kTapeFloats / 256;  // 1-KiB LDS-DMA pieces (16 B per lane)
constexpr int kLds = 2 * kBuf + 3 * 32;
static_assert(kTapeFloats % 256 == 0, "the tape is whole 1-KiB pieces");
static_assert(kBD % 4 == 0 && kBC % 4 == 0 && kBM % 4 == 0 && kBX % 4 == 0 && kBuf % 4 == 0, "16-B regions");
static_assert(kLds * 4 <= 100 * 1024, "LDS: leave room for the lean backward's workgroups on the CU");

#ifndef NSLAM_CW_GATHER_NB
#define NSLAM_CW_GATHER_NB 1  // corners in flight of the feature gather (2: 129 VGPRs, one over the 4-wave budget)
#endif
#ifndef NSLAM_CW_PERM
#define NSLAM_CW_PERM 1  // roles permuted over the SIMDs (k_color_wgrad)
#endif
#ifndef NSLAM_CW_LB
#define NSLAM_CW_LB 4  // min waves per SIMD: <= 128 VGPRs, so the lean backward's waves fit beside it
#endif

struct CwArgs {
  QueryKArgs a;
  float* slab;          // [nchunks][acc]
  int acc;              // floats per slab
  int nchunks;
  int64_t chunk_tiles;  // tiles per chunk
};

__device__ __forceinline__ const float* act(const float* buf, int i) { return buf + kBA + i * kImg32; }
__device__ __forceinline__ float* dimg(float* buf, int i) { return buf + kBD + i * kImg33; }
__device__ __forceinline__ const float* dimg(const float* buf, int i) { return buf + kBD + i * kImg33; }
__device__ __forceinline__ const uint16_t* masks(const float* buf) {
  return reinterpret_cast<const uint16_t*>(buf + kBM);
}

// Operand streams of the weight-gradient MFMAs: element s of lane (j, h) belongs to point 2s + h
// (column j).  The images are point-major, so element s of an image of pitch P is one ds_read at
// row 2s + h (the two rows of one read are P floats apart: disjoint banks).
template <int P>
struct Img {
  const float* p;
  __device__ __forceinline__ Img(const float* im, int lane) : p(im + (lane >> 5) * P + (lane & 31)) {}
  __device__ __forceinline__ float operator()(int s) const { return p[2 * P * s]; }
};
// v if bit `bit` of w is set, else +0 (v_bfe_i32 + v_and)
__device__ __forceinline__ float keep(float v, uint32_t w, int bit) {
  return __builtin_bit_cast(float, __builtin_bit_cast(int, v) & __builtin_amdgcn_sbfe((int)w, bit, 1));
}
// da_i: the dh_i image times the ReLU mask.  Feature j of point P is bit r(j) of the saved mask of lane
// (P, h(j)) (the forward's C layout: feature F(r, h) = j).
struct Masked {
  Img<TPITCH> v;
  const uint16_t* ms;
  int rj;
  __device__ __forceinline__ Masked(const float* buf, int i, int lane)
      : v(dimg(buf, i), lane),
        ms(masks(buf) + i * 64 + 32 * (((lane & 31) >> 2) & 1) + (lane >> 5)),
        rj(((lane & 31) & 3) + 4 * ((lane & 31) >> 3)) {}
  __device__ __forceinline__ float operator()(int s) const { return keep(v(s), ms[2 * s], rj); }
};
// S_b = sin(x B_b) (decoder.py:29-30): the embedding column of lane j at point 2s + h, recomputed (the
// forward's fsin of the same fp32 argument: the same value)
struct Emb {
  const float* xg;
  float b0, b1, b2;
  __device__ __forceinline__ Emb(const float* buf, const float Bk[3], int lane)
      : xg(buf + kBX + (lane >> 5) * 8), b0(Bk[0]), b1(Bk[1]), b2(Bk[2]) {}
  __device__ __forceinline__ float operator()(int s) const {
    const f32x4 x4 = *reinterpret_cast<const f32x4*>(xg + 16 * s);
    const float x[3] = {x4[0], x4[1], x4[2]};
    return fsin(fourier_arg(x, b0, b1, b2));
  }
};

// accA += Σ_s A_s ⊗ B_s and accB += Σ_s C_s ⊗ D_s over the tile's points (two independent MFMA chains,
// interleaved); returns the bias sums Σ A, Σ C.  The operands are formed kG elements at a time with a
// scheduling fence between groups, so kG (not 16) elements of each stream are in registers.
constexpr int kG = 4;
template <bool SHARED_BD, class FA, class FB, class FC, class FD>
__device__ __forceinline__ void chain2(f32x16& accA, f32x16& accB, float& biasA, float& biasC, const FA& fa,
                                       const FB& fb, const FC& fc, const FD& fd) {
  float sa = 0.f, sc = 0.f;
#pragma unroll
  for (int s0 = 0; s0 < 16; s0 += kG) {
    float A[kG], B[kG], C[kG], D[kG];
#pragma unroll
    for (int g = 0; g < kG; ++g) {
      A[g] = fa(s0 + g);
      B[g] = fb(s0 + g);
      C[g] = fc(s0 + g);
      D[g] = SHARED_BD ? B[g] : fd(s0 + g);
    }
#pragma unroll
    for (int g = 0; g < kG; ++g) {
      accA = mfma32(A[g], B[g], accA);
      accB = mfma32(C[g], D[g], accB);
      sa += A[g];
      sc += C[g];
    }
    asm volatile("" : "+v"(sa), "+v"(sc));  // the sums here: no operand stays live to a sunk add
    __builtin_amdgcn_sched_barrier(0);
  }
  biasA += sa;
  biasC += sc;
}
template <class FA, class FB>
__device__ __forceinline__ void chain1(f32x16& acc, float& bias, const FA& fa, const FB& fb) {
  float sa = 0.f;
#pragma unroll
  for (int s0 = 0; s0 < 16; s0 += kG) {
    float A[kG], B[kG];
#pragma unroll
    for (int g = 0; g < kG; ++g) {
      A[g] = fa(s0 + g);
      B[g] = fb(s0 + g);
    }
#pragma unroll
    for (int g = 0; g < kG; ++g) {
      acc = mfma32(A[g], B[g], acc);
      sa += A[g];
    }
    asm volatile("" : "+v"(sa));
    __builtin_amdgcn_sched_barrier(0);
  }
  bias += sa;
}

// dW[F(r, h)][kofs + k] of a C-layout accumulator (lane (k, h)), columns k < kvalid
__device__ __forceinline__ void store_block(float* __restrict__ sl, int64_t base, int ldk, int kofs, int kvalid,
                                            const f32x16& acc, int lane) {
  const int h = lane >> 5, k = lane & 31;
  if (k < kvalid) {
    __attribute__((address_space(1))) float* p = as_global_w(sl) + base + 4 * h * ldk + kofs + k;
#pragma unroll
    for (int r = 0; r < 16; ++r) p[((r & 3) + 8 * (r >> 2)) * ldk] = acc[r];
  }
}
// bias: each lane summed column o over its half's points; the halves are added and lane o stores
__device__ __forceinline__ void store_vec(float* __restrict__ sl, int64_t base, float v, int lane) {
  v += xor32(v);
  if (lane < 32) as_global_w(sl)[base + lane] = v;
}

// The activation tape of tile t into buf by LDS-DMA (global_load_lds: the hardware writes lane l's
// 16 B at the wave-uniform LDS address + 16 l), piece q by wave q % 7.
__device__ __forceinline__ void stage_act(const QueryKArgs& a, int64_t t, float* __restrict__ buf, int wave,
                                          int lane) {
  typedef __attribute__((address_space(3))) void* lds_t;
  const float* src = a.c.act_tape + t * kTapeFloats;
  for (int q = wave; q < kActPieces; q += kStagers)
    __builtin_amdgcn_global_load_lds(src + q * 256 + lane * 4, (lds_t)(buf + kBA + q * 256), 16, 0, 0);
}

// a compiler fence on a tile's 16 values: everything that forms them happens before this point
__device__ __forceinline__ void pin16(f32x16& v) {
  asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
               "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15]));
}

// Wave 7, the cotangent chain of tile t into buf: the ReLU masks, the g half of the x | g table and
// dh4..dh0 of xyz_backward_saved (the colour decoder's outputs 0-2, decoder.py:198-203; the 4th row is
// the stage combiner's, decoder.py:341) without its feature-gradient GEMMs.  Each GEMM's weight
// fragment is loaded one step ahead (a fence per step keeps the rest from being hoisted).
__device__ __forceinline__ void produce_chain(const QueryKArgs& a, int64_t t, float* __restrict__ buf,
                                              const float* __restrict__ wo, int lane) {
  const int h = lane >> 5, p = lane & 31;
  const int64_t idx = t * 32 + p;
  const float* pk = a.c.packed[NSLAM_DEC_COLOR];
  const XyzPack L{1};
  Frag f = load_frag(pk + L.L4T() * NSLAM_FRAG, lane);
  f32x4 gv = {0.f, 0.f, 0.f, 0.f};
  if (idx < a.n) gv = *as_global(reinterpret_cast<const f32x4*>(a.g_raw + idx * 4));  // past the end: g = 0
  gv[3] = 0.f;
  if (h == 1) *reinterpret_cast<f32x4*>(buf + kBX + p * 8 + 4) = gv;
  uint32_t m[5];
  load_masks(a, NSLAM_DEC_COLOR, t, m, lane);
  uint16_t* mt = reinterpret_cast<uint16_t*>(buf + kBM);
#pragma unroll
  for (int i = 0; i < 5; ++i) mt[i * 64 + lane] = (uint16_t)m[i];
  f32x16 dh = zero16();
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const f32x16 w = vec_tile(wo + 32 * j, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) dh[r] += w[r] * gv[j];
  }
  if (a.c.g_h4 && idx < a.n) add_gh4(dh, a.c.g_h4 + idx * 32, lane);  // ABI v17: d/dh4 of a direct caller
  tstore(dimg(buf, 4), dh, lane);
  constexpr int kNext[3] = {3, 2, 1};  // the chain's next GEMMs: L3's h2 block, L2, L1 (transposed)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    __builtin_amdgcn_sched_barrier(0);
    const f32x16 da = apply_mask(dh, m[4 - k]);
    Frag fn = f;
    if (k < 3) {
      const int nf = kNext[k] == 3 ? L.L3T() + 3 : kNext[k] == 2 ? L.L2T() : L.L1T();
      fn = load_frag(pk + nf * NSLAM_FRAG, lane);
    }
    dh = zero16();
    gemm_frag(dh, f, da);
    tstore(dimg(buf, 3 - k), dh, lane);
    f = fn;
  }
}

// Wave 3, the colour feature of tile t (decoder.py:168-175; C layout → pitch-33 image) and the x half
// of the x | g table.  The trilinear gather of gather_tile (the forward's: the same corners, weights and
// summation order, so the same values) with each corner's row and weight formed next to its loads,
// NSLAM_CW_GATHER_NB corners at a time: the 8 corners' 64-bit addresses are never live together.
__device__ __forceinline__ void produce_feature(const QueryKArgs& a, int64_t t, float* __restrict__ buf, int lane) {
  const int h = lane >> 5, p = lane & 31;
  const Pt q = load_point(a, t * 32 + p);
  const nslam_grid& gr = a.c.grid[NSLAM_DEC_COLOR];
  if (h == 0) *reinterpret_cast<f32x4*>(buf + kBX + p * 8) = f32x4{q.x[0], q.x[1], q.x[2], 0.f};
  const int n[3] = {gr.dims[2], gr.dims[1], gr.dims[0]};  // x→W, y→H, z→D (make_corners)
  int i0[3];
  float f0[3], f1[3];
  bool hi_ok[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float gm;
    const float u = unnorm_clip(norm_coord(q.p[k], gr.lo[k], gr.hi[k]), n[k], gm);
    const float fl = floorf(u);
    i0[k] = (int)fl;
    f1[k] = u - fl;
    f0[k] = (float)(i0[k] + 1) - u;
    hi_ok[k] = (i0[k] + 1) <= n[k] - 1;
  }
  const int row0 = (i0[2] * n[1] + i0[1]) * n[0] + i0[0];
  f32x16 acc = zero16();
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (k % NSLAM_CW_GATHER_NB == 0) {
      pin16(acc);  // the previous batch is accumulated here: its loads are not held in registers
      __builtin_amdgcn_sched_barrier(0);
    }
    const int dx = k & 1, dy = (k >> 1) & 1, dz = k >> 2;
    const bool ok = (!dx || hi_ok[0]) && (!dy || hi_ok[1]) && (!dz || hi_ok[2]);
    const float wr = ((dx ? f1[0] : f0[0]) * (dy ? f1[1] : f0[1])) * (dz ? f1[2] : f0[2]);
    const float w = ok ? wr : 0.f;
    const int row = (row0 + (dz * n[1] + dy) * n[0] + dx) & -(int)ok;  // (a select, not a branch)
    const gptr_t<f32x4> rp =
        as_global(reinterpret_cast<const f32x4*>(gr.data + (size_t)(uint32_t)row * NSLAM_C_DIM + 4 * h));
    const f32x4 v0 = rp[0], v1 = rp[2], v2 = rp[4], v3 = rp[6];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[j] += v0[j] * w;
      acc[4 + j] += v1[j] * w;
      acc[8 + j] += v2[j] * w;
      acc[12 + j] += v3[j] * w;
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  tstore(buf + kBC, acc, lane);
}

// Waves 4-6: dB[c][32b + k] += Σ_p x_c[p] cos(x[p] B_b)[k] de_b[p][k], de_b = L3_bᵀ da3 + L0_bᵀ da0
// (decoder.py:29-30 backward).  de_b comes out transposed (lane (k, h), register r = point F(r, h)), so
// each lane sums its 16 points' products for its dim; the halves are added at the end.
__device__ __forceinline__ void fourier_bwd(const float* __restrict__ buf, const float* __restrict__ pk, int b,
                                            const float Bk[3], float dB[3], int lane) {
  const XyzPack L{1};
  const int h = lane >> 5;
  const uint16_t* mt = masks(buf);
  f32x16 de = zero16();
  {
    const f32x16 da3 = apply_mask(tload(dimg(buf, 3), lane), mt[3 * 64 + lane]);
    gemm_acc_t(de, pk + (L.L3T() + b) * NSLAM_FRAG, da3, lane);
  }
  __builtin_amdgcn_sched_barrier(0);
  {
    const f32x16 da0 = apply_mask(tload(dimg(buf, 0), lane), mt[lane]);
    gemm_acc_t(de, pk + (L.L0T() + b) * NSLAM_FRAG, da0, lane);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if (r % 4 == 0) __builtin_amdgcn_sched_barrier(0);
    const f32x4 x4 = *reinterpret_cast<const f32x4*>(buf + kBX + fidx(r, h) * 8);
    const float x[3] = {x4[0], x4[1], x4[2]};
    const float gk = de[r] * fcos(fourier_arg(x, Bk[0], Bk[1], Bk[2]));
    dB[0] = fmaf(x[0], gk, dB[0]);
    dB[1] = fmaf(x[1], gk, dB[1]);
    dB[2] = fmaf(x[2], gk, dB[2]);
  }
}

// The hand-over of a buffer: every wave's LDS-DMA into it has landed (an explicit vmcnt(0): with
// gfx950's back-off barriers the compiler does not drain it before s_barrier) and its LDS stores
// are visible (the barrier's fence).
__device__ __forceinline__ void handover() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}


// One role's pass over the chunk: prod(t, buf) fills buffer (t - t0) & 1 with tile t's share of this
// wave; cons(t, buf) consumes tile t.  Every role runs the same number of hand-overs (t1 - t0 + 1), so
// the workgroup's barriers match; each role's loop-carried values are its own (one role per wave: the
// register budget is the largest role's, not the union of all of them).
#ifdef NSLAM_PHASES
// phases build: per wave, the cycles spent producing, consuming and waiting at the hand-overs
#define CW_MARK(acc)                                           \
  do {                                                         \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    acc += now_ - last_;                                       \
    last_ = now_;                                              \
  } while (0)
#else
#define CW_MARK(acc) \
  do {               \
  } while (0)
#endif
template <class Prod, class Cons>
__device__ __forceinline__ void role_loop(float* lds, int64_t t0, int64_t t1, const Prod& prod, const Cons& cons) {
#ifdef NSLAM_PHASES
  unsigned long long last_ = __builtin_amdgcn_s_memtime(), tp = 0, tc = 0, th = 0;
#endif
  prod(t0, lds);
  CW_MARK(tp);
  handover();
  CW_MARK(th);
#pragma nounroll
  for (int64_t t = t0; t < t1; ++t) {
    const float* buf = lds + ((t - t0) & 1) * kBuf;
    float* nbuf = lds + ((t + 1 - t0) & 1) * kBuf;
    if (t + 1 < t1) prod(t + 1, nbuf);  // (its loads fly while this tile is computed)
    CW_MARK(tp);
    __builtin_amdgcn_sched_barrier(0);
    cons(t, buf);
    CW_MARK(tc);
    handover();  // the next buffer is complete / this one is free
    CW_MARK(th);
  }
#ifdef NSLAM_PHASES
  const int64_t w_ = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && w_ < kPhaseWaves) {
    unsigned long long* o = g_phase + ((size_t)4 * kPhaseWaves + w_) * 16;
    o[0] = tp;
    o[1] = tc;
    o[2] = th;
    o[3] = (unsigned long long)(t1 - t0);
  }
#endif
}

// The laundered lane: LDS addresses are functions of the lane only, i.e. loop-invariant; letting LICM
// hoist them out of the tile loop pins (and spills) the register file.  Re-derived per use.
__device__ __forceinline__ int fresh_lane(int lane0) {
  int lane = lane0;
  asm volatile("" : "+v"(lane));
  return lane;
}

}  // namespace

__global__ __launch_bounds__(64 * kCwWaves, NSLAM_CW_LB) void k_color_wgrad(CwArgs w) {
  // ONE __shared__ array (a second one can make hipcc drain the LDS-DMA early)
  __shared__ __attribute__((aligned(16))) float lds[kLds];
  const QueryKArgs& a = w.a;
  // role of this wave (the "wave" numbers of the header comment); hardware waves w and w + 4 share a
  // SIMD, and the permutation pairs each producer with a light S_b role and the three fc_c roles apart:
  // SIMD 0 chain + S_0, SIMD 1 feature + S_1, SIMD 2 fc_c.2 + S_2, SIMD 3 fc_c.0 + fc_c.1
  // (tools/probes/phases.py: the two producers on one SIMD made it the busiest by ~35 %)
  const int hw = wave_id();
  const int lane0 = threadIdx.x & 63, wave = NSLAM_CW_PERM ? (int)((0x52104637u >> (4 * hw)) & 15u) : hw;
  const int chunk = (int)blockIdx.x;
  const int64_t ntiles = (a.n + 31) / 32;
  const int64_t t0 = chunk * w.chunk_tiles;
  const int64_t t1 = t0 + w.chunk_tiles < ntiles ? t0 + w.chunk_tiles : ntiles;
  TL(2, 0, chunk);
  const nslam_dec_grad& dg = a.c.dgrad[NSLAM_DEC_COLOR];
  const float* pk = a.c.packed[NSLAM_DEC_COLOR];
  const XyzPack L{1};
  float* sl = w.slab + (size_t)chunk * w.acc;
  const int h0 = lane0 >> 5, j0 = lane0 & 31;
  // the output layer's rows 0-2 (decoder.py:198-203), read by every chain
  if (wave == 7)
    for (int i = lane0; i < 96; i += 64) lds[kWoOff + i] = as_global(pk + L.Wo())[i];
  __syncthreads();
  const auto stage = [&](int64_t t, float* buf) { stage_act(a, t, buf, wave, fresh_lane(lane0)); };

  if (wave < 3) {  // the embedding columns of dW_3 and dW_0: S_b = sin(x B_b) (decoder.py:29-30)
    const int b = wave, dim = 32 * b + j0;
    const float Bk[3] = {as_global(pk + L.FB())[dim], as_global(pk + L.FB())[96 + dim],
                         as_global(pk + L.FB())[192 + dim]};
    f32x16 acc3 = zero16(), acc0 = zero16();
    float unused = 0.f, db0 = 0.f;
    role_loop(lds, t0, t1, stage, [&](int64_t, const float* buf) {
      const int lane = fresh_lane(lane0);
      chain2<true>(acc3, acc0, unused, db0, Masked(buf, 3, lane), Emb(buf, Bk, lane), Masked(buf, 0, lane),
                   Emb(buf, Bk, lane));
    });
    const int kv = b < 2 ? 32 : NSLAM_EMB - 64;  // valid embedding columns of block b
    store_block(sl, dg.w[3], 125, 32 * b, kv, acc3, lane0);
    store_block(sl, dg.w[0], NSLAM_EMB, 32 * b, kv, acc0, lane0);
    if (b == 0) store_vec(sl, dg.b[0], db0, lane0);
  } else if (wave == 3) {  // the colour feature; layer 3's h2 columns, layer 2
    f32x16 acc3 = zero16(), acc2 = zero16();
    float db3 = 0.f, db2 = 0.f;
    role_loop(
        lds, t0, t1,
        [&](int64_t t, float* buf) {
          stage(t, buf);
          produce_feature(a, t, buf, fresh_lane(lane0));
        },
        [&](int64_t, const float* buf) {
          const int lane = fresh_lane(lane0);
          chain2<false>(acc3, acc2, db3, db2, Masked(buf, 3, lane), Img<32>(act(buf, 2), lane), Masked(buf, 2, lane),
                        Img<32>(act(buf, 1), lane));
        });
    store_block(sl, dg.w[3], 125, 93, 32, acc3, lane0);
    store_vec(sl, dg.b[3], db3, lane0);
    store_block(sl, dg.w[2], 32, 0, 32, acc2, lane0);
    store_vec(sl, dg.b[2], db2, lane0);
  } else if (wave < 7) {  // fc_c (dWc_i = Σ dh_i ⊗ c), layer 4, the Fourier B
    const int b = wave - 4, dim = 32 * b + j0;
    const float Bk[3] = {as_global(pk + L.FB())[dim], as_global(pk + L.FB())[96 + dim],
                         as_global(pk + L.FB())[192 + dim]};
    f32x16 accA = zero16(), accB = zero16();
    float bA = 0.f, bB = 0.f;
    float dB[4] = {0.f, 0.f, 0.f, 0.f};
    role_loop(lds, t0, t1, stage, [&](int64_t, const float* buf) {
      const int lane = fresh_lane(lane0);
      const Img<TPITCH> C(buf + kBC, lane);
      if (b == 2)
        chain2<false>(accA, accB, bA, bB, Img<TPITCH>(dimg(buf, 2), lane), C, Masked(buf, 4, lane),
                      Img<32>(act(buf, 3), lane));
      else
        chain2<true>(accA, accB, bA, bB, Img<TPITCH>(dimg(buf, b), lane), C, Img<TPITCH>(dimg(buf, b + 3), lane), C);
      fourier_bwd(buf, pk, b, Bk, dB, lane);
    });
    if (b == 2) {
      store_block(sl, dg.wc[2], 32, 0, 32, accA, lane0);
      store_vec(sl, dg.bc[2], bA, lane0);
      store_block(sl, dg.w[4], 32, 0, 32, accB, lane0);
      store_vec(sl, dg.b[4], bB, lane0);
    } else {
      store_block(sl, dg.wc[b], 32, 0, 32, accA, lane0);
      store_vec(sl, dg.bc[b], bA, lane0);
      store_block(sl, dg.wc[b + 3], 32, 0, 32, accB, lane0);
      store_vec(sl, dg.bc[b + 3], bB, lane0);
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = dB[c] + xor32(dB[c]);
      if (h0 == 0 && dim < NSLAM_EMB) as_global_w(sl)[dg.B + c * NSLAM_EMB + dim] = v;
    }
  } else {  // wave 7: the cotangent chain; layer 1; the output layer
    const float* wo = lds + kWoOff;
    f32x16 acc1 = zero16();
    float db1 = 0.f;
    float e[4] = {0.f, 0.f, 0.f, 0.f};  // dWo rows 0-2, dbo
    role_loop(
        lds, t0, t1, [&](int64_t t, float* buf) { produce_chain(a, t, buf, wo, fresh_lane(lane0)); },
        [&](int64_t, const float* buf) {
          const int lane = fresh_lane(lane0);
          const int h = lane >> 5, j = lane & 31;
          chain1(acc1, db1, Masked(buf, 1, lane), Img<32>(act(buf, 0), lane));
          // output layer: dWo = Σ g ⊗ h4 (rows 0-2), dbo
          const Img<32> H4(act(buf, 4), lane);
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            if (s % kG == 0) __builtin_amdgcn_sched_barrier(0);
            const f32x4 g = *reinterpret_cast<const f32x4*>(buf + kBX + (2 * s + h) * 8 + 4);
            const float hv = H4(s);
            e[0] = fmaf(g[0], hv, e[0]);
            e[1] = fmaf(g[1], hv, e[1]);
            e[2] = fmaf(g[2], hv, e[2]);
            e[3] += j == 0 ? g[0] : (j == 1 ? g[1] : g[2]);
          }
        });
    store_block(sl, dg.w[1], 32, 0, 32, acc1, lane0);
    store_vec(sl, dg.b[1], db1, lane0);
    const float wo0 = e[0] + xor32(e[0]), wo1 = e[1] + xor32(e[1]), wo2 = e[2] + xor32(e[2]);
    const float bo = e[3] + xor32(e[3]);
    if (h0 == 0) {
      as_global_w(sl)[dg.wo + j0] = wo0;
      as_global_w(sl)[dg.wo + 32 + j0] = wo1;
      as_global_w(sl)[dg.wo + 64 + j0] = wo2;
      as_global_w(sl)[dg.wo + 96 + j0] = 0.f;  // row 3 (occupancy) is replaced by the stage combiner
      if (j0 < 4) as_global_w(sl)[dg.bo + j0] = j0 < 3 ? bo : 0.f;
    }
  }
  TL(2, 1, 0);
}

int launch_color_wgrad(const QueryKArgs& a, float* ws, hipStream_t s) {
  const nslam_dec_grad& dg = a.c.dgrad[NSLAM_DEC_COLOR];
  const CwPlan pl = cw_plan(dg, a.n);
  CwArgs w{a, ws, acc_floats_of(dg), pl.nchunks, pl.chunk_tiles};
  hipLaunchKernelGGL(k_color_wgrad, dim3((unsigned)pl.nchunks), dim3(64 * kCwWaves), 0, s, w);
  const int rc = hip_status();
  return rc ? rc : slab_reduce(dg, w.slab, false, pl.nchunks, 0, w.acc, s);
}

}  // namespace nslamq
