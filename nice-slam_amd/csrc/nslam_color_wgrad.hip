// nslam_color_wgrad.hip — the colour decoder's parameter gradients of a mapping iteration
// (Mapper.py:503 reaching color_decoder.parameters(), fix_color False; decoder.py:177-203 backward)
// as a split-K reduction over the points, from three tapes of the iteration:
//   activation tape (forward):  h0..h4 and the colour feature c of every 32-point tile
//   cotangent tape (lean chain): dh0..dh4, the hidden-layer cotangents before their ReLU masks, and
//                                each point's x and colour cotangent g
//   saved ReLU masks (forward):  da_i = mask_i ⊙ dh_i
// One workgroup (8 waves, one per CU: LDS) owns a chunk of consecutive tiles.  Each tile's tapes
// (45 KiB) are staged into LDS once by LDS-DMA (double-buffered: the next tile's copies are in
// flight while the waves compute on the current one), and the waves share them: every weight block
// dW = Σ_points (cotangent ⊗ input) is an MFMA chain whose A and B operands are point-major LDS
// image streams (element s of lane (j, h) = point P(s, h), column j; any bijection of the points
// serves, since they are the reduction axis), accumulated in registers over the whole chunk and
// written once: a chunk's partial sums fill one slab (each wave a disjoint part of it), and
// k_slab_reduce sums the chunks' slabs in a fixed order (deterministic).
//
// Blocks, assigned to the 8 waves (waves w and w + 4 share a SIMD), in two phases per tile split by
// a bare barrier (the next tile's LDS-DMA keeps flying across it):
//   Fourier block b = 0..2 (dims 32b..32b+31 of the embedding, decoder.py:26-30), on SIMD b:
//     wave b, A:     e = sin(x B_b), cs = cos(x B_b) by one range reduction, points in the C-layout
//                    order F(s, h); dW_3[:, 32b..] = Σ da3 ⊗ e, dW_0[:, 32b..] = Σ da0 ⊗ e (db_0, b = 0)
//     wave b + 4, A: G^T = da3 L3_b + da0 L0_b (MFMA, C rows = points) → LDS, lane-private
//     wave b, B:     dB[:, 32b..] += Σ_points x ⊗ (G^T ⊙ cs)  (VALU: lane j owns dim 32b+j)
//     wave b + 4, B: fc_c.b  dWc_b = Σ dh_b ⊗ c, dbc_b = Σ dh_b
//   wave 3: fc_c.3, fc_c.4 (A); layer 4: dW_4 = Σ da4 ⊗ h3, db_4 (B)
//   wave 7: layer 3's h2 columns dW_3[:, 93:125] = Σ da3 ⊗ h2, db_3, and layer 2 (A); layer 1 (B)
//   wave 0, B: output dWo = Σ g ⊗ h4 (rows 0-2; row 3 is replaced by the stage combiner), dbo (VALU)
#include "nslam_query_impl.h"

namespace nslamq {

namespace {

constexpr int kCwWaves = 8;
constexpr int kImg = 1024;                // one [32 points][32 features] image (lane-linear rows: glds)
constexpr int kImgs = 11;                 // dh0..dh4, h0..h4, c
constexpr int kXgOff = kImgs * kImg;      // [32][8]: x (3 + pad), g (3 + pad) of each point
constexpr int kMaskOff = kXgOff + 32 * 8;  // u16 [layer 5][64 lanes]: the forward's saved masks (C layout)
constexpr int kBuf = kMaskOff + 5 * 32;    // floats per staged tile
constexpr int kPieces = 21 + 24;           // 1-KiB LDS-DMA pieces per tile (cotangent tape, activation tape)
constexpr int kFragPitch = 20;             // floats per lane of an LDS fragment (conflict-free b128 reads)
constexpr int kFragOff = 2 * kBuf;                     // [6][64][20]: L3T_b, L0T_b fragments (b = 0..2)
constexpr int kFbOff = kFragOff + 6 * 64 * kFragPitch;  // [3][96] Fourier B
constexpr int kGtOff = kFbOff + 3 * 96;                 // [3][64][20]: G^T blocks, lane-private (wave b+4 → b)
constexpr int kLds = kGtOff + 3 * 64 * kFragPitch;
static_assert(kBuf % 4 == 0 && kFragOff % 4 == 0 && kGtOff % 4 == 0, "16-B aligned LDS regions");

struct CwArgs {
  QueryKArgs a;
  float* slab;          // [nchunks][acc]
  int acc;              // floats per slab
  int nchunks;
  int64_t chunk_tiles;  // tiles per chunk
};

enum : int { kDh = 0, kH = 5, kC = 10 };
__device__ __forceinline__ const float* img(const float* buf, int k) { return buf + k * kImg; }
__device__ __forceinline__ const uint16_t* masks(const float* buf) {
  return reinterpret_cast<const uint16_t*>(buf + kMaskOff);
}
// the point of stream element s in half h: the C layout's order F(s, h)
__device__ __forceinline__ int pnt(int s, int h) { return fidx(s, h); }

// Point-major stream of an image: element s of lane (j, h) = image[P(s, h)][j]
__device__ __forceinline__ f32x16 lstream(const float* __restrict__ im, int lane) {
  const int h = lane >> 5, j = lane & 31;
  f32x16 v;
#pragma unroll
  for (int s = 0; s < 16; ++s) v[s] = im[pnt(s, h) * 32 + j];
  return v;
}
// v if bit `bit` of w is set, else +0 (v_bfe_i32 + v_and)
__device__ __forceinline__ float keep(float v, uint32_t w, int bit) {
  return __builtin_bit_cast(float, __builtin_bit_cast(int, v) & __builtin_amdgcn_sbfe((int)w, bit, 1));
}
// da_i stream: the dh_i stream times the ReLU mask.  Feature j of point P is bit r(j) of the saved
// mask of lane (P, h(j)) (C layout: feature F(r, h) = j).
__device__ __forceinline__ f32x16 lstream_masked(const float* __restrict__ buf, int i, int lane) {
  const int h = lane >> 5, j = lane & 31;
  const int hj = (j >> 2) & 1, rj = (j & 3) + 4 * (j >> 3);
  f32x16 v = lstream(img(buf, kDh + i), lane);
  const uint16_t* ms = masks(buf) + i * 64 + 32 * hj;
#pragma unroll
  for (int s = 0; s < 16; ++s) v[s] = keep(v[s], ms[pnt(s, h)], rj);
  return v;
}
// C-layout read of da_i: lane (p, h) gets features F(r, h) of point p, masked
__device__ __forceinline__ f32x16 lcload_masked(const float* __restrict__ buf, int i, int lane) {
  const int p = lane & 31, h = lane >> 5;
  const float* im = img(buf, kDh + i);
  const uint32_t m = masks(buf)[i * 64 + lane];
  f32x16 v;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x4 w = *reinterpret_cast<const f32x4*>(im + p * 32 + 8 * k + 4 * h);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[4 * k + e] = keep(w[e], m, 4 * k + e);
  }
  return v;
}

__device__ __forceinline__ void mfma_chain(f32x16& acc, const f32x16& A, const f32x16& B) {
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = mfma32(A[s], B[s], acc);
}
__device__ __forceinline__ float sum16(const f32x16& v) {
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += v[r];
  return s;
}
// acc += da ⊗ input over the tile's points (and the bias sum of da)
__device__ __forceinline__ void wblock(f32x16& acc, float& bias, const f32x16& A, const float* __restrict__ in,
                                       int lane) {
  mfma_chain(acc, A, lstream(in, lane));
  bias += sum16(A);
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

// Tile staging by LDS-DMA (global_load_lds; the hardware writes lane l's bytes at the wave-uniform
// LDS address + l × size): 45 pieces of 1 KiB (16 B per lane) from the two tapes and the 640-B mask
// row block in pieces of 256 B (4 B per lane).  Piece q is issued by wave q % 8.
__device__ __forceinline__ void stage(const QueryKArgs& a, int64_t t, float* __restrict__ buf, int wave, int lane) {
  typedef __attribute__((address_space(3))) void* lds_t;
  const float* cot = a.cot + t * kCotFloats;
  const float* act = a.c.act_tape + t * kTapeFloats;
  for (int q = wave; q < kPieces; q += kCwWaves) {
    const float* src = q < 21 ? cot + q * 256 : act + (q - 21) * 256;  // dh0..4, xg | h0..4, c
    float* dst = q < 20 ? buf + q * 256 : q == 20 ? buf + kXgOff : buf + kH * kImg + (q - 21) * 256;
    __builtin_amdgcn_global_load_lds(src + lane * 4, (lds_t)dst, 16, 0, 0);
  }
  if (wave == kPieces % kCwWaves) {  // the mask rows: 2 full pieces and one of 32 lanes
    const uint16_t* ms = mask_slot(a, NSLAM_DEC_COLOR, t);
    float* dst = buf + kMaskOff;
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (i < 2 || lane < 32)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint32_t*>(ms) + i * 64 + lane,
                                         (lds_t)(dst + i * 64), 4, 0, 0);
  }
}

// phases build: lane 0 of each wave marks its chunk's third tile (and kernel start / end) into
// g_phase slot 0, waves 16384 + 8 chunk + wave
#ifdef NSLAM_PHASES
#define CW_PHASE(k, cond)                                                                      \
  do {                                                                                         \
    const int w_ = 16384 + (int)blockIdx.x * kCwWaves + (int)(threadIdx.x >> 6);               \
    if ((cond) && (threadIdx.x & 63) == 0 && w_ < kPhaseWaves)                                 \
      g_phase[(size_t)w_ * 16 + (k)] = __builtin_amdgcn_s_memtime();                           \
  } while (0)
#else
#define CW_PHASE(k, cond) \
  do {                    \
  } while (0)
#endif

}  // namespace

__global__ __launch_bounds__(64 * kCwWaves, 1) void k_color_wgrad(CwArgs w) {
  // ONE __shared__ array (a second one can make hipcc drain the LDS-DMA early)
  __shared__ __attribute__((aligned(16))) float lds[kLds];
  const QueryKArgs& a = w.a;
  const int tid = threadIdx.x, lane0 = tid & 63, wave = wave_id();
  const int chunk = (int)blockIdx.x;
  const int64_t ntiles = (a.n + 31) / 32;
  const int64_t t0 = chunk * w.chunk_tiles;
  const int64_t t1 = t0 + w.chunk_tiles < ntiles ? t0 + w.chunk_tiles : ntiles;
  const nslam_dec_grad& dg = a.c.dgrad[NSLAM_DEC_COLOR];
  const float* pk = a.c.packed[NSLAM_DEC_COLOR];
  const XyzPack L{1};
  CW_PHASE(0, true);
  stage(a, t0, lds, wave, lane0);
  // loop-invariant operands into LDS: the Fourier blocks' L3T_b / L0T_b fragments and B
  for (int e = tid; e < 6 * 64 * 16; e += 64 * kCwWaves) {
    const int f = e >> 10, l = (e >> 4) & 63, k = e & 15;
    const int blk = f < 3 ? L.L3T() + f : L.L0T() + (f - 3);
    lds[kFragOff + (f * 64 + l) * kFragPitch + k] = as_global(pk)[blk * NSLAM_FRAG + l * 16 + k];
  }
  for (int e = tid; e < 3 * 96; e += 64 * kCwWaves) lds[kFbOff + e] = as_global(pk + L.FB())[e];
  __syncthreads();  // (its vmcnt(0) retires the LDS-DMA)
  const int fb = wave < 3 ? wave : 0;  // Fourier block of waves 0-2
  const int dim = 32 * fb + (lane0 & 31);  // the embedding dim of lane j (< 96: B is padded)
  const float B0 = lds[kFbOff + dim], B1 = lds[kFbOff + 96 + dim], B2 = lds[kFbOff + 192 + dim];

  f32x16 accA = zero16(), accB = zero16(), accC = zero16();  // role accumulators
  float bA = 0.f, bB = 0.f, bC = 0.f;                          // bias sums
  float dB0 = 0.f, dB1 = 0.f, dB2 = 0.f;                       // Fourier: dB[c][dim] partial sums
  float wo0 = 0.f, wo1 = 0.f, wo2 = 0.f, bo = 0.f;             // output layer (VALU)
  f32x16 cs;                                                   // Fourier: cos, phase A → B
#pragma nounroll
  for (int64_t t = t0; t < t1; ++t) {
    // The LDS addresses are functions of the lane only, i.e. loop-invariant; letting LICM hoist them
    // pins (and spills) the register file.  Re-derive them per tile.
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const int h = lane >> 5, j = lane & 31;
    const float* buf = lds + ((t - t0) & 1) * kBuf;
    const bool mk = t == t0 + 2;
    CW_PHASE(1, mk);
    if (t + 1 < t1) stage(a, t + 1, lds + ((t + 1 - t0) & 1) * kBuf, wave, lane);  // flies during this tile
    CW_PHASE(2, mk);
    // phase A
    if (wave < 3) {  // e = sin, cs = cos of (x B)[P(s, h)][dim]; dW_3 / dW_0 columns of block fb
      f32x16 e;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(buf + kXgOff + pnt(s, h) * 8);
        const float xv[3] = {x[0], x[1], x[2]};
        float sv, cv;
        fsincos(fourier_arg(xv, B0, B1, B2), sv, cv);  // decoder.py:29-30
        e[s] = sv;
        cs[s] = cv;
      }
      const f32x16 A3 = lstream_masked(buf, 3, lane);
      mfma_chain(accA, A3, e);
      const f32x16 A0 = lstream_masked(buf, 0, lane);
      mfma_chain(accB, A0, e);
      if (wave == 0) bA += sum16(A0);
    } else if (wave != 3 && wave != 7) {
      // G^T[point][dim] = Σ_m da3[point][m] L3_b[m][dim] + (da0, L0_b) of block b = wave - 4: C rows =
      // points F(r, h), lane (dim, h) — the lane / register order of wave b's cs, so the hand-over is
      // lane-private
      const int b = wave - 4;
      f32x16 gt = zero16();
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const f32x16 da = lcload_masked(buf, f == 0 ? 3 : 0, lane);
        const f32x4* fr = reinterpret_cast<const f32x4*>(lds + kFragOff + ((3 * f + b) * 64 + lane) * kFragPitch);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const f32x4 q = fr[k];
#pragma unroll
          for (int u = 0; u < 4; ++u) gt = mfma32(da[4 * k + u], q[u], gt);
        }
      }
      f32x4* o = reinterpret_cast<f32x4*>(lds + kGtOff + (b * 64 + lane) * kFragPitch);
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = f32x4{gt[4 * k], gt[4 * k + 1], gt[4 * k + 2], gt[4 * k + 3]};
    } else if (wave == 3) {  // fc_c.3, fc_c.4
      wblock(accA, bA, lstream(img(buf, kDh + 3), lane), img(buf, kC), lane);
      wblock(accB, bB, lstream(img(buf, kDh + 4), lane), img(buf, kC), lane);
    } else {  // layer 3's h2 columns, layer 2
      wblock(accA, bA, lstream_masked(buf, 3, lane), img(buf, kH + 2), lane);
      wblock(accB, bB, lstream_masked(buf, 2, lane), img(buf, kH + 1), lane);
    }
    CW_PHASE(3, mk);
    // G^T hand-over: LDS writes retired, then a bare barrier (no vmcnt(0): the next tile's LDS-DMA
    // keeps flying)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // phase B
    if (wave < 3) {  // dB[c][dim] += Σ_points x_c G^T ⊙ cs; output layer (wave 0)
      const f32x4* gi = reinterpret_cast<const f32x4*>(lds + kGtOff + (wave * 64 + lane) * kFragPitch);
      int xo = kXgOff;  // laundered: keeps the x loads of phase A from being CSE'd across (64 VGPRs)
      asm volatile("" : "+s"(xo));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f32x4 g4 = gi[k];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = 4 * k + u;
          const float gv = g4[u] * cs[r];
          const f32x4 x = *reinterpret_cast<const f32x4*>(buf + xo + pnt(r, h) * 8);
          dB0 = fmaf(x[0], gv, dB0);
          dB1 = fmaf(x[1], gv, dB1);
          dB2 = fmaf(x[2], gv, dB2);
        }
      }
      if (wave == 0) {  // dWo = g ⊗ h4 (rows 0-2), dbo
        const f32x16 H4 = lstream(img(buf, kH + 4), lane);
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) {
          const f32x4 g = *reinterpret_cast<const f32x4*>(buf + xo + pnt(s2, h) * 8 + 4);
          wo0 = fmaf(g[0], H4[s2], wo0);
          wo1 = fmaf(g[1], H4[s2], wo1);
          wo2 = fmaf(g[2], H4[s2], wo2);
          bo += j == 0 ? g[0] : (j == 1 ? g[1] : g[2]);
        }
      }
    } else if (wave != 3 && wave != 7) {  // fc_c.(wave - 4)
      wblock(accA, bA, lstream(img(buf, kDh + wave - 4), lane), img(buf, kC), lane);
    } else if (wave == 3) {  // layer 4
      wblock(accC, bC, lstream_masked(buf, 4, lane), img(buf, kH + 3), lane);
    } else {  // layer 1
      wblock(accC, bC, lstream_masked(buf, 1, lane), img(buf, kH + 0), lane);
    }
    CW_PHASE(4, mk);
    __syncthreads();  // next buffer landed (vmcnt(0) retires this wave's LDS-DMA) / this one free
    CW_PHASE(5, mk);
  }
  CW_PHASE(8, true);

  // write the chunk's slab (each wave its disjoint blocks)
  const int lane = lane0, h = lane >> 5, j = lane & 31;
  float* sl = w.slab + (size_t)chunk * w.acc;
  if (wave < 3) {
    const int kv = fb < 2 ? 32 : NSLAM_EMB - 64;
    store_block(sl, dg.w[3], 125, 32 * fb, kv, accA, lane);
    store_block(sl, dg.w[0], NSLAM_EMB, 32 * fb, kv, accB, lane);
    dB0 += xor32(dB0);
    dB1 += xor32(dB1);
    dB2 += xor32(dB2);
    if (h == 0 && dim < NSLAM_EMB) {
      as_global_w(sl)[dg.B + dim] = dB0;
      as_global_w(sl)[dg.B + NSLAM_EMB + dim] = dB1;
      as_global_w(sl)[dg.B + 2 * NSLAM_EMB + dim] = dB2;
    }
    if (wave == 0) {
      store_vec(sl, dg.b[0], bA, lane);
      wo0 += xor32(wo0);
      wo1 += xor32(wo1);
      wo2 += xor32(wo2);
      bo += xor32(bo);
      if (h == 0) {
        as_global_w(sl)[dg.wo + j] = wo0;
        as_global_w(sl)[dg.wo + 32 + j] = wo1;
        as_global_w(sl)[dg.wo + 64 + j] = wo2;
        as_global_w(sl)[dg.wo + 96 + j] = 0.f;  // row 3 (occupancy) is replaced by the stage combiner
        if (j < 4) as_global_w(sl)[dg.bo + j] = j < 3 ? bo : 0.f;
      }
    }
  } else if (wave != 3 && wave != 7) {
    store_block(sl, dg.wc[wave - 4], 32, 0, 32, accA, lane);
    store_vec(sl, dg.bc[wave - 4], bA, lane);
  } else if (wave == 3) {
    store_block(sl, dg.wc[3], 32, 0, 32, accA, lane);
    store_vec(sl, dg.bc[3], bA, lane);
    store_block(sl, dg.wc[4], 32, 0, 32, accB, lane);
    store_vec(sl, dg.bc[4], bB, lane);
    store_block(sl, dg.w[4], 32, 0, 32, accC, lane);
    store_vec(sl, dg.b[4], bC, lane);
  } else {
    store_block(sl, dg.w[3], 125, 93, 32, accA, lane);
    store_vec(sl, dg.b[3], bA, lane);
    store_block(sl, dg.w[2], 32, 0, 32, accB, lane);
    store_vec(sl, dg.b[2], bB, lane);
    store_block(sl, dg.w[1], 32, 0, 32, accC, lane);
    store_vec(sl, dg.b[1], bC, lane);
  }
  CW_PHASE(9, true);
}

int launch_color_wgrad(const QueryKArgs& a, float* ws, hipStream_t s) {
  const nslam_dec_grad& dg = a.c.dgrad[NSLAM_DEC_COLOR];
  const CwPlan pl = cw_plan(dg, a.n);
  CwArgs w{a, ws + pl.cot_bytes / sizeof(float), acc_floats_of(dg), pl.nchunks, pl.chunk_tiles};
  w.a.cot = ws;
  hipLaunchKernelGGL(k_color_wgrad, dim3((unsigned)pl.nchunks), dim3(64 * kCwWaves), 0, s, w);
  const int rc = hip_status();
  return rc ? rc : slab_reduce(dg, w.slab, false, pl.nchunks, 0, w.acc, s);
}

}  // namespace nslamq
