// nslam_color_wgrad.hip — the colour decoder's parameter gradients of a mapping iteration
// (Mapper.py:503 reaching color_decoder.parameters(), fix_color False; decoder.py:177-203 backward)
// as a split-K reduction over the points, from the tapes of the iteration:
//   activation tape (forward):  h0..h4 of every 32-point tile
//   cotangent tape (lean chain): dh0..dh4 (the hidden-layer cotangents before their ReLU masks), the
//                                embedding S = sin(x B) and Gc = (embedding cotangent) ⊙ cos(x B), the
//                                colour feature c, and each point's x and colour cotangent g
//   saved ReLU masks (forward):  da_i = mask_i ⊙ dh_i
// so this kernel is MFMA chains over LDS images and a little VALU: no transcendental work.
// One workgroup (8 waves; its LDS holds two staged tiles, so one per CU) owns a chunk of consecutive
// tiles.  Each tile's tapes (70 KiB) are staged into LDS once by LDS-DMA, double-buffered: every wave
// issues its share of the next tile's pieces at the top of the current one, and they land while the
// waves compute.  Every weight block dW = Σ_points (cotangent ⊗ input) is an MFMA chain whose A and
// B operands are point-major LDS image streams (element s of lane (j, h) = point 2s + h, column j:
// the two rows of one read are 32 floats apart, i.e. on disjoint banks; any bijection of the points
// serves, since they are the reduction axis), accumulated in registers over the whole chunk and
// written once: a chunk's partial sums fill one slab (each wave a disjoint part of it), and
// k_slab_reduce sums the chunks' slabs in a fixed order (deterministic).
//
// Roles (waves w and w + 4 share a SIMD; at most 64 MFMAs per SIMD per tile):
//   wave b = 0..2 (embedding dims 32b..32b+31, decoder.py:26-30):
//            dW_3[:, 32b..] = Σ da3 ⊗ S_b, dW_0[:, 32b..] = Σ da0 ⊗ S_b (+ db_0, b = 0)
//   wave 4: fc_c.0, fc_c.3    wave 5: fc_c.1, fc_c.4    wave 6: fc_c.2, layer 4 (da4 ⊗ h3)
//           and each dB[:, 32b..] += Σ_p x ⊗ Gc_b for b = wave - 4 (VALU: lane j owns dim 32b + j)
//   wave 3: layer 3's h2 columns dW_3[:, 93:125] = Σ da3 ⊗ h2 (+ db_3), layer 2 (da2 ⊗ h1)
//   wave 7: layer 1 (da1 ⊗ h0); output dWo = Σ g ⊗ h4 (rows 0-2; row 3 is replaced by the stage
//           combiner), dbo (VALU)
// One barrier per tile (the double buffer's hand-over); no wave waits on another inside a tile.
#include "nslam_query_impl.h"

namespace nslamq {

namespace {

constexpr int kCwWaves = 8;
constexpr int kImg = 1024;                     // one [32 points][32 features] image
constexpr int kXgOff = kCotXg;                 // [32][8]: x (3 + pad), g (3 + pad) of each point
constexpr int kActOff = kCotFloats;            // the activation tape's h0..h4 follow the cotangent tape
constexpr int kMaskOff = kActOff + kTapeFloats;  // u16 [layer 5][64 lanes]: the forward's saved masks
constexpr int kBuf = kMaskOff + 5 * 32;          // floats per staged tile
constexpr int kCotPieces = kCotFloats / 256;     // 1-KiB LDS-DMA pieces (16 B per lane)
constexpr int kPieces = kCotPieces + kTapeFloats / 256;
constexpr int kLds = 2 * kBuf;
static_assert(kCotFloats % 256 == 0 && kTapeFloats % 256 == 0, "tapes are whole 1-KiB pieces");
static_assert(kBuf % 4 == 0, "16-B aligned LDS regions");
static_assert(kLds * 4 <= 160 * 1024, "LDS");

struct CwArgs {
  QueryKArgs a;
  float* slab;          // [nchunks][acc]
  int acc;              // floats per slab
  int nchunks;
  int64_t chunk_tiles;  // tiles per chunk
};

__device__ __forceinline__ const float* img(const float* buf, int k) { return buf + k * kImg; }
__device__ __forceinline__ const float* act(const float* buf, int i) { return buf + kActOff + i * kImg; }
__device__ __forceinline__ const uint16_t* masks(const float* buf) {
  return reinterpret_cast<const uint16_t*>(buf + kMaskOff);
}
// the point of stream element s in half h
__device__ __forceinline__ int pnt(int s, int h) { return 2 * s + h; }

// Point-major stream of an image: element s of lane (j, h) = image[2s + h][j]
__device__ __forceinline__ f32x16 lstream(const float* __restrict__ im, int lane) {
  const float* p = im + lane;  // (j, h) → row h, column j; element s adds two rows
  f32x16 v;
#pragma unroll
  for (int s = 0; s < 16; ++s) v[s] = p[64 * s];
  return v;
}
// v if bit `bit` of w is set, else +0 (v_bfe_i32 + v_and)
__device__ __forceinline__ float keep(float v, uint32_t w, int bit) {
  return __builtin_bit_cast(float, __builtin_bit_cast(int, v) & __builtin_amdgcn_sbfe((int)w, bit, 1));
}
// da_i stream: the dh_i stream times the ReLU mask.  Feature j of point P is bit r(j) of the saved
// mask of lane (P, h(j)) (the forward's C layout: feature F(r, h) = j).
__device__ __forceinline__ f32x16 lstream_masked(const float* __restrict__ buf, int i, int lane) {
  const int h = lane >> 5, j = lane & 31;
  const int hj = (j >> 2) & 1, rj = (j & 3) + 4 * (j >> 3);
  f32x16 v = lstream(img(buf, i), lane);
  const uint16_t* ms = masks(buf) + i * 64 + 32 * hj + h;
#pragma unroll
  for (int s = 0; s < 16; ++s) v[s] = keep(v[s], ms[2 * s], rj);
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
// acc += A ⊗ B over the tile's points, and the bias sum of A
__device__ __forceinline__ void wblock(f32x16& acc, float& bias, const f32x16& A, const f32x16& B) {
  mfma_chain(acc, A, B);
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
// LDS address + l × size).  The staged buffer is the tile's cotangent tape then its activation tape
// exactly as they lie in global memory (pieces of 1 KiB, 16 B per lane), then the 640-B mask rows
// (pieces of 256 B, 4 B per lane).  Piece q is issued by wave q % 8 (an LDS-DMA piece costs its
// wave ~100 issue cycles: spread, they cost every wave the same ~1k); wave 7 also takes the masks.
__device__ __forceinline__ void stage(const QueryKArgs& a, int64_t t, float* __restrict__ buf, int wave, int lane) {
  typedef __attribute__((address_space(3))) void* lds_t;
  const float* cot = a.cot + t * kCotFloats;
  const float* act = a.c.act_tape + t * kTapeFloats;
  for (int q = wave; q < kPieces; q += kCwWaves) {
    const float* src = q < kCotPieces ? cot + q * 256 : act + (q - kCotPieces) * 256;
    __builtin_amdgcn_global_load_lds(src + lane * 4, (lds_t)(buf + q * 256), 16, 0, 0);
  }
  if (wave == 7) {  // the mask rows: 2 full pieces and one of 32 lanes
    const uint16_t* ms = mask_slot(a, NSLAM_DEC_COLOR, t);
    float* dst = buf + kMaskOff;
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (i < 2 || lane < 32)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint32_t*>(ms) + i * 64 + lane,
                                         (lds_t)(dst + i * 64), 4, 0, 0);
  }
}

// Register staging (NSLAM_CW_REGSTAGE, default): the same pieces moved by ordinary 16-B global loads
// into registers at the top of a tile and written to the other LDS buffer (ds_write_b128) at its
// end.  An LDS-DMA piece costs its wave 100-190 issue cycles inside this loop (MI355X guide), and
// the two waves of a SIMD issued ~18 of them per tile: ~2.8k of the tile's 8.6k cycles (phase
// marks, profiles/r03_experiments); a global load + ds_write pair issues in a few tens.
#ifndef NSLAM_CW_REGSTAGE
#define NSLAM_CW_REGSTAGE 0  // measured equal (206.2 vs 205.9 M ray-samples/s): the LDS-DMA path stays
#endif
constexpr int kPiecesPerWave = (kPieces + kCwWaves - 1) / kCwWaves;
struct Staged {
  f32x4 v[kPiecesPerWave];
  uint32_t m[3];
};
__device__ __forceinline__ void fetch(const QueryKArgs& a, int64_t t, Staged& st, int wave, int lane) {
  const float* cot = a.cot + t * kCotFloats;
  const float* act = a.c.act_tape + t * kTapeFloats;
#pragma unroll
  for (int k = 0; k < kPiecesPerWave; ++k) {
    const int q = wave + kCwWaves * k;
    if (q < kPieces) {
      const float* src = q < kCotPieces ? cot + q * 256 : act + (q - kCotPieces) * 256;
      st.v[k] = *as_global(reinterpret_cast<const f32x4*>(src) + lane);
    }
  }
  if (wave == 7) {
    const uint32_t* ms = reinterpret_cast<const uint32_t*>(mask_slot(a, NSLAM_DEC_COLOR, t));
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (i < 2 || lane < 32) st.m[i] = *as_global(ms + i * 64 + lane);
  }
}
__device__ __forceinline__ void commit(float* __restrict__ buf, const Staged& st, int wave, int lane) {
#pragma unroll
  for (int k = 0; k < kPiecesPerWave; ++k) {
    const int q = wave + kCwWaves * k;
    if (q < kPieces) reinterpret_cast<f32x4*>(buf + q * 256)[lane] = st.v[k];
  }
  if (wave == 7) {
    uint32_t* dst = reinterpret_cast<uint32_t*>(buf + kMaskOff);
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (i < 2 || lane < 32) dst[i * 64 + lane] = st.m[i];
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
  CW_PHASE(0, true);
#if NSLAM_CW_REGSTAGE
  Staged st;
  fetch(a, t0, st, wave, lane0);
  commit(lds, st, wave, lane0);
#else
  stage(a, t0, lds, wave, lane0);
#endif
  __syncthreads();  // (its vmcnt(0) retires the LDS-DMA)
  const int fb = wave < 3 ? wave : wave >= 4 && wave < 7 ? wave - 4 : 0;  // embedding block (S: 0-2, dB: 4-6)
  const int dim = 32 * fb + (lane0 & 31);                              // the embedding dim of lane j

  f32x16 accA = zero16(), accB = zero16();  // role accumulators
  float bA = 0.f, bB = 0.f;                 // bias sums
  float dB0 = 0.f, dB1 = 0.f, dB2 = 0.f;    // Fourier: dB[c][dim] partial sums
  float wo0 = 0.f, wo1 = 0.f, wo2 = 0.f, bo = 0.f;  // output layer (VALU)
#pragma nounroll
  for (int64_t t = t0; t < t1; ++t) {
    // The LDS addresses are functions of the lane only, i.e. loop-invariant; letting LICM hoist them
    // pins (and spills) the register file.  Re-derive them per tile.
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const int h = lane >> 5, j = lane & 31;
    const float* buf = lds + ((t - t0) & 1) * kBuf;
    [[maybe_unused]] const bool mk = t == t0 + 2;
    CW_PHASE(1, mk);
#if NSLAM_CW_REGSTAGE
    if (t + 1 < t1) fetch(a, t + 1, st, wave, lane);  // flies during this tile
#else
    if (t + 1 < t1) stage(a, t + 1, lds + ((t + 1 - t0) & 1) * kBuf, wave, lane);  // flies during this tile
#endif
    CW_PHASE(2, mk);
    if (wave < 3) {  // the embedding columns of dW_3 and dW_0
      const f32x16 S = lstream(img(buf, kCotS + wave), lane);
      mfma_chain(accA, lstream_masked(buf, 3, lane), S);
      const f32x16 A0 = lstream_masked(buf, 0, lane);
      mfma_chain(accB, A0, S);
      if (wave == 0) bA += sum16(A0);
    } else if (wave != 3 && wave != 7) {
      if (wave == 6) {  // fc_c.2, layer 4
        wblock(accA, bA, lstream(img(buf, 2), lane), lstream(img(buf, kCotC), lane));
        wblock(accB, bB, lstream_masked(buf, 4, lane), lstream(act(buf, 3), lane));
      } else {  // fc_c.(wave - 4), fc_c.(wave - 1): dWc_i = Σ dh_i ⊗ c
        const f32x16 C = lstream(img(buf, kCotC), lane);
        wblock(accA, bA, lstream(img(buf, wave - 4), lane), C);
        wblock(accB, bB, lstream(img(buf, wave - 1), lane), C);
      }
      // dB[c][dim] += Σ_points x_c Gc[point][dim]  (Gc = embedding cotangent ⊙ cos)
      const f32x16 Gc = lstream(img(buf, kCotG + wave - 4), lane);
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(buf + kXgOff + pnt(s, h) * 8);
        dB0 = fmaf(x[0], Gc[s], dB0);
        dB1 = fmaf(x[1], Gc[s], dB1);
        dB2 = fmaf(x[2], Gc[s], dB2);
      }
    } else if (wave == 3) {  // layer 3's h2 columns, layer 2
      wblock(accA, bA, lstream_masked(buf, 3, lane), lstream(act(buf, 2), lane));
      wblock(accB, bB, lstream_masked(buf, 2, lane), lstream(act(buf, 1), lane));
    } else {  // wave 7: layer 1; output layer dWo = g ⊗ h4 (rows 0-2), dbo
      wblock(accA, bA, lstream_masked(buf, 1, lane), lstream(act(buf, 0), lane));
      const f32x16 H4 = lstream(act(buf, 4), lane);
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const f32x4 g = *reinterpret_cast<const f32x4*>(buf + kXgOff + pnt(s, h) * 8 + 4);
        wo0 = fmaf(g[0], H4[s], wo0);
        wo1 = fmaf(g[1], H4[s], wo1);
        wo2 = fmaf(g[2], H4[s], wo2);
        bo += j == 0 ? g[0] : (j == 1 ? g[1] : g[2]);
      }
    }
    CW_PHASE(3, mk);
#if NSLAM_CW_REGSTAGE
    if (t + 1 < t1) commit(lds + ((t + 1 - t0) & 1) * kBuf, st, wave, lane);
#endif
    __syncthreads();  // next buffer landed (the stagers' vmcnt(0) retires their LDS-DMA) / this one free
    CW_PHASE(4, mk);
  }
  CW_PHASE(8, true);

  // write the chunk's slab (each wave its disjoint blocks)
  const int lane = lane0, h = lane >> 5, j = lane & 31;
  float* sl = w.slab + (size_t)chunk * w.acc;
  const int kv = fb < 2 ? 32 : NSLAM_EMB - 64;  // valid embedding columns of block fb
  if (wave < 3) {
    store_block(sl, dg.w[3], 125, 32 * fb, kv, accA, lane);
    store_block(sl, dg.w[0], NSLAM_EMB, 32 * fb, kv, accB, lane);
    if (wave == 0) store_vec(sl, dg.b[0], bA, lane);
  } else if (wave != 3 && wave != 7) {
    if (wave == 6) {
      store_block(sl, dg.wc[2], 32, 0, 32, accA, lane);
      store_vec(sl, dg.bc[2], bA, lane);
      store_block(sl, dg.w[4], 32, 0, 32, accB, lane);
      store_vec(sl, dg.b[4], bB, lane);
    } else {
      store_block(sl, dg.wc[wave - 4], 32, 0, 32, accA, lane);
      store_vec(sl, dg.bc[wave - 4], bA, lane);
      store_block(sl, dg.wc[wave - 1], 32, 0, 32, accB, lane);
      store_vec(sl, dg.bc[wave - 1], bB, lane);
    }
    dB0 += xor32(dB0);
    dB1 += xor32(dB1);
    dB2 += xor32(dB2);
    if (h == 0 && dim < NSLAM_EMB) {
      as_global_w(sl)[dg.B + dim] = dB0;
      as_global_w(sl)[dg.B + NSLAM_EMB + dim] = dB1;
      as_global_w(sl)[dg.B + 2 * NSLAM_EMB + dim] = dB2;
    }
  } else if (wave == 3) {
    store_block(sl, dg.w[3], 125, 93, 32, accA, lane);
    store_vec(sl, dg.b[3], bA, lane);
    store_block(sl, dg.w[2], 32, 0, 32, accB, lane);
    store_vec(sl, dg.b[2], bB, lane);
  } else {
    store_block(sl, dg.w[1], 32, 0, 32, accA, lane);
    store_vec(sl, dg.b[1], bA, lane);
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
  CW_PHASE(9, true);
}

int launch_color_wgrad(const QueryKArgs& a, float* ws, hipStream_t s, const SlabAdam* adam) {
  const nslam_dec_grad& dg = a.c.dgrad[NSLAM_DEC_COLOR];
  const CwPlan pl = cw_plan(dg, a.n);
  CwArgs w{a, ws + pl.cot_bytes / sizeof(float), acc_floats_of(dg), pl.nchunks, pl.chunk_tiles};
  w.a.cot = ws;
  hipLaunchKernelGGL(k_color_wgrad, dim3((unsigned)pl.nchunks), dim3(64 * kCwWaves), 0, s, w);
  const int rc = hip_status();
  return rc ? rc : slab_reduce(dg, w.slab, false, pl.nchunks, 0, w.acc, s, adam);
}

}  // namespace nslamq
