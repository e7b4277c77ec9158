// nslam_query.hip — C-ABI entry points of the fused point query (include/nslam.h): forward
// launches, backward dispatch (the per-decoder backward launchers are compiled in
// nslam_query_dec.hip), workspace / tape / mask sizes and the pack layout.
#include <string.h>

#include "nslam_query_impl.h"

using namespace nslamq;

extern "C" int nslam_query_fwd(const nslam_query_cfg* cfg, const double* pts, int64_t n_pts, float* raw,
                               void* stream) {
  const int rc = check_cfg(cfg, false);
  if (rc) return rc;
  if (n_pts < 0 || (n_pts > 0 && ((!pts && !cfg->rays_o) || !raw))) return NSLAM_EINVAL;
  if (cfg->rays_o && (n_pts >= (int64_t(1) << 31) || n_pts % cfg->n_samples)) return NSLAM_EINVAL;
  if (n_pts == 0) return NSLAM_OK;
  QueryKArgs a{*cfg, pts, n_pts, raw, nullptr, nullptr};
  const int64_t tiles = (n_pts + 31) / 32;
  const dim3 grid((unsigned)((tiles + 3) / 4)), block(256);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (cfg->stage) {
    case NSLAM_STAGE_COARSE: hipLaunchKernelGGL(k_query_fwd<NSLAM_STAGE_COARSE>, grid, block, 0, s, a); break;
    case NSLAM_STAGE_MIDDLE: hipLaunchKernelGGL(k_query_fwd<NSLAM_STAGE_MIDDLE>, grid, block, 0, s, a); break;
    case NSLAM_STAGE_FINE: hipLaunchKernelGGL(k_query_fwd<NSLAM_STAGE_FINE>, grid, block, 0, s, a); break;
    default: hipLaunchKernelGGL(k_query_fwd<NSLAM_STAGE_COLOR>, grid, block, 0, s, a); break;
  }
  return hip_status();
}

extern "C" size_t nslam_query_fwd_workspace_size(const nslam_query_cfg* cfg, int64_t n_pts) {
  if (!cfg || n_pts <= 0 || cfg->stage < NSLAM_STAGE_FINE || cfg->stage > NSLAM_STAGE_COLOR) return 0;
  return (((size_t)n_pts * sizeof(float) + 255) & ~(size_t)255) + 256;  // + the dynamic forward's counter
}

extern "C" int nslam_query_fwd_ws(const nslam_query_cfg* cfg, const double* pts, int64_t n_pts, float* raw, void* ws,
                                  size_t ws_bytes, void* stream) {
  const size_t need = nslam_query_fwd_workspace_size(cfg, n_pts);
  if (need == 0) return nslam_query_fwd(cfg, pts, n_pts, raw, stream);  // coarse / middle: one decoder
  const int rc = check_cfg(cfg, false);
  if (rc) return rc;
  if (!ws || ws_bytes < need) return NSLAM_EWORKSPACE;
  if ((!pts && !cfg->rays_o) || !raw || (((uintptr_t)raw) & 15)) return NSLAM_EINVAL;
  if (cfg->rays_o && (n_pts >= (int64_t(1) << 31) || n_pts % cfg->n_samples)) return NSLAM_EINVAL;
  QueryKArgs a{*cfg, pts, n_pts, raw, nullptr, nullptr};
  const int64_t groups = ((n_pts + 31) / 32 + 3) / 4;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* occ = reinterpret_cast<float*>(ws);
  // Colour stage: 3 parts (middle | fine | colour) while 3 waves per tile fit the chip's wave slots
  // in one round (3 per SIMD at the forward's 168 VGPRs; e.g. tracking, 300 tiles), else 2 parts
  // (middle then colour | fine: fewer, balanced waves — room0 mapping: 3000 instead of 4500 for
  // 4096 slots, 187 -> 198 M ray-samples/s).  NSLAM_FWD_PARTS=2|3 forces one (experiments).
  static const int forced_parts = [] {
    const char* e = getenv("NSLAM_FWD_PARTS");
    return e ? atoi(e) : 0;
  }();
  static const int64_t n_cus = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    return (int64_t)cus;
  }();
  const int64_t wave_slots = n_cus * 4 * 3;
  const int64_t tiles = (n_pts + 31) / 32;
  const int color_parts = forced_parts == 2 || forced_parts == 3 ? forced_parts : (3 * tiles <= wave_slots ? 3 : 2);
  const dim3 b256(256);
  // forward variant: cfg->fwd_variant, else NSLAM_FWD_MODE=pc (producer / consumer waves, one persistent
  // workgroup per CU), units (one-wave workgroups per decoder-tile), dyn (a counter; experiment), parts
  // (an unrecognised NSLAM_FWD_MODE is an error, not a silent fallback: a typo must not change the kernel)
  static const int env_mode = [] {
    const char* e = getenv("NSLAM_FWD_MODE");
    if (!e || !*e || !strcmp(e, "units")) return 1;
    return !strcmp(e, "pc") ? 3 : !strcmp(e, "dyn") ? 2 : !strcmp(e, "parts") ? 0 : -1;
  }();
  if (cfg->fwd_variant < 0 || cfg->fwd_variant > NSLAM_FWD_PARTS) return NSLAM_EINVAL;
  if (cfg->fwd_variant == NSLAM_FWD_DEFAULT && env_mode < 0) return NSLAM_EINVAL;
  const int mode = cfg->fwd_variant == NSLAM_FWD_UNITS ? 1
                   : cfg->fwd_variant == NSLAM_FWD_PC  ? 3
                   : cfg->fwd_variant == NSLAM_FWD_PARTS ? 0
                                                         : env_mode;
  if (mode == 3) {
    const int64_t units = tiles * (cfg->stage == NSLAM_STAGE_COLOR ? 3 : 2);
    const dim3 g((unsigned)(units < n_cus ? units : n_cus)), b(64 * kPcWaves);
    if (cfg->stage == NSLAM_STAGE_FINE)
      hipLaunchKernelGGL((k_query_fwd_pc<NSLAM_STAGE_FINE, false>), g, b, 0, s, a, occ);
    else if (cfg->act_tape)
      hipLaunchKernelGGL((k_query_fwd_pc<NSLAM_STAGE_COLOR, true>), g, b, 0, s, a, occ);
    else
      hipLaunchKernelGGL((k_query_fwd_pc<NSLAM_STAGE_COLOR, false>), g, b, 0, s, a, occ);
  } else if (mode == 1) {
    const int np = cfg->stage == NSLAM_STAGE_COLOR ? 3 : 2;
    const dim3 g((unsigned)(tiles * np)), b64(64);
    if (cfg->stage == NSLAM_STAGE_FINE)
      hipLaunchKernelGGL((k_query_fwd_units<NSLAM_STAGE_FINE, false>), g, b64, 0, s, a, occ);
    else if (cfg->act_tape)
      hipLaunchKernelGGL((k_query_fwd_units<NSLAM_STAGE_COLOR, true>), g, b64, 0, s, a, occ);
    else
      hipLaunchKernelGGL((k_query_fwd_units<NSLAM_STAGE_COLOR, false>), g, b64, 0, s, a, occ);
  } else if (mode == 2) {
    const int np = cfg->stage == NSLAM_STAGE_COLOR ? 3 : 2;
    unsigned* ctr = reinterpret_cast<unsigned*>(static_cast<char*>(ws) + (need - 256));
    if (hipMemsetAsync(ctr, 0, 8, s) != hipSuccess) return hip_status();
    const int64_t waves = tiles * np < wave_slots ? tiles * np : wave_slots;
    const dim3 g((unsigned)((waves + 3) / 4));
    if (cfg->stage == NSLAM_STAGE_FINE)
      hipLaunchKernelGGL((k_query_fwd_dyn<NSLAM_STAGE_FINE, false>), g, b256, 0, s, a, occ, ctr);
    else if (cfg->act_tape)
      hipLaunchKernelGGL((k_query_fwd_dyn<NSLAM_STAGE_COLOR, true>), g, b256, 0, s, a, occ, ctr);
    else
      hipLaunchKernelGGL((k_query_fwd_dyn<NSLAM_STAGE_COLOR, false>), g, b256, 0, s, a, occ, ctr);
  } else if (cfg->stage == NSLAM_STAGE_FINE)
    hipLaunchKernelGGL((k_query_fwd_parts<NSLAM_STAGE_FINE, 2, false>), dim3((unsigned)(groups * 2)), b256, 0, s, a,
                       occ);
  else if (color_parts == 2 && cfg->act_tape)
    hipLaunchKernelGGL((k_query_fwd_parts<NSLAM_STAGE_COLOR, 2, true>), dim3((unsigned)(groups * 2)), b256, 0, s, a,
                       occ);
  else if (color_parts == 2)
    hipLaunchKernelGGL((k_query_fwd_parts<NSLAM_STAGE_COLOR, 2, false>), dim3((unsigned)(groups * 2)), b256, 0, s, a,
                       occ);
  else if (cfg->act_tape)
    hipLaunchKernelGGL((k_query_fwd_parts<NSLAM_STAGE_COLOR, 3, true>), dim3((unsigned)(groups * 3)), b256, 0, s, a,
                       occ);
  else
    hipLaunchKernelGGL((k_query_fwd_parts<NSLAM_STAGE_COLOR, 3, false>), dim3((unsigned)(groups * 3)), b256, 0, s, a,
                       occ);
  if (!cfg->defer_occ)  // else the consumer adds ws on read (nslam_loss_cfg.occ_add)
    hipLaunchKernelGGL(k_occ_combine, dim3((unsigned)((n_pts + 255) / 256)), dim3(256), 0, s, raw, occ, n_pts);
  return hip_status();
}


extern "C" int nslam_query_bwd_decoder(const nslam_query_cfg* cfg, int32_t dec, int32_t accumulate_pts,
                                       const double* pts, int64_t n_pts, const float* g_raw, double* g_pts, void* ws,
                                       size_t ws_bytes, void* stream) {
  const int rc = check_cfg(cfg, true);
  if (rc) return rc;
  if (dec < 0 || dec > 3 || !stage_uses(cfg->stage, dec)) return NSLAM_EINVAL;
  if (n_pts < 0 || (n_pts > 0 && ((!pts && !cfg->rays_o) || !g_raw))) return NSLAM_EINVAL;
  if (cfg->rays_o && (n_pts >= (int64_t(1) << 31) || n_pts % cfg->n_samples)) return NSLAM_EINVAL;
  if (cfg->need_pts_grad && n_pts > 0 && !g_pts) return NSLAM_EINVAL;
  if (n_pts == 0) return NSLAM_OK;
  if (cfg->dgrad[dec].base && cfg->dgrad[dec].count <= 0) return NSLAM_EUNSUPPORTED;
  const size_t need = dec_ws_bytes(cfg, dec, n_pts);
  if (ws_bytes < need || (need > 0 && !ws)) return NSLAM_EWORKSPACE;
  QueryKArgs a{*cfg, pts, n_pts, nullptr, g_raw, g_pts};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* slab = reinterpret_cast<float*>(ws);
  const bool first = !accumulate_pts;
  switch (dec) {
    case NSLAM_DEC_COARSE: return dispatch_dec_bwd<NSLAM_DEC_COARSE>(a, first, slab, s);
    case NSLAM_DEC_MIDDLE: return dispatch_dec_bwd<NSLAM_DEC_MIDDLE>(a, first, slab, s);
    case NSLAM_DEC_FINE: return dispatch_dec_bwd<NSLAM_DEC_FINE>(a, first, slab, s);
    default: return dispatch_dec_bwd<NSLAM_DEC_COLOR>(a, first, slab, s);
  }
}

extern "C" size_t nslam_query_bwd_decoder_workspace_size(const nslam_query_cfg* cfg, int32_t dec, int64_t n_pts) {
  if (!cfg || dec < 0 || dec > 3 || n_pts <= 0) return 0;
  return dec_ws_bytes(cfg, dec, n_pts);
}

extern "C" size_t nslam_query_tape_size(int64_t n_pts) {
  if (n_pts <= 0) return 0;
  return (size_t)((n_pts + 31) / 32) * kTapeFloats * sizeof(float);
}

extern "C" size_t nslam_query_saved_size(int64_t n_pts) {
  if (n_pts <= 0) return 0;
  return (size_t)4 * ((n_pts + 31) / 32) * 5 * 64 * sizeof(uint16_t);
}

extern "C" size_t nslam_query_bwd_workspace_size(const nslam_query_cfg* cfg, int64_t n_pts) {
  if (!cfg || n_pts <= 0) return 0;
  return bwd_ws_bytes(cfg, n_pts);
}

extern "C" int nslam_query_bwd(const nslam_query_cfg* cfg, const double* pts, int64_t n_pts, const float* g_raw,
                               double* g_pts, void* ws, size_t ws_bytes, void* stream) {
  const int rc = check_cfg(cfg, true);
  if (rc) return rc;
  if (n_pts < 0 || (n_pts > 0 && ((!pts && !cfg->rays_o) || !g_raw))) return NSLAM_EINVAL;
  if (cfg->rays_o && (n_pts >= (int64_t(1) << 31) || n_pts % cfg->n_samples)) return NSLAM_EINVAL;
  if (cfg->need_pts_grad && n_pts > 0 && !g_pts) return NSLAM_EINVAL;
  if (n_pts == 0) return NSLAM_OK;
  for (int d = 0; d < 4; ++d)
    if (cfg->dgrad[d].base && cfg->dgrad[d].count <= 0)
      return NSLAM_EUNSUPPORTED;
  if (ws_bytes < bwd_ws_bytes(cfg, n_pts) || (bwd_ws_bytes(cfg, n_pts) > 0 && !ws)) return NSLAM_EWORKSPACE;
  QueryKArgs a{*cfg, pts, n_pts, nullptr, g_raw, g_pts};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* slab = reinterpret_cast<float*>(ws);
  int r = NSLAM_OK;
  switch (cfg->stage) {
    case NSLAM_STAGE_COARSE:
      r = dispatch_dec_bwd<NSLAM_DEC_COARSE>(a, true, slab, s);
      break;
    case NSLAM_STAGE_MIDDLE:
      r = dispatch_dec_bwd<NSLAM_DEC_MIDDLE>(a, true, slab, s);
      break;
    case NSLAM_STAGE_FINE:
      r = dispatch_dec_bwd<NSLAM_DEC_MIDDLE>(a, true, slab, s);
      if (!r) r = dispatch_dec_bwd<NSLAM_DEC_FINE>(a, false, slab, s);
      break;
    default:
      r = dispatch_dec_bwd<NSLAM_DEC_MIDDLE>(a, true, slab, s);
      if (!r) r = dispatch_dec_bwd<NSLAM_DEC_FINE>(a, false, slab, s);
      if (!r) r = dispatch_dec_bwd<NSLAM_DEC_COLOR>(a, false, slab, s);
      break;
  }
  return r;
}

extern "C" int nslam_pack_layout(int kind, int nc, int32_t* out, int n) {
  if (!out || n < 4) return NSLAM_EINVAL;
  if (kind == 0) {
    if (nc != 1 && nc != 2) return NSLAM_EINVAL;
    const XyzPack L{nc};
    out[0] = L.total();
    out[1] = L.V();
    out[2] = L.nf();
    out[3] = L.nfrag() - L.nf();
  } else if (kind == 1) {
    const NoXyzPack L;
    out[0] = L.total();
    out[1] = L.V();
    out[2] = L.nf();
    out[3] = L.nfrag() - L.nf();
  } else {
    return NSLAM_EINVAL;
  }
  return 4;
}

#ifdef NSLAM_PHASES
extern "C" int nslam_debug_phases(unsigned long long* out, int64_t n) {
  if (n > (int64_t)5 * kPhaseWaves * 16) n = (int64_t)5 * kPhaseWaves * 16;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
#if defined(NSLAM_PHASES) || defined(NSLAM_TIMELINE)
// per-wave timeline {start, end, HW_ID | XCC_ID << 32, tag} of slots 0 forward, 1 mask-only bwd, 2 wgrad
extern "C" int nslam_debug_timeline(unsigned long long* out, int64_t n) {
  if (n > (int64_t)3 * kTlWaves * 4) n = (int64_t)3 * kTlWaves * 4;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tl), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
