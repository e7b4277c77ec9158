// nslam_query_multi.hip — ABI v10 nslam_query_bwd_decoders (the mask-only backward of several decoders
// in one launch, k_dec_bwd_multi in nslam_query_impl.h) and ABI v16 nslam_color_wgrad (the colour
// decoder's parameter gradients, k_color_wgrad in nslam_color_wgrad.hip).  Its own translation unit:
// the multi-decoder kernel instantiates every decoder's backward tile.
#include "nslam_query_impl.h"

using namespace nslamq;

extern "C" int nslam_query_bwd_decoders(const nslam_query_cfg* cfg, int32_t dec_mask, const double* pts,
                                        int64_t n_pts, const float* g_raw, double* const* g_pts, void* stream) {
  const int rc = check_cfg(cfg, true);
  if (rc) return rc;
  if (dec_mask <= 0 || dec_mask > 15) return NSLAM_EINVAL;
  if (n_pts < 0 || (n_pts > 0 && ((!pts && !cfg->rays_o) || !g_raw))) return NSLAM_EINVAL;
  if (cfg->rays_o && (n_pts >= (int64_t(1) << 31) || n_pts % cfg->n_samples)) return NSLAM_EINVAL;
  if (cfg->need_pts_grad && n_pts > 0 && !g_pts) return NSLAM_EINVAL;
  MultiDecArgs m{};
  for (int d = 0; d < 4; ++d) {
    if (!((dec_mask >> d) & 1)) continue;
    if (!stage_uses(cfg->stage, d)) return NSLAM_EINVAL;
    // parameter gradients are not formed here (the colour decoder's: nslam_color_wgrad)
    if (cfg->dgrad[d].base) return NSLAM_EUNSUPPORTED;
    if (cfg->need_pts_grad && n_pts > 0 && !g_pts[d]) return NSLAM_EINVAL;
    m.dec[m.ndec] = d;
    m.gp[m.ndec] = cfg->need_pts_grad ? g_pts[d] : nullptr;
    ++m.ndec;
  }
  if (n_pts > 0 && !cfg->saved_masks) return NSLAM_EUNSUPPORTED;
  if (n_pts == 0) return NSLAM_OK;
  const int64_t tiles = (n_pts + 31) / 32;
  const int64_t groups = (tiles + kWavesBwd - 1) / kWavesBwd;
  QueryKArgs a{*cfg, pts, n_pts, nullptr, g_raw, nullptr};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)(groups * m.ndec)), block(64 * kWavesBwd);
  if (cfg->need_pts_grad)
    hipLaunchKernelGGL((k_dec_bwd_multi<true>), grid, block, 0, s, a, m);
  else
    hipLaunchKernelGGL((k_dec_bwd_multi<false>), grid, block, 0, s, a, m);
  return hip_status();
}

// ABI v16: the colour decoder's parameter gradients of a colour-stage backward, from the forward's
// activation tape and ReLU masks and the cotangent g_raw — independent of the lean backward that
// forms the colour grid's gradient (nslam_query_bwd_decoders), so the two may run concurrently.
extern "C" int nslam_color_wgrad(const nslam_query_cfg* cfg, const double* pts, int64_t n_pts, const float* g_raw,
                                 void* ws, size_t ws_bytes, void* stream) {
  const int rc = check_cfg(cfg, true);
  if (rc) return rc;
  if (cfg->stage != NSLAM_STAGE_COLOR || n_pts < 0) return NSLAM_EINVAL;
  if (!cfg->dgrad[NSLAM_DEC_COLOR].base || cfg->dgrad[NSLAM_DEC_COLOR].count <= 0) return NSLAM_EUNSUPPORTED;
  if (n_pts > 0 && !cw_tape_path(cfg)) return NSLAM_EUNSUPPORTED;
  if (n_pts > 0 && ((!pts && !cfg->rays_o) || !g_raw)) return NSLAM_EINVAL;
  if (cfg->rays_o && (n_pts >= (int64_t(1) << 31) || n_pts % cfg->n_samples)) return NSLAM_EINVAL;
  if (n_pts == 0) return NSLAM_OK;
  if (!ws || ws_bytes < dec_ws_bytes(cfg, NSLAM_DEC_COLOR, n_pts)) return NSLAM_EWORKSPACE;
  QueryKArgs a{*cfg, pts, n_pts, nullptr, g_raw, nullptr};
  return launch_color_wgrad(a, reinterpret_cast<float*>(ws), reinterpret_cast<hipStream_t>(stream));
}
