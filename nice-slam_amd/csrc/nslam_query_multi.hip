// nslam_query_multi.hip — ABI v10 nslam_query_bwd_decoders: the mask-only backward of several
// frozen decoders in one launch (k_dec_bwd_multi, nslam_query_impl.h).  Its own translation unit:
// the kernel instantiates every decoder's backward tile.
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
    if (cfg->dgrad[d].base) return NSLAM_EUNSUPPORTED;  // weight gradients: nslam_query_bwd_decoder
    if (cfg->need_pts_grad && n_pts > 0 && !g_pts[d]) return NSLAM_EINVAL;
    m.dec[m.ndec] = d;
    m.gp[m.ndec] = cfg->need_pts_grad ? g_pts[d] : nullptr;
    ++m.ndec;
  }
  if (n_pts > 0 && !cfg->saved_masks) return NSLAM_EUNSUPPORTED;
  if (n_pts == 0) return NSLAM_OK;
  QueryKArgs a{*cfg, pts, n_pts, nullptr, g_raw, nullptr};
  const int64_t groups = ((n_pts + 31) / 32 + kWavesBwd - 1) / kWavesBwd;
  const dim3 grid((unsigned)(groups * m.ndec)), block(64 * kWavesBwd);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (cfg->need_pts_grad)
    hipLaunchKernelGGL(k_dec_bwd_multi<true>, grid, block, 0, s, a, m);
  else
    hipLaunchKernelGGL(k_dec_bwd_multi<false>, grid, block, 0, s, a, m);
  return hip_status();
}
