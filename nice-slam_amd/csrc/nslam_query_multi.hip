// nslam_query_multi.hip — ABI v10 nslam_query_bwd_decoders: the backward of several decoders in one
// launch (k_dec_bwd_multi, nslam_query_impl.h).  Its own translation unit: the kernel instantiates
// every decoder's backward tile.
#include "nslam_query_impl.h"

using namespace nslamq;

extern "C" int nslam_query_bwd_decoders(const nslam_query_cfg* cfg, int32_t dec_mask, const double* pts,
                                        int64_t n_pts, const float* g_raw, double* const* g_pts, void* ws,
                                        size_t ws_bytes, void* stream) {
  const int rc = check_cfg(cfg, true);
  if (rc) return rc;
  const bool sum_pts = (dec_mask & NSLAM_BWD_SUM_PTS) != 0;
  const bool defer = (dec_mask & NSLAM_BWD_DEFER_WGRAD) != 0;
  dec_mask &= ~(NSLAM_BWD_SUM_PTS | NSLAM_BWD_DEFER_WGRAD);
  if (dec_mask <= 0 || dec_mask > 15) return NSLAM_EINVAL;
  if (sum_pts && (!cfg->need_pts_grad || (n_pts > 0 && (!g_pts || !g_pts[0])))) return NSLAM_EINVAL;
  if (n_pts < 0 || (n_pts > 0 && ((!pts && !cfg->rays_o) || !g_raw))) return NSLAM_EINVAL;
  if (cfg->rays_o && (n_pts >= (int64_t(1) << 31) || n_pts % cfg->n_samples)) return NSLAM_EINVAL;
  if (cfg->need_pts_grad && n_pts > 0 && !g_pts) return NSLAM_EINVAL;
  MultiDecArgs m{};
  bool cw = false;  // the colour decoder's weight gradients are part of the call
  for (int d = 0; d < 4; ++d) {
    if (!((dec_mask >> d) & 1)) continue;
    if (!stage_uses(cfg->stage, d)) return NSLAM_EINVAL;
    if (cfg->dgrad[d].base) {
      // only the colour decoder's tape backward joins a merged launch (as its lean chain + k_color_wgrad)
      if (d != NSLAM_DEC_COLOR || cfg->need_pts_grad || !cfg->act_tape || cfg->dgrad[d].count <= 0)
        return NSLAM_EUNSUPPORTED;
      cw = true;
    }
    if (cfg->need_pts_grad && n_pts > 0 && !sum_pts && !g_pts[d]) return NSLAM_EINVAL;
    m.dec[m.ndec] = d;
    m.gp[m.ndec] = cfg->need_pts_grad && !sum_pts ? g_pts[d] : nullptr;
    ++m.ndec;
  }
  if (defer && !cw) return NSLAM_EINVAL;
  if (n_pts > 0 && !cfg->saved_masks) return NSLAM_EUNSUPPORTED;
  if (n_pts == 0) return NSLAM_OK;
  const int64_t tiles = (n_pts + 31) / 32;
  const int64_t groups = (tiles + kWavesBwd - 1) / kWavesBwd;
  if (cw) {
    const size_t need = dec_ws_bytes(cfg, NSLAM_DEC_COLOR, n_pts);
    if (!ws || ws_bytes < need) return NSLAM_EWORKSPACE;
  }
  QueryKArgs a{*cfg, pts, n_pts, nullptr, g_raw, nullptr};
  a.defer_wgrad = defer;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // the colour decoder alone (its lean chain + weight gradients): its own kernel, which has the
  // lean kernels' registers (the multi-decoder kernel with the tape path takes ~170)
  if (cw && m.ndec == 1) return dispatch_dec_bwd<NSLAM_DEC_COLOR>(a, true, reinterpret_cast<float*>(ws), s);
  if (sum_pts) {  // one workgroup per tile, one wave per decoder, d/dpts summed in decoder order
    if (cw) return NSLAM_EUNSUPPORTED;
    hipLaunchKernelGGL(k_dec_bwd_multi_sum<>, dim3((unsigned)tiles), dim3(64 * m.ndec), 0, s, a, m, g_pts[0]);
    return hip_status();
  }
  const dim3 grid((unsigned)(groups * m.ndec)), block(64 * kWavesBwd);
  if (cw) a.cot = reinterpret_cast<float*>(ws);  // the colour part stores its cotangent tape
  if (cfg->need_pts_grad)  // (a tape backward has no d/dpts)
    hipLaunchKernelGGL((k_dec_bwd_multi<true, false>), grid, block, 0, s, a, m);
  else if (cw)
    hipLaunchKernelGGL((k_dec_bwd_multi<false, true>), grid, block, 0, s, a, m);
  else
    hipLaunchKernelGGL((k_dec_bwd_multi<false, false>), grid, block, 0, s, a, m);
  const int lrc = hip_status();
  if (lrc || !cw || defer) return lrc;
  return launch_color_wgrad(a, reinterpret_cast<float*>(ws), s);
}

// ABI v11: the colour decoder's weight gradients of a tape backward whose lean chain ran earlier
// (nslam_query_bwd_decoders with NSLAM_BWD_DEFER_WGRAD) and left its cotangent tape in ws.
extern "C" int nslam_color_wgrad(const nslam_query_cfg* cfg, int64_t n_pts, void* ws, size_t ws_bytes, void* stream) {
  const int rc = check_cfg(cfg, true);
  if (rc) return rc;
  if (cfg->stage != NSLAM_STAGE_COLOR || n_pts < 0) return NSLAM_EINVAL;
  if (!cfg->dgrad[NSLAM_DEC_COLOR].base || cfg->dgrad[NSLAM_DEC_COLOR].count <= 0 || cfg->need_pts_grad)
    return NSLAM_EUNSUPPORTED;
  if (n_pts > 0 && !cw_tape_path(cfg)) return NSLAM_EUNSUPPORTED;
  if (n_pts == 0) return NSLAM_OK;
  if (!ws || ws_bytes < dec_ws_bytes(cfg, NSLAM_DEC_COLOR, n_pts)) return NSLAM_EWORKSPACE;
  QueryKArgs a{*cfg, nullptr, n_pts, nullptr, nullptr, nullptr};
  return launch_color_wgrad(a, reinterpret_cast<float*>(ws), reinterpret_cast<hipStream_t>(stream));
}

// ABI v12/v14: nslam_color_wgrad, then the Adam step of the colour decoder (segs[0]: its dense
// segment, grad == cfg->dgrad[COLOR].base) and of up to kSlabAdamExtra further segments (segs[1..]:
// e.g. the colour grid's frustum rows) inside the slab-reduction launch — one launch fewer on the
// mapping iteration's critical path.  The same element update as nslam_adam_step.
extern "C" int nslam_color_wgrad_adam(const nslam_query_cfg* cfg, int64_t n_pts, void* ws, size_t ws_bytes,
                                      const nslam_adam_seg* segs, int32_t n_segs, float beta1, float beta2,
                                      float eps, int32_t zero_grad, uint32_t* ticket, void* stream) {
  const int rc = check_cfg(cfg, true);
  if (rc) return rc;
  if (cfg->stage != NSLAM_STAGE_COLOR || n_pts < 0 || !segs || n_segs < 1 || n_segs > 1 + kSlabAdamExtra || !ticket)
    return NSLAM_EINVAL;
  const nslam_dec_grad& dg = cfg->dgrad[NSLAM_DEC_COLOR];
  if (!dg.base || dg.count <= 0 || cfg->need_pts_grad) return NSLAM_EUNSUPPORTED;
  const nslam_adam_seg& seg = segs[0];
  if (seg.rows || seg.grad != dg.base || seg.n != dg.count || !seg.step || !seg.param || !seg.exp_avg ||
      !seg.exp_avg_sq || (seg.mirror && !seg.mirror_idx))
    return NSLAM_EINVAL;
  SlabAdam ad{};
  ad.seg = seg;
  ad.b1 = beta1;
  ad.b2 = beta2;
  ad.eps = eps;
  ad.zero_grad = zero_grad;
  ad.ticket = ticket;
  ad.on = 1;
  ad.n_extra = n_segs - 1;
  for (int k = 1; k < n_segs; ++k) {  // nslam_adam_step's checks
    const nslam_adam_seg& g = segs[k];
    if (g.n <= 0 || !g.step || !g.param || !g.grad || !g.exp_avg || !g.exp_avg_sq) return NSLAM_EINVAL;
    if (g.rows) {
      if (g.row_len <= 0 || g.row_len % 4 || g.row_len / 4 > 64 * kReduceWaves) return NSLAM_EINVAL;
      const uintptr_t al = (uintptr_t)g.param | (uintptr_t)g.grad | (uintptr_t)g.exp_avg | (uintptr_t)g.exp_avg_sq;
      if (al & 15) return NSLAM_EINVAL;
    }
    ad.extra[k - 1] = g;
  }
  if (n_pts == 0) return NSLAM_OK;  // (nothing to reduce: like a segment without a gradient, no step)
  if (!cw_tape_path(cfg)) return NSLAM_EUNSUPPORTED;
  if (!ws || ws_bytes < dec_ws_bytes(cfg, NSLAM_DEC_COLOR, n_pts)) return NSLAM_EWORKSPACE;
  QueryKArgs a{*cfg, nullptr, n_pts, nullptr, nullptr, nullptr};
  return launch_color_wgrad(a, reinterpret_cast<float*>(ws), reinterpret_cast<hipStream_t>(stream), &ad);
}
