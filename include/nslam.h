/*
 * nslam.h — C-ABI of libnslam.so, the MI355X (gfx950) hot path of NICE-SLAM's volumetric renderer.
 *
 * The reference (LongruiDong/nice-slam) is pure PyTorch; it has no native/FFI boundary.  Each
 * entry point below replaces a specific piece of the reference's Python hot path (file:line are
 * relative to the reference checkout), and is bound from Python by ctypes in
 * nice-slam_amd/_lib.py (see INTEGRATION.md for the binding a maintainer would add).
 *
 * Contract (all entry points):
 *   - every pointer is a DEVICE pointer owned by the caller (PyTorch caching allocator);
 *   - work is enqueued on `stream` (a hipStream_t passed as void*); nothing synchronises;
 *   - no globals, no persistent allocations: re-entrant across threads/processes (the reference
 *     runs tracker, mapper and coarse mapper concurrently on one GPU, src/NICE_SLAM.py:288-307);
 *   - return 0 on success, a negative NSLAM_E* code on bad arguments, or NSLAM_EHIP - hipError
 *     when a launch fails.  nslam_strerror() maps codes to text.
 *
 * Grid layout: a feature grid is the reference's [1, C=32, Z, Y, X] float32 tensor stored
 * channels-last, i.e. physically [Z][Y][X][32] (torch.channels_last_3d); one trilinear corner
 * is one 128-byte row.
 */
#ifndef NSLAM_H
#define NSLAM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NSLAM_C_DIM 32
#define NSLAM_HIDDEN 32
#define NSLAM_EMB 93

enum {
  NSLAM_OK = 0,
  NSLAM_EINVAL = -1,       /* bad pointer / size / enum */
  NSLAM_EUNSUPPORTED = -2, /* configuration outside the NICE-SLAM path (e.g. S > 256) */
  NSLAM_EWORKSPACE = -3,   /* workspace too small */
  NSLAM_EHIP = -1000       /* NSLAM_EHIP - hipError_t */
};

enum { NSLAM_STAGE_COARSE = 0, NSLAM_STAGE_MIDDLE = 1, NSLAM_STAGE_FINE = 2, NSLAM_STAGE_COLOR = 3 };
enum { NSLAM_DEC_COARSE = 0, NSLAM_DEC_MIDDLE = 1, NSLAM_DEC_FINE = 2, NSLAM_DEC_COLOR = 3 };
/* nslam_query_cfg.fwd_variant (ABI v18): UNITS = one one-wave workgroup per decoder and 32-point tile;
 * PC = one persistent workgroup per CU whose producer waves gather and embed while its consumer waves
 * run the decoder GEMM chains; PARTS = 4-wave workgroups of one decoder part. */
enum { NSLAM_FWD_DEFAULT = 0, NSLAM_FWD_UNITS = 1, NSLAM_FWD_PC = 2, NSLAM_FWD_PARTS = 3 };

/* One feature grid (src/NICE_SLAM.py:192-250) with the bound it is normalised against
 * (decoder.bound, src/NICE_SLAM.py:152-157; the coarse decoder uses bound*2). */
typedef struct nslam_grid {
  const float* data; /* channels-last [Z][Y][X][32]; NULL when the stage does not read it */
  float* grad;       /* same layout, accumulated with atomics; NULL = no grid gradient      */
  int32_t dims[3];   /* Z, Y, X (= D, H, W of F.grid_sample)                                 */
  int32_t pad_;
  double lo[3];      /* x, y, z lower bound (float64, as the reference)                      */
  double hi[3];      /* x, y, z upper bound                                                  */
  /* ABI v6, frustum-compacted gradient: slot == NULL -> `grad` is a dense grid like `data`; else
   * `grad` is [n_rows][32] for the frustum-selected voxels (Mapper.py:314-333) and slot[Z*Y*X]
   * maps a voxel row to its compact row (-1: not selected, its gradient is not formed — the
   * reference optimises only the masked vector, Mapper.py:394-401). */
  const int32_t* slot;
} nslam_grid;

/* Where a decoder's parameter gradients go: `base` is a flat float32 buffer and the offsets are
 * element offsets of each parameter in it (natural row-major [out][in] layout, i.e. the layout
 * of nn.Linear.weight).  base == NULL: no parameter gradients for this decoder. */
typedef struct nslam_dec_grad {
  float* base;
  int64_t w[5], b[5];   /* pts_linears.i.weight / .bias                       */
  int64_t wc[5], bc[5]; /* fc_c.i.weight / .bias (unused for the coarse MLP)  */
  int64_t wo, bo;       /* output_linear.weight / .bias                       */
  int64_t B;            /* embedder._B [3][93] (unused for the coarse MLP)    */
  int64_t count;        /* floats in the flat buffer (all parameters)         */
} nslam_dec_grad;

/* Point query: NICE.forward + Renderer.eval_points
 * (src/conv_onet/models/decoder.py:168-342, src/utils/Renderer.py:23-61). */
typedef struct nslam_query_cfg {
  int32_t stage;            /* NSLAM_STAGE_*                                             */
  int32_t need_pts_grad;    /* backward: write d loss / d pts                             */
  double bound_lo[3];       /* OOB test bound (strict <, >), Renderer.py:43-46            */
  double bound_hi[3];
  nslam_grid grid[4];       /* indexed by NSLAM_DEC_*                                     */
  const float* packed[4];   /* packed decoder weights (nslam_pack_layout), NULL if unused */
  nslam_dec_grad dgrad[4];  /* parameter-gradient destinations                            */
  /* Ray form of the point list (ABI v4): when rays_o != NULL the points are generated in-kernel
   * as pts[r*S + s] = rays_o[r] + rays_d[r] * z_vals[r][s] in float64 (Renderer.py:172-174,
   * float32 rays promoted) and the `pts` argument is ignored.  The backward's g_pts (ABI v5: also
   * in ray form) is d loss / d pts per generated point, [M][3] float64. */
  const float* rays_o;      /* [M/S][3] float32 */
  const float* rays_d;      /* [M/S][3] float32 */
  const double* z_vals;     /* [M/S][S] float64 */
  int64_t n_samples;        /* S */
  /* ReLU masks saved by the forward (ABI v4; NULL = none): nslam_query_fwd writes every
   * evaluated decoder's masks here and nslam_query_bwd then skips the forward recompute of the
   * decoders that have no parameter gradients (their backward needs only the masks).
   * nslam_query_saved_size(M) bytes; layout [decoder][tile of 32 points][layer 0..4][64] uint16. */
  uint16_t* saved_masks;
  /* ABI v7: nslam_query_fwd_ws with defer_occ = 1 leaves raw[...,3] = the fine occupancy and the
   * middle occupancy in ws (float [M]) instead of adding them in a separate pass: the consumer
   * adds it on read (nslam_loss_cfg.occ_add = ws), saving a launch per query. */
  int32_t defer_occ;
  /* ABI v18: how nslam_query_fwd_ws spreads the fine / colour stage over the chip (NSLAM_FWD_*; 0 = the
   * library's default).  Every variant computes the same values in the same order: bit-identical
   * outputs, masks and activation tape. */
  int32_t fwd_variant;
  /* ABI v9: activation tape of the colour decoder (NULL = none).  nslam_query_fwd[_ws] writes the
   * post-ReLU hidden tiles h0..h4 of every 32-point tile ([tile][layer][32 points][32 features]
   * float, nslam_query_tape_size(M) bytes; layout private to the library); with it and saved_masks the colour decoder's weight-gradient
   * backward reads them instead of recomputing its forward (Mapper.py:503). */
  float* act_tape;
  /* ABI v17: cotangent of the colour decoder's last hidden layer h4, [M][32] float32, 16-byte aligned
   * (else NSLAM_EINVAL; NULL = none),
   * added to its output layer's Woᵀg in every backward of the colour decoder.  A direct caller of
   * MLP(color=True) (decoder.py:154-159,198-203) forms the 4th output row h4·Wo[3] + bo[3] itself
   * (NICE.forward overwrites that row, decoder.py:341) and passes d/dh4 here. */
  const float* g_h4;
} nslam_query_cfg;

/* ---- packing ------------------------------------------------------------------------------
 * Decoder weights are re-laid-out into MFMA fragment order by the caller (a gather with the
 * index map described here).  kind 0 = MLP with Fourier embedding and `nc` feature blocks
 * (middle/color nc=1, fine nc=2); kind 1 = MLP_no_xyz (coarse).  Writes up to `n` int32 values:
 *   out[0] = total packed floats, out[1] = offset of the vector section, out[2] = fwd frag count,
 *   out[3] = bwd frag count.  Returns the number of values written or <0. */
int nslam_pack_layout(int kind, int nc, int32_t* out, int n);

/* ---- sampler: src/utils/Renderer.py:82-174 (perturb=0, N_importance=0) ---------------------
 * z_vals[N][S0+S1] (float64) for rays_o/rays_d [N][3] float32 and gt_depth [N] float32
 * (NULL = no depth: S1 is forced to 0 and near = 0.01).  t_strat = torch.linspace(0,1,S0)
 * (float32), t_surf = torch.linspace(0,1,S1).double() — passed in so the sampler uses the very
 * values the reference uses.  The batch-global max(gt_depth) (Renderer.py:109,144) is computed
 * over the N rays unless gt_max (a DEVICE float) is given — a ray-sharded job passes the
 * all-reduced maximum so every shard samples exactly as the full batch would.
 * ws must hold nslam_workspace_size(NSLAM_WS_SAMPLER, N) bytes. */
int nslam_sample_rays(const float* rays_o, const float* rays_d, const float* gt_depth, const float* gt_max,
                      int64_t n_rays, const double* bound_lo, const double* bound_hi, /* HOST pointers, 3 each */
                      const float* t_strat, int32_t s0, const double* t_surf, int32_t s1,
                      int32_t lindisp, double* z_vals, void* ws, size_t ws_bytes, void* stream);

/* ---- fused point query ------------------------------------------------------------------------
 * raw[M][4] float32 for pts[M][3] float64 (Renderer.eval_points incl. `ret[~mask,3]=100`). */
int nslam_query_fwd(const nslam_query_cfg* cfg, const double* pts, int64_t n_pts, float* raw, void* stream);
/* The same result with the decoders evaluated by separate workgroups (ABI v5): fine and colour
 * stages launch 2-3x the waves of nslam_query_fwd (latency hiding at mapping batch sizes) and
 * combine fine + middle occupancy afterwards.  ws: nslam_query_fwd_workspace_size(cfg, M) bytes
 * (0 for the coarse and middle stages, which fall through to nslam_query_fwd). */
int nslam_query_fwd_ws(const nslam_query_cfg* cfg, const double* pts, int64_t n_pts, float* raw, void* ws,
                       size_t ws_bytes, void* stream);
size_t nslam_query_fwd_workspace_size(const nslam_query_cfg* cfg, int64_t n_pts);

/* Backward of nslam_query_fwd for cotangent g_raw[M][4]: accumulates grid gradients into
 * cfg->grid[i].grad (atomics, caller zero-initialises), adds parameter gradients into
 * cfg->dgrad[i] (per-workgroup LDS accumulation → partial slabs in `ws` → deterministic
 * reduction) and writes g_pts[M][3] float64 when cfg->need_pts_grad.
 * ws must hold nslam_query_bwd_workspace_size(cfg, n_pts) bytes (0 when no parameter grads). */
int nslam_query_bwd(const nslam_query_cfg* cfg, const double* pts, int64_t n_pts, const float* g_raw,
                    double* g_pts, void* ws, size_t ws_bytes, void* stream);
size_t nslam_query_bwd_workspace_size(const nslam_query_cfg* cfg, int64_t n_pts);
/* One decoder's share of nslam_query_bwd (ABI v4): its grid gradient, its parameter gradients
 * and its d/dpts (written, or added when accumulate_pts).  Decoders whose gradients go to
 * different buffers may run concurrently on different streams (the mapping iteration does:
 * grids and decoder gradients are disjoint; with need_pts_grad the calls must be ordered).
 * ws: nslam_query_bwd_decoder_workspace_size(cfg, dec, n_pts) bytes. */
int nslam_query_bwd_decoder(const nslam_query_cfg* cfg, int32_t dec, int32_t accumulate_pts, const double* pts,
                            int64_t n_pts, const float* g_raw, double* g_pts, void* ws, size_t ws_bytes,
                            void* stream);
size_t nslam_query_bwd_decoder_workspace_size(const nslam_query_cfg* cfg, int32_t dec, int64_t n_pts);
size_t nslam_query_saved_size(int64_t n_pts);
size_t nslam_query_tape_size(int64_t n_pts); /* ABI v9 */
/* ABI v10 (v16 signature): the backward of several decoders in ONE launch — the grid gradient and
 * d/dpts share of nslam_query_bwd_decoder of every decoder d in dec_mask (bit d), their workgroups
 * interleaved over the grid, so decoders that would run as concurrent launches on separate streams
 * need no cross-stream fork / join.  Requires cfg->saved_masks (the forward's ReLU masks): every
 * decoder runs the mask-only backward.  No parameter gradients are formed here: a decoder in dec_mask
 * with dgrad[d].base != NULL is NSLAM_EUNSUPPORTED (the colour decoder's come from nslam_color_wgrad).
 * With cfg->need_pts_grad, g_pts[d] (a host array of 4 device pointers) receives decoder d's d/dpts
 * [M][3] float64 (written, not accumulated).  Replaces the per-decoder loop of
 * Tracker.optimize_cam_in_batch's backward (Tracker.py:125) / Mapper.optimize_map's (Mapper.py:503). */
int nslam_query_bwd_decoders(const nslam_query_cfg* cfg, int32_t dec_mask, const double* pts, int64_t n_pts,
                             const float* g_raw, double* const* g_pts, void* stream);
/* ABI v16: the colour decoder's parameter gradients of a colour-stage backward (added into
 * cfg->dgrad[COLOR]; Mapper.py:503 for color_decoder.parameters(), decoder.py:177-203) from the
 * forward's activation tape and ReLU masks (cfg->act_tape, cfg->saved_masks) and the cotangent
 * g_raw[M][4] — the cotangent chain, the colour feature and the Fourier features are recomputed, so
 * the call reads nothing the grid-gradient backward (nslam_query_bwd_decoders) writes and the two may
 * run concurrently on different streams.  Split-K over the points, deterministic.
 * ws >= nslam_query_bwd_decoder_workspace_size(cfg, NSLAM_DEC_COLOR, M) bytes. */
int nslam_color_wgrad(const nslam_query_cfg* cfg, const double* pts, int64_t n_pts, const float* g_raw, void* ws,
                      size_t ws_bytes, void* stream);

/* ---- compositing: raw2outputs_nerf_color, src/common.py:204-245 (occupancy mode) ------------ */
int nslam_composite_fwd(const float* raw, const double* z_vals, int64_t n_rays, int32_t n_samples,
                        double* depth, double* var, float* color, void* stream);
/* g_raw[N][S][4] from cotangents g_depth[N], g_var[N] (float64), g_color[N][3] (float32);
 * any cotangent pointer may be NULL (= zeros). */
int nslam_composite_bwd(const float* raw, const double* z_vals, int64_t n_rays, int32_t n_samples,
                        const double* g_depth, const double* g_var, const float* g_color, float* g_raw,
                        void* stream);

/* ---- standalone trilinear lookup (F.grid_sample 5-D, bilinear, border, align_corners=True;
 *      the op of src/conv_onet/models/decoder.py:173-174) ----------------------------------------
 * coords[M][3] float32 normalised (x,y,z in [-1,1]); out[M][32]. */
int nslam_grid_sample_fwd(const float* grid, const int32_t* dims, const float* coords, int64_t n,
                          float* out, void* stream);
/* grad_grid (atomics, may be NULL) and grad_coords[M][3] (may be NULL) from grad_out[M][32].
 * `dims` (Z, Y, X) is a HOST pointer in both grid_sample entry points. */
int nslam_grid_sample_bwd(const float* grid, const int32_t* dims, const float* coords, int64_t n,
                          const float* grad_out, float* grad_grid, float* grad_coords, void* stream);

/* ---- mapping / tracking iteration (ABI v4) ------------------------------------------------ */
#define NSLAM_MAX_FRAMES 32

/* One RGB-D frame resident on the device (keyframe_dict entry / current frame). */
typedef struct nslam_frame {
  const float* depth; /* [H][W] float32                              */
  const float* color; /* [H][W][3] float32                           */
  const float* c2w;   /* [3 or 4][4] float32 row-major camera-to-world (may be NULL when cam is set) */
  /* ABI v21: the pose given by its camera 7-vector instead (get_camera_from_tensor, common.py:137-176, the
   * arithmetic of nslam_cam_pose): the gather forms it itself and, when c2w_out is not NULL, also writes
   * it there ([3][4] row-major) for later launches — the tracker's camera iteration needs no pose launch */
  const float* cam;   /* [7] float32 (q, t) or NULL                   */
  float* c2w_out;     /* [3][4] float32 or NULL                        */
} nslam_frame;

/* In-kernel pixel draws (ABI v7): with pix == NULL and draw != NULL the select_uv indices are drawn
 * on the device — uniform over the window, from a counter-based splitmix64 stream keyed by
 * (seed, *counter, ray), NOT torch.randint's Philox sequence — and *counter advances by one per
 * call (the last workgroup bumps it, stream-ordered), so a hipGraph replay draws fresh pixels
 * without host RNG work.  ticket: device uint32, zero-initialised once, reserved for the call. */
typedef struct nslam_draw {
  uint64_t seed;
  uint64_t* counter;
  uint32_t* ticket;
  /* Ray sharding without a collective (world > 1; world = 1, rank = 0: a single rank).  The
   * global batch holds n_per * world pixels per frame, drawn from ONE stream (every rank passes
   * the same seed); this call's ray (f, k) is global ray f*n_per*world + rank*n_per + k.
   * gt_max (device float, may be NULL) receives max(gt_depth) over the kept rays of the whole
   * global batch (Renderer.py:107-111,144), which every rank evaluates itself — each thread
   * re-draws its pixel slot for every rank — so the sampler needs no all-reduce.
   * gt_max_key: device uint32, zero-initialised once, required with gt_max. */
  int32_t world;
  int32_t rank;
  float* gt_max;
  uint32_t* gt_max_key;
} nslam_draw;

/* n_kept (ABI v7, device int64, may be NULL) is incremented by the number of kept rays.
 * get_samples (src/common.py:92-134: get_sample_uv + select_uv + get_rays_from_uv) for
 * n_frames frames (HOST array, <= NSLAM_MAX_FRAMES) x n_per pixels each, plus the inside-mask
 * prefilter of Mapper.py:469-481 / Tracker.py:93-104.  pix[f*n_per + k] is select_uv's randint
 * index into the frame's window [h0,h1) x [w0,w1) (row-major over the window).  Outputs are
 * [n_frames*n_per] rays in frame order.  With bound_lo/bound_hi (HOST, float64 [3]) a ray whose
 * bound-exit distance is < gt depth gets keep = 0 and gt_depth = 0 (it then contributes nothing:
 * the prefilter removes it in the reference); NULL bounds keep every ray. */
int nslam_gather_rays(const nslam_frame* frames, int32_t n_frames, int64_t n_per, const int64_t* pix,
                      int32_t H, int32_t W, int32_t h0, int32_t h1, int32_t w0, int32_t w1, float fx, float fy,
                      float cx, float cy, const double* bound_lo, const double* bound_hi, float* rays_o,
                      float* rays_d, float* gt_depth, float* gt_color, uint8_t* keep, const struct nslam_draw* draw,
                      int64_t* n_kept, void* stream);

/* Rendering loss fused with compositing and its backward (the loss is a sum of per-ray terms).
 *   mode NSLAM_LOSS_MAPPER (Mapper.py:487-501):
 *     L = sum_{keep, gt>0} |gt - depth| + [use_color] w_color * sum_{keep} |gt_c - color|
 *   mode NSLAM_LOSS_TRACKER (Tracker.py:110-123), u = var (detached):
 *     r = |gt - depth| / sqrt(u + 1e-10);  m = keep & gt>0 [& r < 10 median_{keep}(r) if handle_dynamic]
 *     L = sum_m r + [use_color] w_color * sum_m |gt_c - color|
 * Writes depth/var (float64 [N]) and color (float32 [N][3]) like nslam_composite_fwd, the
 * per-ray loss terms ray_loss (float64 [N], may be NULL) and, when g_raw != NULL, dL/draw
 * [N][S][4] for dL = 1.  keep may be NULL (all rays kept).  The tracker's median needs
 * N <= 16384 rays. ws: nslam_render_loss_workspace_size bytes. */
enum { NSLAM_LOSS_MAPPER = 0, NSLAM_LOSS_TRACKER = 1 };
typedef struct nslam_loss_cfg {
  int32_t mode;
  int32_t use_color;
  int32_t handle_dynamic;
  float w_color;
  const float* occ_add; /* ABI v7: NULL, or [N*S] float added to raw[...,3] on read (the middle
                           occupancy of a deferred-combine query, decoder.py:331-334 order) */
} nslam_loss_cfg;
int nslam_render_loss(const nslam_loss_cfg* cfg, const float* raw, const double* z_vals, int64_t n_rays,
                      int32_t n_samples, const float* gt_depth, const float* gt_color, const uint8_t* keep,
                      double* depth, double* var, float* color, double* ray_loss, float* g_raw, void* ws,
                      size_t ws_bytes, void* stream);
size_t nslam_render_loss_workspace_size(const nslam_loss_cfg* cfg, int64_t n_rays);

/* Adam (torch.optim.Adam, weight_decay 0, amsgrad off: Tracker.py:126, Mapper.py:504) over up to
 * NSLAM_ADAM_MAX_SEGS parameter segments in one launch.  A segment is dense (rows == NULL: n
 * floats) or row-masked (n row indices of row_len floats each, row_len % 4 == 0 and 16-byte
 * aligned param/grad/state): the frustum-selected voxels of a channels-last grid
 * (Mapper.py:314-333), updated in place in the dense grid with state for the selected rows only
 * (exp_avg/exp_avg_sq are [n][row_len], in row-list order).  Like torch, every segment has its
 * own step count (`step`, a device float, 0 before the first update): the launch uses step+1
 * and a second single-wave launch advances every segment's step (graph-replay safe); `ticket`
 * is unused since ABI v5 (may be NULL).  Pass only segments that have a gradient
 * this iteration (torch skips parameters whose .grad is None).  With zero_grad the grad entries
 * read are reset to 0. */
#define NSLAM_ADAM_MAX_SEGS 16
typedef struct nslam_adam_seg {
  float* param;
  float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  float* step;
  const int32_t* rows;
  int64_t n;
  int32_t row_len;
  float lr;
  int32_t grad_rows; /* ABI v6, row-masked segments: 1 = grad is compact [n][row_len] in row-list order
                        (the frustum-compacted gradient of nslam_grid.slot); 0 = grad is dense like param */
  int32_t pad_;
  /* ABI v7, dense segments: after the update param[e] is also stored to mirror[mirror_idx[2e]] and
   * mirror[mirror_idx[2e+1]] (-1 = none): the MFMA-packed copy of a decoder (nslam_pack_layout)
   * stays current without a re-pack pass.  mirror == NULL: no mirror. */
  const int32_t* mirror_idx;
  float* mirror;
  /* ABI v19: NULL, or a DEVICE int64: the segment updates only its first min(*n_live, n) rows (row-masked)
   * or elements (dense).  A frustum selection made on the device (Mapper.optimize_map's per-call mask,
   * Mapper.py:314-333) then needs no host read-back of its size: the segment, its Adam state and its
   * launch are sized for the capacity n (every voxel of the grid), so a captured hipGraph of the
   * iteration stays valid for every later call's selection. */
  const int64_t* n_live;
} nslam_adam_seg;
/* ticket: NULL = the step counts advance in a second single-wave launch; else a device uint32
 * (zero-initialised, re-armed by the call itself) with which the update kernel's last workgroup
 * advances them — one launch per step (ABI v9).  A ticket belongs to one call at a time: calls that
 * may run concurrently (other streams, other processes) each pass their own. */
int nslam_adam_step(const nslam_adam_seg* segs, int32_t n_segs, float beta1, float beta2, float eps,
                    int32_t zero_grad, uint32_t* ticket, void* stream);
/* Sparse gradient exchange of a ray-sharded mapping iteration (ABI v5).  Only the frustum-
 * selected grid rows reach Adam (Mapper.py:314-333,394-401,504), so only they need summing across
 * ranks: nslam_rows_pack copies rows[i] (row_len floats each, row_len % 4 == 0, 16-byte aligned
 * grid and out) of `grid` to out[i*row_len ...] and appends the n_tail floats of `tail` (the
 * decoder gradients); the caller all-reduces `out` (n_rows*row_len + n_tail floats) and
 * nslam_rows_unpack writes it back.  Row indices are in units of row_len floats from `grid`, so
 * one call covers every grid of a flat gradient buffer. */
int nslam_rows_pack(const float* grid, const int32_t* rows, int64_t n_rows, int32_t row_len, const float* tail,
                    int64_t n_tail, float* out, void* stream);
int nslam_rows_unpack(const float* in, const int32_t* rows, int64_t n_rows, int32_t row_len, float* grid,
                      float* tail, int64_t n_tail, void* stream);

/* ABI v9.  Camera gradient of a tracking iteration (Tracker.py:110-126): the 7-vector gradient of
 * the loss through pts = t + (R·dir)·z (Renderer.py:172-174, common.py:80-89) and
 * get_camera_from_tensor (common.py:137-176), in one single-workgroup launch:
 *   g_t = Σ g_pts;  g_R = (Σ_r g_d,r d_rᵀ)·R with g_d,r = Σ_s z_rs g_pts,rs (dir = Rᵀ d);
 *   g_q = s (G + Gᵀ) q − s² (qᵀ G q) q,  s = 2/|q|²,  G = Σ_ij g_R,ij M_ij  (R = I + s·P(q)).
 * cam [7] (w,x,y,z,tx,ty,tz), c2w [3,4] the pose rendered with, g_pts [n_rays*n_samples,3] f64,
 * z_vals [n_rays,n_samples] f64, rays_d [n_rays,3] f32; writes g_cam [7] f32.
 * NSLAM_EUNSUPPORTED when 3*n_rays*n_samples >= 2^31 (32-bit g_pts offsets). */
int nslam_cam_grad(const float* cam, const float* c2w, const double* g_pts, const double* z_vals, const float* rays_d,
                   int64_t n_rays, int32_t n_samples, float* g_cam, void* stream);
/* ABI v15: the same gradient from n_parts (1..4) d/dpts buffers — the frozen decoders' shares of
 * nslam_query_bwd_decoders — summed per point in buffer order ((g0 + g1) + g2, float64), over up to
 * 32 workgroups whose partial sums meet in ws (NSLAM_CAM_GRAD_WS_DOUBLES doubles; the last workgroup,
 * by `ticket` — a device uint32 zeroed once and re-armed by the call — adds them in workgroup order:
 * deterministic).  Replaces the buffer adds + single-workgroup nslam_cam_grad of a tracking iteration. */
#define NSLAM_CAM_GRAD_WS_DOUBLES (32 * 12)
int nslam_cam_grad_parts(const float* cam, const float* c2w, const double* const* g_pts, int32_t n_parts,
                         const double* z_vals, const float* rays_d, int64_t n_rays, int32_t n_samples, float* g_cam,
                         double* ws, uint32_t* ticket, void* stream);

/* ABI v19.  The camera gradients of bundle adjustment (Mapper.py:346-363, 441-448, 503): n_cams
 * cameras, camera k's rays being rays [ray_begin[k], ray_begin[k] + n_rays_per) of the batch (one frame
 * of the mapping window each).  cams [n_cams][7] and g_cam [n_cams][7] contiguous f32; c2w: camera k's
 * pose rendered with at c2w + k * c2w_stride floats ([3,4] row-major rows of 4); g_pts as in
 * nslam_cam_grad_parts (1..4 buffers over the whole batch, summed per point in buffer order), z_vals /
 * rays_d over the whole batch.  ray_begin: HOST array.  One launch, up to 32 workgroups per camera;
 * ws: n_cams * NSLAM_CAM_GRAD_WS_DOUBLES doubles; tickets: n_cams device uint32 zeroed once (re-armed by
 * the call).  Per camera the arithmetic and order are nslam_cam_grad_parts' over its slice: the same
 * values bit for bit. */
int nslam_cam_grad_batch(const float* cams, const float* c2w, int64_t c2w_stride, int32_t n_cams,
                         const int64_t* ray_begin, int64_t n_rays_per, const double* const* g_pts, int32_t n_parts,
                         const double* z_vals, const float* rays_d, int64_t n_rays, int32_t n_samples, float* g_cam,
                         double* ws, uint32_t* tickets, void* stream);
/* ABI v23.  A tracking iteration's camera tail fused into nslam_cam_grad_parts' last workgroup: after g_cam
 * is formed, Adam on the camera 7-vector in place (torch.optim.Adam, Tracker.py:126: nslam_adam_step's
 * element update and bias corrections with the step count *step, then *step += 1), *loss_out = the sum of
 * ray_loss[0..n_rays) (nslam_loss_sum_best's fixed-order tree: the same value), and, when best_loss is not
 * NULL, the best-pose update (Tracker.py:245-247) with the stepped camera.  Bit-identical to
 * nslam_cam_grad_parts + nslam_adam_step + nslam_loss_sum_best in that order, in one launch. */
typedef struct nslam_cam_tail {
  float* cam;        /* [7], read by the gradient and stepped in place */
  float* exp_avg;    /* [7] Adam state */
  float* exp_avg_sq; /* [7] */
  float* step;       /* [1] step count */
  float lr, beta1, beta2, eps;
  const double* ray_loss; /* [n_rays] the iteration's per-ray losses */
  int64_t n_rays;
  double* loss_out;  /* [1] */
  double* best_loss; /* [1] or NULL */
  float* best;       /* [7] (with best_loss) */
} nslam_cam_tail;
int nslam_cam_grad_step(const nslam_cam_tail* tail, const float* c2w, const double* const* g_pts, int32_t n_parts,
                        const double* z_vals, const float* rays_d, int64_t n_rays, int32_t n_samples, float* g_cam,
                        double* ws, uint32_t* ticket, void* stream);

/* ABI v19: nslam_cam_pose for n cameras in one launch: c2w + k * c2w_stride = get_camera_from_tensor(cams[k]). */
int nslam_cam_pose_batch(const float* cams, float* c2w, int64_t c2w_stride, int32_t n, void* stream);

/* ABI v20.  The frustum voxel selection of Mapper.get_mask_from_c2w (Mapper.py:93-164) after its two
 * projection GEMMs, compacted into a capacity-bound row list (what MappingEngine.bind_masks builds with
 * torch ops, in one pass of four launches).  Inputs in the reference's point order
 * i = (ix*ny + iy)*nz + iz of its meshgrid: uvz [N][3] float64 = (points @ w2c[:3,:3]ᵀ + w2c[:3,3])
 * .double() * (-1, 1, 1) @ Kᵀ and near [N] (uint8 bool) = |points - t|² < 0.25, both formed by the
 * caller; depth [H][W] float32 (the current frame).  Computes uv = (uvz[:2] / (uvz[2] + 1e-5)) as
 * float, cv2.remap's bilinear depth at uv (1/32-pixel fixed-point positions, zero border), zero depths
 * replaced by the maximum over all N points, and mask = (0 < u < W, 0 < v < H, 0 <= -z <= depth + 0.5)
 * | near; then, over voxels v = (iz*ny + iy)*nx + ix (channels-last order): slot[v] = the rank of v among
 * the selected voxels or -1, rows[rank] = v (ascending), *n_live = their count.  mask_ref: optional [N]
 * uint8 mask in the reference order.  ws: nslam_frustum_rows_workspace_size(N) bytes. */
int nslam_frustum_rows(const double* uvz, const uint8_t* near, const float* depth, int32_t H, int32_t W, int32_t nx,
                       int32_t ny, int32_t nz, int32_t* slot, int32_t* rows, int64_t* n_live, uint8_t* mask_ref,
                       void* ws, size_t ws_bytes, void* stream);
size_t nslam_frustum_rows_workspace_size(int64_t n_vox);

/* ABI v20.  The tracker's best-pose bookkeeping of one camera iteration (Tracker.py:245-247: if loss <
 * best_loss: best_loss = loss, candidate = camera_tensor), on the device: if *loss < *best_loss (float64),
 * *best_loss = *loss and best[0..n) = cam[0..n) (n <= 64, float32).  One single-wave launch. */
int nslam_track_best(const double* loss, double* best_loss, const float* cam, float* best, int32_t n, void* stream);
/* ABI v21.  The camera iteration's loss and its best-pose bookkeeping in one launch: *loss_out = the sum of
 * ray_loss[0..n_rays) (float64; a fixed-order tree over one workgroup: the same value every call), then,
 * when best_loss is not NULL, nslam_track_best's update with that sum (cam, best: n <= 64 float32).
 * Replaces optimize_cam_in_batch's loss.sum() (Tracker.py:110-123) and the comparison of Tracker.py:245-247,
 * so the tracker's camera loop needs no reduction launch of its own. */
int nslam_loss_sum_best(const double* ray_loss, int64_t n_rays, double* loss_out, double* best_loss, const float* cam,
                        float* best, int32_t n, void* stream);

/* ABI v22.  The inverse map for n poses in one launch: cams[k] (7 float32) = get_tensor_from_camera(c2w +
 * k * c2w_stride) (common.py:179-201, as common.camera_tensors restates it on the device: quaternion
 * (w,x,y,z) by the trace / largest-diagonal branch rule in float64, normalised, w >= 0, then T, rounded to
 * float32 once); cams_copy (optional) receives the same 7-vectors.  Replaces the tracker's per-frame
 * camera_tensor and best-pose initialisation (Tracker.py:199-200, 225) and bundle adjustment's camera
 * set-up (Mapper.py:349-363), each ~70 torch launches.  n <= 64, c2w_stride >= 12 floats. */
int nslam_cam_vector_batch(const float* c2w, int64_t c2w_stride, int32_t n, float* cams, float* cams_copy,
                           void* stream);

/* ABI v9.  c2w [3,4] f32 = get_camera_from_tensor(cam [7]) (common.py:137-176, quad2rotation's
 * products and differences, no FMA contraction), one thread.  |q|² is summed ((w²+x²)+y²)+z²;
 * the order of torch's (quad*quad).sum(-1) reduction is not pinned, so the pose matches the
 * reference to within ~1 ulp per entry (bit-identical for most poses), not bit-for-bit. */
int nslam_cam_pose(const float* cam, float* c2w, void* stream);

enum { NSLAM_WS_SAMPLER = 0 };
size_t nslam_workspace_size(int which, int64_t n);

const char* nslam_strerror(int code);
int nslam_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* NSLAM_H */
