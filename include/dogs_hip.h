/*
 * dogs_hip.h -- C ABI of libdogs_hip.so, the MI355X (gfx950) implementation of the DOGS hot path:
 * the Taming-3DGS differentiable tile rasterizer, fused SSIM, sparse Adam and simple-knn.
 *
 * Every entry point replaces one function of the reference's pybind11 tables; the binding stub a
 * maintainer adds on the reference side is in INTEGRATION.md.  Conventions:
 *   - all pointers are device pointers (HBM) unless noted, fp32 row-major exactly as the torch tensors
 *     the reference passes (rasterize_points.cu:127-147), NULL = "empty tensor" (absent);
 *   - `stream` is a hipStream_t (the caller's current stream); nothing runs on the null stream;
 *   - return 0 on success, non-zero on error; dg_last_error() gives the message (thread-local);
 *   - scratch memory comes from the caller through dg_alloc_fn, like the reference's
 *     std::function<char*(size_t)> resize callbacks (rasterize_points.cu:30-52).  The forward's
 *     geometry/binning/image blocks are private state the caller hands back to the backward.
 */
#ifndef DOGS_HIP_H
#define DOGS_HIP_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* dg_stream_t; /* hipStream_t */

/* which: DG_BUF_* below.  Must return a device pointer aligned to >= 256 bytes, or NULL. */
typedef void* (*dg_alloc_fn)(void* user, int which, uint64_t nbytes);
enum { DG_BUF_GEOM = 0, DG_BUF_BINNING = 1, DG_BUF_IMAGE = 2, DG_BUF_BACKWARD = 3, DG_BUF_TEMP = 4,
       DG_BUF_BINNING2 = 5 };

/* The scalar + tensor arguments of _C.rasterize_gaussians (rasterize_points.h:18-40). */
typedef struct {
    int P;              /* means3D.size(0) */
    int D;              /* sh degree (raster_settings.sh_degree) */
    int M;              /* sh.size(1) (0 when sh is absent) */
    int W, H;           /* image_width, image_height */
    int prefiltered, antialiasing, debug;
    int prefix_per_tile;        /* depth-prefix binning: phase-1 capacity = this x tiles in tile-rect area
                                   units; 0 -> adaptive (448, grown x1.5 per image size while views keep
                                   needing phase 2); < 0 bins every instance in one phase.  Must agree in
                                   sign between forward and backward of one view. */
    float scale_modifier, tanfovx, tanfovy;
    const float* bg;            /* [3] */
    const float* means3D;       /* [P,3] */
    const float* colors;        /* [P,3] or NULL (colors_precomp) */
    const float* opacities;     /* [P,1] */
    const float* scales;        /* [P,3] or NULL */
    const float* rotations;     /* [P,4] or NULL */
    const float* cov3D_precomp; /* [P,6] or NULL */
    const float* viewmatrix;    /* [4,4] = world_to_camera^T */
    const float* projmatrix;    /* [4,4] = world_to_camera^T @ P^T */
    const float* dc;            /* [P,1,3] */
    const float* sh;            /* [P,M,3] or NULL */
    const float* campos;        /* [3] */
    int capacity_ctx;           /* adaptive capacity context (prefix_per_tile == 0): the growth state is per (device,
                                   image size, context); 0 is the process-wide default.  A trainer that passes its
                                   own context sees a capacity history -- and so an instance numbering and the
                                   rounding of its per-Gaussian gradient sums -- that does not depend on what else
                                   the process rendered (the ADMM ranks and the sequential baseline agree bit for
                                   bit).  No reference counterpart (the reference bins every instance). */
} dg_raster_args;

/* Replaces RasterizeGaussiansCUDA (rasterize_points.cu:55-154) / _C.rasterize_gaussians.
 * Outputs out_color [3,H,W], out_invdepth [1,H,W], radii [P] (int32).
 * *num_rendered = the reference's num_rendered (sum of tile-rect areas);
 * *num_instances = the phase-1 binning capacity this view used (returned where the reference returns num_buckets;
 * both are opaque tokens handed back to the backward; dg_binned_instances gives the instance count).
 * Binning is depth-prefix (DESIGN.md "Binning"):
 * phase 1 bins the first instances of the global depth order (a prefix of every tile's list), phase 2 bins
 * the rest only for tiles that phase 1 left unfinished -- same images and gradients, far fewer instances.
 * Allocates DG_BUF_GEOM, DG_BUF_IMAGE, DG_BUF_BINNING and, only when phase 2 runs, DG_BUF_BINNING2 through
 * `alloc`; the caller keeps the four pointers (*binning2 = NULL when absent; the reference's sampleBuffer
 * slot carries it) and passes them to dg_rasterize_backward.  One host sync, after the binning is queued (two
 * with prefix_per_tile < 0, which sizes the binning from the rect total first). */
int dg_rasterize_forward(const dg_raster_args* a, float* out_color, float* out_invdepth, int* radii,
                         dg_alloc_fn alloc, void* user, void** geom, void** binning, void** image, void** binning2,
                         int64_t* num_rendered, int64_t* num_instances, dg_stream_t stream);

/* Replaces RasterizeGaussiansBackwardCUDA (rasterize_points.cu:157-252).  Every output is fully
 * written (no zero-fill needed): dmeans2D [P,3], dcolors [P,3], dopacity [P,1], dmeans3D [P,3],
 * dcov3D [P,6], ddc [P,1,3], dsh [P,M,3] (may be NULL when M == 0), dscales [P,3], drot [P,4],
 * depth [P,1].  dL_dout_invdepth may be NULL (treated as zeros).  Allocates DG_BUF_BACKWARD. */
/* LightGaussian count mode (old_diff-gaussian-rasterization: CountGaussiansCUDA, rasterize_points.cu:148-233, and
 * renderCUDA_count, forward.cu:392-500): the forward above plus, per Gaussian, the number of pixels it contributes
 * to (gaussians_count, int32[P]) and important_score = opacity x that count (float[P]).  The counts are exact
 * (integer atomics; the reference's non-atomic increments race).  The private state blocks are requested from
 * alloc as in dg_rasterize_forward and are not needed afterwards. */
int dg_rasterize_count(const dg_raster_args* a, float* out_color, int* radii, int32_t* gaussians_count,
                       float* important_score, dg_alloc_fn alloc, void* user, int64_t* num_rendered,
                       dg_stream_t stream);

int dg_rasterize_backward(const dg_raster_args* a, const int* radii, const void* geom, const void* binning,
                          const void* image, const void* binning2, int64_t num_rendered, int64_t num_instances,
                          const float* dL_dout_color, const float* dL_dout_invdepth, float* dmeans2D,
                          float* dcolors, float* dopacity, float* dmeans3D, float* dcov3D, float* ddc,
                          float* dsh, float* dscales, float* drot, float* depth, dg_alloc_fn alloc, void* user,
                          dg_stream_t stream);

/* Replaces markVisible (rasterize_points.cu:254-273) / _C.mark_visible: present [P] bool. */
int dg_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                    uint8_t* present, dg_stream_t stream);

/* The weight gradient of the appearance embedding's 3x3 convolutions (conerf/model/gaussian_fields/masks.py:8-54,
 * geometry.mask; replaces the MIOpen/cuDNN backward-weights call torch makes for nn.Conv2d(k=3, padding=1)):
 * dw [Cout][Cin][3][3] = sum over pixels of dy[co] x [ci] shifted, db [Cout] = sum of dy[co], for x [Cin][H][W] and
 * dy [Cout][H][W] (one image).  gate (may be NULL, [Cout][H][W]): dy counts only where gate > 0 -- the backward of a
 * ReLU applied to the convolution's output (gate = that output) folded in.  flags DG_CONV_SHUFFLE: x is [4 Cin][H/2]
 * [W/2], read as its PixelShuffle(2) (H, W even).  Deterministic (fixed-order partial sums, no atomics).  Cin, Cout <= 4000 (an error otherwise); scratch of dg_conv3x3_wgrad_scratch_bytes() bytes. */
size_t dg_conv3x3_wgrad_scratch_bytes(int Cin, int Cout, int H, int W);
int dg_conv3x3_wgrad(int Cin, int Cout, int H, int W, const float* x, const float* dy, const float* gate, int flags,
                     float* dw, float* db, void* scratch, size_t scratch_bytes, dg_stream_t stream);

/* The same convolutions' forward and data gradient (masks.py:8-54: nn.Conv2d(k=3, padding=1) on one image; replaces
 * the MIOpen forward and backward-data calls, whose algorithm choice depends on MIOpen's find database and on what the
 * process ran before).  flags 0: y [Cout][H][W] = conv(x [Cin][H][W], w [Cout][Cin][3][3]) + b (b may be NULL);
 * | DG_CONV_RELU: max(y, 0) (nn.Sequential's following ReLU folded into the store);  DG_CONV_ADJOINT: y [Cin][H][W] =
 * the input gradient for the output gradient x [Cout][H][W] (b unused), counting x only where gate > 0 when gate is
 * given (the ReLU's backward, gate = the forward's output; NULL: no ReLU).  DG_CONV_SHUFFLE (H, W even): the
 * forward's x is [4 Cin][H/2][W/2] read as its PixelShuffle(2), and the adjoint writes y as [4 Cin][H/2][W/2] (the
 * shuffle's input gradient) -- the upsampling stages' nn.PixelShuffle folded in.  Each output sums over (input
 * channel, tap) in a fixed order.  Cin, Cout <= 65536 and Cin * Cout <= 2^24 (an error otherwise). */
enum { DG_CONV_ADJOINT = 1, DG_CONV_RELU = 2, DG_CONV_SHUFFLE = 4 };
int dg_conv3x3(int Cin, int Cout, int H, int W, const float* x, const float* w, const float* b, float* y, int flags,
               const float* gate, dg_stream_t stream);

/* The appearance embedding's full-resolution head (masks.py:8-54: F.interpolate(x, (H, W), "bilinear") then
 * out_conv = Conv2d(16, 8, 3, pad 1) -> ReLU -> Conv2d(8, 3, 3, pad 1); replaces the resize, the two nn.Conv2d calls
 * and their autograd backward): u [16][h2][w2] (the last upsampling stage's output), w1 [8][16][3][3], b1 [8],
 * w2p [3][8][3][3], b2 [3] -> mask [3][H][W]; `hidden` [8][H][W] (may be NULL) receives relu(conv1(resize(u))).
 * The backward takes dmask [3][H][W] and `hidden` (the forward's; NULL: recomputed) and writes du [16][h2][w2] and
 * dparams [dg_mask_head_nparams()] = dW1 | db1 | dW2 | db2, with scratch of dg_mask_head_scratch_bytes(H, W) bytes.
 * Deterministic (fixed-order sums, no atomics; the same bits with and without `hidden`).  H <= 4 h2 and W <= 4 w2
 * (an error otherwise). */
int dg_mask_head_forward(int H, int W, int h2, int w2, const float* u, const float* w1, const float* b1,
                         const float* w2p, const float* b2, float* mask, float* hidden, dg_stream_t stream);
size_t dg_mask_head_scratch_bytes(int H, int W);
int dg_mask_head_nparams(void);
int dg_mask_head_backward(int H, int W, int h2, int w2, const float* u, const float* w1, const float* b1,
                          const float* w2p, const float* b2, const float* dmask, const float* hidden, float* du,
                          float* dparams, void* scratch, size_t scratch_bytes, dg_stream_t stream);

/* The precise tile cull's threshold logf(opacity / (1/255)) of each of n opacities, with the arithmetic the binning
 * uses (duplicateWithKeys, rasterizer_impl.cu:149-151: the correctly rounded logf).  A parity probe:
 * the reference has no such entry; the tests compare it with the oracle on every opacity in (2^-24, 1]. */
int dg_cull_log_threshold(int64_t n, const float* opacity, float* thr, dg_stream_t stream);

/* Replaces RasterizeGaussiansFilterCUDA (rasterize_points.cu:276-334) / _C.rasterize_gaussians_filter:
 * radii [P] only (no low-pass filter), uses P, W, H, tanfov*, scale_modifier, means3D, scales,
 * rotations, cov3D_precomp, viewmatrix, projmatrix, prefiltered of `a`. */
int dg_rasterize_filter(const dg_raster_args* a, int* radii, dg_stream_t stream);

/* Replaces adamUpdate (rasterize_points.cu:336-361, adam.cu:10-38) / _C.adamUpdate, in place. */
int dg_adam_update(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, const uint8_t* visible,
                   float lr, float b1, float b2, float eps, uint32_t N, uint32_t M, dg_stream_t stream);

/* ---- the optimizer side of a training view ---- */

/* One parameter group of SparseGaussianAdam (diff_gaussian_rasterization/__init__.py:303-332): M floats per Gaussian. */
typedef struct {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    float lr, eps;
    uint32_t M;
} dg_adam_group;

/* The view's densification statistics (gaussian_trainer.py:433-438, gaussian_splat_model.py:533-541), for the
 * Gaussians with visible[i]: max_radii2D = max(max_radii2D, radii); grad_accum += ||dmeans2D[i, :2]||; denom += 1.
 * dmeans2D is the screen-space-point gradient [N, stride] (stride 3 for the [N,3] tensor of the reference). */
typedef struct {
    const int* radii;
    const float* dmeans2D;
    uint32_t dmeans2D_stride;
    float* max_radii2D;
    float* grad_accum;
    float* denom;
} dg_densify_stats;

/* The view's photometric L1 term (gaussian_trainer.py: rendered_image.clamp(0, 1), l1_loss(image, gt) = mean |image -
 * gt|): clamped [n] and per-block partial sums of |clamped - gt| (partial [dg_clamp_l1_blocks(n)]; the caller sums
 * them and divides by n, e.g. with dg_mean_of_parts).  Backward: d_img = (g_clamped + *g_l1 * sgn(clamp(img) - gt) / n)
 * where 0 <= img <= 1, else 0 (g_clamped, g_l1: device, NULL = zero; `clamped` is not read -- the clamp is recomputed
 * from img -- and may be NULL).  img, gt, clamped 16-byte aligned. */
uint32_t dg_clamp_l1_blocks(uint32_t n);
int dg_clamp_l1_forward(uint32_t n, const float* img, const float* gt, float* clamped, float* partial,
                        dg_stream_t stream);
int dg_clamp_l1_backward(uint32_t n, const float* img, const float* clamped, const float* gt, const float* g_clamped,
                         const float* g_l1, float* d_img, dg_stream_t stream);

/* torch.prod(x, dim=1) of x [N, M], 1 <= M <= 3 -- the scale regulariser lambda_scale * get_scaling.prod(dim=1).mean()
 * (gaussian_trainer.py:405-408) -- in torch's row order (x0 x2) x1 on the GPU; when some element is 0 the forward
 * writes `stamp` to the device word *zero_stamp (not zeroed: give every forward a stamp of its own, e.g. a counter).
 * The backward is torch's prod_backward (FunctionsManual.cpp) with the zero test on the device instead of a host read:
 * dx = dprod (prod / x) when *zero_stamp != stamp (the forward's), else for every row dprod (exclusive left cumprod x
 * exclusive right cumprod). */
int dg_row_prod_forward(uint32_t N, uint32_t M, const float* x, float* prod, uint32_t* zero_stamp, uint32_t stamp,
                        dg_stream_t stream);
int dg_row_prod_backward(uint32_t N, uint32_t M, const float* x, const float* prod, const float* dprod,
                         const uint32_t* zero_stamp, uint32_t stamp, float* dx, dg_stream_t stream);

/* GaussianSplatModel activations (gaussian_splat_model.py get_opacity / get_scaling / get_quaternion): opacity =
 * sigmoid(raw_opacity) [N,1], scaling = exp(raw_scaling) [N,3], rotation = raw_rotation / max(|raw_rotation|, 1e-12)
 * [N,4] (16-B aligned rows), one launch; and the backward from the activated values and raw rotation (a NULL
 * incoming gradient counts as zeros). */
int dg_activate_forward(uint32_t N, const float* raw_opacity, const float* raw_scaling, const float* raw_rotation,
                        float* opacity, float* scaling, float* rotation, dg_stream_t stream);
int dg_activate_backward(uint32_t N, const float* opacity, const float* scaling, const float* raw_rotation,
                         const float* d_opacity, const float* d_scaling, const float* d_rotation, float* d_raw_opacity,
                         float* d_raw_scaling, float* d_raw_rotation, dg_stream_t stream);

/* SparseGaussianAdam.step(visible, N) over up to 8 groups in one launch (each group as dg_adam_update), plus the
 * densification statistics of the same view when stats != NULL (they read nothing Adam writes). */
int dg_adam_update_groups(const dg_adam_group* groups, int n_groups, const uint8_t* visible, uint32_t N, float b1,
                          float b2, const dg_densify_stats* stats, dg_stream_t stream);
/* The ADMM penalty of a block trainer's loss, 0.5 * rho_p * F.mse_loss(x_p + u_p, z_p) per parameter tensor
 * (SlaveGaussianSplatTrainer.add_admm_penalties, slave_gaussian_trainer.py:161-202), as its gradient
 * coef * ((x + u) - z) with coef = rho_p / numel(x_p), added to the loss gradient of the rows Adam updates (the
 * visible ones; SparseGaussianAdam ignores every other row's gradient, penalty included).  u (duals) and z (global
 * values) have the parameter's shape; u == NULL: no term for that group. */
typedef struct {
    const float* u;
    const float* z;
    float coef;
} dg_adam_prox;
/* dg_adam_update_groups with one dg_adam_prox per group (prox may be NULL). */
int dg_adam_update_groups_prox(const dg_adam_group* groups, const dg_adam_prox* prox, int n_groups,
                               const uint8_t* visible, uint32_t N, float b1, float b2, const dg_densify_stats* stats,
                               dg_stream_t stream);
/* ---- the native training step of a block trainer (dogs_amd.admm_trainer.BlockTrainer's fast path) ----
 * One GaussianSplatTrainer.train_iteration after densify_end_iter (gaussian_trainer.py:324-476) with the ADMM
 * penalty of SlaveGaussianSplatTrainer.add_admm_penalties (slave_gaussian_trainer.py:161-202), as one call:
 *   activations (get_opacity / get_scaling / get_quaternion) -> dg_rasterize_forward -> clamp(0, 1) + L1
 *   -> fused SSIM -> dL/dimage of (1 - lambda_dssim) L1 + lambda_dssim (1 - SSIM) -> dg_rasterize_backward
 *   -> lambda_scale mean(prod(scaling, 1)) + activation backward -> SparseGaussianAdam.step(radii > 0) with the ADMM
 *   proximal gradient and the densification statistics, one launch.
 * The kernels and arithmetic of the autograd path (the drop-in API), issued from C: after the forward's one wait the
 * host enqueues ~15 launches instead of ~100 Python-level operations, so the GPU does not wait on the host.
 * Allocates DG_BUF_GEOM/IMAGE/BINNING(2)/BACKWARD as the rasterizer does, and DG_BUF_TRAIN (the step's scratch). */
enum { DG_BUF_TRAIN = 9 };
typedef struct {
    dg_raster_args view;        /* camera, image size and settings; its Gaussian pointers are ignored */
    const float* gt;            /* [3,H,W] target image */
    float lambda_dssim, lambda_scale;
    /* the model's six raw tensors, in place, in setup_optimizer's order: xyz [P,3], f_dc [P,1,3], f_rest [P,M,3],
     * opacity [P,1] (logit), scaling [P,3] (log), quaternion [P,4]; with Adam moments, lr and eps (grad ignored) */
    dg_adam_group groups[6];
    dg_adam_prox prox[6];       /* ADMM penalty per tensor; u == NULL: none */
    const dg_densify_stats* stats;  /* optional; only max_radii2D / grad_accum / denom are read */
    int* radii;                 /* [P] out */
    float* image;               /* [3,H,W] out: the clamped render */
    float* loss;                /* optional, device [4] out: L1, SSIM, mean prod(scaling), mean((mask - 1)^2) (0
                                   without a mask) of this view */
    /* optional [P] device scratch: overlap the f_dc / f_rest part of the update (81% of its bytes) with the NEXT
     * step's forward up to its binning emission, the first kernel that reads them.  The call returns with that part
     * still running on a side stream; the next dg_train_step on the same stream waits for it before its emission, and
     * any other use of the SH tensors or their moments needs dg_train_sync first. */
    uint8_t* sh_status;
    /* optional: the decoupled appearance mask of geometry.mask (gaussian_trainer.py:392-401, AppearanceEmbedding of
     * masks.py:8-54, evaluated by the caller): mask [3,H,W] (NULL: none).  The photometric term becomes
     * (1 - lambda_dssim) L1(clamp(render) * mask, gt) + lambda_dssim (1 - SSIM(clamp(render), gt))
     * + lambda_mask mean((mask - 1)^2), and dmask [3,H,W] receives dL/dmask for the caller's backward through the
     * embedding network.  Both 16-byte aligned when given. */
    const float* mask;
    float* dmask;
    float lambda_mask;
    /* geometry.depth_threshold (gaussian_trainer.py:376 -> _RasterizeGaussians.backward): > 0 scales the screen-space
     * gradient the densification statistics read by min(1, (depth / depth_threshold)^2); 0: unscaled. */
    float depth_threshold;
} dg_train_step_args;
int dg_train_step(const dg_train_step_args* a, dg_alloc_fn alloc, void* user, dg_stream_t stream);
/* Make `stream` wait for an overlapped f_dc / f_rest update of the last dg_train_step on it (no-op when none). */
int dg_train_sync(dg_stream_t stream);
/* The statistics alone (replaces the max_radii2D update + add_densification_stats of gaussian_trainer.py:433-438). */
int dg_add_densification_stats(const dg_densify_stats* stats, const uint8_t* visible, uint32_t N, dg_stream_t stream);

/* The six optimised tensors of a GaussianSplatModel, in the order xyz [N,3], f_dc [N,1,3], f_rest [N,M,3],
 * opacity [N,1] (raw), scaling [N,3] (raw, log), quaternion [N,4] (raw), with their Adam moments (NULL pair: the
 * optimizer holds no state for that tensor) and the densification statistics. */
typedef struct {
    uint32_t N;
    const float* params[6];
    const float* exp_avg[6];
    const float* exp_avg_sq[6];
    uint32_t width[6];      /* floats per Gaussian: 3, 3, 3*M, 1, 3, 4 */
    const float* grad_accum; /* [N] xyz_gradient_accum */
    const float* denom;      /* [N] */
} dg_gaussian_set;

/* densify_and_prune (gaussian_splat_model.py:434-531) as GPU stream compaction, in four calls sharing this struct:
 *   1. dg_densify_select      clone / split selection -> nc, ns (one sync);
 *   2. dg_densify_split_stds  stds [replicas*ns, 3] = get_scaling of the split Gaussians, repeated replica-major: the
 *                             caller draws samples = torch.normal(mean=0, std=stds) exactly as the reference does;
 *   3. dg_densify_count       prune test over the candidate rows [originals not split | clones | children] ->
 *                             n_out (one sync);
 *   4. dg_densify_gather      every kept row of every tensor and its Adam moments (originals keep theirs, appended
 *                             rows get zeros) into out_* [n_out, width].
 * The statistics are zeros of n_out afterwards (densification_postfix); the caller allocates them. */
typedef struct {
    dg_gaussian_set set;
    float max_grad;          /* densify_grad_threshold */
    float dense_extent;      /* percent_dense * extent */
    uint32_t replicas;       /* num_replica of densify_and_split (0 -> 2) */
    float min_opacity;
    int use_bbox;            /* bounding_box is not None */
    float bbox_z;            /* bounding_box[2] */
    int use_screen;          /* max_screen_size is not None */
    float max_screen_size;
    float big_extent;        /* 0.1 * extent */
    const float* samples;    /* [replicas*ns, 3] */
    float* out_params[6];
    float* out_exp_avg[6];
    float* out_exp_avg_sq[6];
    /* filled by the library */
    void* state;
    void* state2;
    uint32_t nc, ns, n_out;
} dg_densify_args;
enum { DG_BUF_DENSIFY = 6, DG_BUF_DENSIFY2 = 7 };
int dg_densify_select(dg_densify_args* a, dg_alloc_fn alloc, void* user, dg_stream_t stream);
int dg_densify_split_stds(const dg_densify_args* a, float* stds, dg_stream_t stream);
int dg_densify_count(dg_densify_args* a, dg_alloc_fn alloc, void* user, dg_stream_t stream);
int dg_densify_gather(const dg_densify_args* a, dg_stream_t stream);

/* prune_points (gaussian_splat_model.py:396-410; prune_optimizer :86-108), used by prune_gaussians_with_opt (:412-418)
 * and prune_gaussians (:420-432): drop the rows with prune_mask[i] != 0 from every tensor and its Adam moments (kept
 * rows keep theirs), in row order.  dg_prune_select fills the keep list and n_out (one sync); then
 * dg_densify_gather writes the out_* tensors (nc = ns = 0: every candidate is an original), and
 * dg_prune_gather_stats the kept rows of xyz_gradient_accum / denom (set.grad_accum / set.denom) and max_radii2D
 * (any output may be NULL).  set.grad_accum / denom may be NULL when not gathered. */
int dg_prune_select(dg_densify_args* a, const uint8_t* prune_mask, dg_alloc_fn alloc, void* user,
                    dg_stream_t stream);
int dg_prune_gather_stats(const dg_densify_args* a, const float* max_radii2D, float* out_grad_accum,
                          float* out_denom, float* out_max_radii2D, dg_stream_t stream);

/* ---- export formats of the trained / fused Gaussians ---- */

/* GaussianSplatModel.save_splat (gaussian_splat_model.py:666-708): out [N * 32] device bytes, the .splat records
 * (position f32x3, exp(scale) f32x3, RGBA u8x4, normalised quaternion u8x4) in ascending order of
 * -exp(s0 + s1 + s2) / (1 + exp(opacity)) (stable: equal keys keep index order).  Raw (pre-activation) tensors:
 * xyz [N,3], scaling [N,3], opacity [N,1], rotation [N,4], f_dc [N,1,3].  Allocates DG_BUF_TEMP. */
int dg_splat_pack(uint32_t N, const float* xyz, const float* scaling, const float* opacity, const float* rotation,
                  const float* f_dc, uint8_t* out, dg_alloc_fn alloc, void* user, dg_stream_t stream);
/* GaussianSplatModel.save_ply (gaussian_splat_model.py:616-640): out [N * 27] device bytes, the binary vertex
 * records (x y z f32, nx ny nz = 0, red green blue u8 = the degree-0 SH colour x 255). */
int dg_ply_pack(uint32_t N, const float* xyz, const float* f_dc, uint8_t* out, dg_stream_t stream);

/* ---- the training image path (ImageReader, conerf/base/task_queue.py:89-152) ---- */

/* A ring of `slots` pinned host buffers (max_bytes each) filled by `threads` reader threads with raw u8 HWC images
 * (a decoded cache, e.g. the data section of a .npy file at `offset`).  Completion order, like the reference's
 * image queue.  NULL on failure. */
typedef struct dg_image_ring dg_image_ring;
dg_image_ring* dg_ring_create(int slots, uint64_t max_bytes, int threads);
/* Queue one image: h x w x c bytes (c = 1, 3 or 4) read from `path` at `offset`, tagged `index`. */
int dg_ring_submit(dg_image_ring* ring, const char* path, uint64_t offset, int index, int h, int w, int c);
/* Block until an image is ready: its tag, shape and slot (return 3: the read failed, the slot is released). */
int dg_ring_next(dg_image_ring* ring, int* index, int* h, int* w, int* c, int* slot);
/* Copy the slot's bytes to dev_staging [h*w*c] on `stream` and convert them into out_chw [c', h, w] float
 * (read_image: x / 255; with rgba_composite (its num_channels == 4) an RGBA image is composited over black ->
 * c' = 3, else c' = c).  The slot is reused once the copy completed. */
int dg_ring_upload(dg_image_ring* ring, int slot, int h, int w, int c, int rgba_composite, uint8_t* dev_staging,
                   float* out_chw, dg_stream_t stream);
int dg_ring_pending(dg_image_ring* ring);   /* submitted images not yet taken by dg_ring_next */
void dg_ring_destroy(dg_image_ring* ring);
/* The conversion alone, device to device. */
int dg_image_u8_to_chw(const uint8_t* dev_hwc, int h, int w, int c, int rgba_composite, float* out_chw,
                       dg_stream_t stream);

/* Replaces fusedssim (fused-ssim/ssim.cu:368-404) / fused_ssim_cuda.fusedssim: img [B,CH,H,W];
 * dm_dmu1/dm_dsigma1_sq/dm_dsigma12 NULL <=> train == false. */
int dg_fused_ssim_forward(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                          float* ssim_map, float* dm_dmu1, float* dm_dsigma1_sq, float* dm_dsigma12,
                          dg_stream_t stream);

/* Replaces fusedssim_backward (fused-ssim/ssim.cu:406-444). */
int dg_fused_ssim_backward(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                           const float* dL_dmap, const float* dm_dmu1, const float* dm_dsigma1_sq,
                           const float* dm_dsigma12, float* dL_dimg1, dg_stream_t stream);

/* fused_ssim(img1, img2) with padding "same" (fused_ssim/__init__.py:35-41: FusedSSIMMap(...).mean()) in one pass:
 * *mean (device) = the mean of the SSIM map, which is never written -- per-wave partial sums into part
 * [dg_fused_ssim_parts(B, CH, H, W)] (scratch), totalled in a fixed order and divided by B CH H W (the native training
 * step's SSIM term, bit for bit).  dm_* as dg_fused_ssim_forward (NULL <=> train == false). */
uint32_t dg_fused_ssim_parts(int B, int CH, int H, int W);
int dg_fused_ssim_mean(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                       float* dm_dmu1, float* dm_dsigma1_sq, float* dm_dsigma12, float* part, float* mean,
                       dg_stream_t stream);
/* Its backward: dL/dimg1 for the mean's incoming gradient *dL_dmean (device scalar); dL/dmap = *dL_dmean / (B CH H W),
 * torch's mean backward, is never materialised (the reference path expands it into a full map first). */
int dg_fused_ssim_mean_backward(int B, int CH, int H, int W, const float* img1, const float* img2,
                                const float* dL_dmean, const float* dm_dmu1, const float* dm_dsigma1_sq,
                                const float* dm_dsigma12, float* dL_dimg1, dg_stream_t stream);

/* *out (device) = sum(part[0..n_part)) / denom in a fixed order (strided over 256 threads, the 64-lane sums, then
 * (w0 + w1) + (w2 + w3)): the mean from per-block partial sums, e.g. dg_clamp_l1_forward's (the L1 term). */
int dg_mean_of_parts(const float* part, uint32_t n_part, uint32_t denom, float* out, dg_stream_t stream);

/* Replaces distCUDA2 (simple-knn/spatial.cu:18-35): mean squared distance to the 3 nearest
 * neighbours (approximate, Morton boxes).  out [P].  Allocates DG_BUF_TEMP. */
int dg_dist_cuda2(int P, const float* points, float* out, dg_alloc_fn alloc, void* user, dg_stream_t stream);

/* Bytes of each private state block for P Gaussians / W x H image / K instances (introspection). */
uint64_t dg_geom_bytes(int P);
uint64_t dg_image_bytes(int W, int H);
uint64_t dg_binning_bytes(int64_t K, int W, int H);

/* Bytes dg_rasterize_backward will request as DG_BUF_BACKWARD after a forward that returned num_rendered (the caller can
 * allocate them while the forward's render runs). */
uint64_t dg_backward_scratch_bytes(const dg_raster_args* a, int64_t num_rendered);
/* A dg_alloc_fn over one caller-owned device buffer (user: dg_fixed_buffer*): every request gets ptr when it fits, NULL
 * (an error) when it does not.  Passing this C function instead of a host-language callback takes the allocation
 * round trip out of the call (the drop-in backward prepares its scratch during the forward). */
typedef struct {
    void* ptr;
    uint64_t bytes;
} dg_fixed_buffer;
void* dg_fixed_alloc(void* user, int which, uint64_t nbytes);

/* Introspection of the private forward state, for parity tests (device output pointers):
 * the binned (tile, Gaussian) instance lists -- phase 1 (*e1 entries) then phase 2 (dg_binned_instances - *e1),
 * each grouped by tile in (depth, index) order -- per-Gaussian geometry (tile_count = instances binned for the
 * Gaussian), per-pixel/per-tile image state (ranges = phase 1).  num_rendered: the forward's first return. */
int dg_debug_sorted_instances(const dg_raster_args* a, const void* geom, const void* binning, const void* binning2,
                              const void* image, int64_t num_rendered, int64_t num_instances, uint32_t* tiles_out,
                              uint32_t* gauss_out, int64_t* e1, dg_stream_t stream);
/* Instances actually binned by the last forward on this geometry block: phase 1 + phase 2 (synchronises). */
int dg_binned_instances(const void* geom, int P, int64_t* binned, dg_stream_t stream);
/* The 16 per-view counters of the last forward on this geometry block (synchronises): [0] tile-rect area of the
 * visible Gaussians (u32, saturating), [2..3] num_rendered (u64), [5] phase-1 instances E1, [6] tiles left unfinished
 * by phase 1, [7] phase-2 instances, [8] nonzero when phase 1 was a cut prefix.  Introspection for the bench. */
int dg_debug_counters(const void* geom, int P, uint32_t* counters16, dg_stream_t stream);
/* The adaptive phase-1 capacity (prefix_per_tile == 0) of image size W x H on the current device, in tile-rect
 * units per tile (*per_tile_out, may be NULL); reset != 0 sets it back to its cold default first.  Tests and the
 * bench use it to start a scene cold and to report what the views settled on. */
int dg_adaptive_capacity(int W, int H, int reset, int* per_tile_out);
/* The same for one capacity context (dg_raster_args.capacity_ctx) only; dg_adaptive_capacity resets every context at
 * (device, W, H) and reports context 0. */
int dg_adaptive_capacity_ctx(int ctx, int W, int H, int reset, int* per_tile_out);
/* Drop a capacity context's state and device probes (a trainer that is gone); context 0 is never released.  The
 * probes are freed once no library call is in flight. */
int dg_release_capacity_context(int ctx);
/* Number of capacity contexts that hold a device probe (diagnostics and tests). */
int dg_capacity_contexts(int* n_out);
int dg_debug_geometry(const void* geom, int P, float* means2D, float* conic_opacity, float* rgb_invdepth,
                      uint32_t* tile_count, dg_stream_t stream);
int dg_debug_image_state(const void* image, int W, int H, float* final_T, uint32_t* n_contrib,
                         uint32_t* max_contrib, uint32_t* ranges, dg_stream_t stream);

/* ---- Grid2D block split (load_colmap.py:98-177, cluster.py:73-199) ---- */

/* Axis-aligned 2D boxes [A0, A1, B0, B1] tested in an optional planar frame x' = (T0 x + T1 y) + T2,
 * y' = (T3 x + T4 y) + T5 (trimesh.transform_points of a 3x3 world-to-OBB matrix, rows 0-1). */
#define DG_MAX_BOXES 64
typedef struct {
    uint32_t C;                      /* number of boxes, 1..DG_MAX_BOXES */
    int has_T;                       /* 0: points are tested as given */
    double T[6];
    double box[DG_MAX_BOXES][4];
} dg_box2d_set;
enum { DG_BUF_MEMBERS = 8 };
/* points_in_bbox2D (conerf/datasets/utils.py:186-206) for every box at once, plus Grid2DClustering's labels
 * (cluster.py:173-178: label = the LAST box containing the point, 0 when none).  points: device f64, point i at
 * points[i * stride], points[i * stride + 1].  Optional outputs (NULL = skip): labels u8 [N], transformed f64 [N,2]
 * (the points in the box frame).  counts: host u32 [C], points per box (synchronises once).  When want_members, the
 * concatenated ascending member indices of box 0, 1, ... (u32, counts[k] each) are written to a DG_BUF_MEMBERS
 * buffer.  Allocates DG_BUF_TEMP. */
int dg_points_in_boxes2d(uint32_t N, const double* points, uint32_t stride, const dg_box2d_set* boxes,
                         uint8_t* labels, double* transformed, uint32_t* counts, int want_members, dg_alloc_fn alloc,
                         void* user, dg_stream_t stream);

/* Device primitives used by the rasterizer, exported for tests: stable LSD radix sort of (key, value)
 * pairs over bits [begin_bit, end_bit) in place, and an exclusive scan (total -> *total, device). */
int dg_sort_pairs_u32(uint32_t* keys, uint32_t* vals, uint32_t n, int begin_bit, int end_bit, dg_alloc_fn alloc,
                      void* user, dg_stream_t stream);
int dg_exclusive_scan_u32(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* total, dg_alloc_fn alloc,
                          void* user, dg_stream_t stream);

/* Per-phase hipEvent profiling on the caller's stream (off by default).  collect() synchronises and
 * writes "phase=total_ms/launches;..." for everything recorded since the previous collect. */
void dg_profile_enable(int on);
int dg_profile_collect(char* buf, int buflen);

/* ---- COLMAP binary model readers (host code; the block split's input) ----
 * Replace SceneManager._load_cameras_bin / _load_images_bin / _load_points3D_bin
 * (conerf/pycolmap/pycolmap/scene_manager.py:137-310), called by load_colmap (load_colmap.py:221-226).  Each call
 * maps the file and walks it: with the output arrays NULL it only counts (sizes for the caller), otherwise it fills
 * them.  Return 0, or 1 (cannot open), 2 (truncated), 3 (unknown camera model).
 * cameras: ids [n] u32, models [n] i32, wh [n,2] u64, params8 [n,8] f64 (zero-padded past the model's count). */
int dg_colmap_cameras(const char* path, uint64_t* n, uint32_t* ids, int32_t* models, uint64_t* wh, double* params8);
/* images: ids [n], qt7 [n,7] (qvec w,x,y,z then tvec), camera_ids [n], name_offsets [n+1] into names (no NUL),
 * p2d_offsets [n+1] into xy [m,2] / point3d_ids [m] -- points2D without a 3D point (id -1) dropped as the reference. */
int dg_colmap_images(const char* path, uint64_t* n, uint64_t* name_bytes, uint64_t* n_points2d, uint32_t* ids,
                     double* qt7, uint32_t* camera_ids, uint64_t* name_offsets, char* names, uint64_t* p2d_offsets,
                     double* xy, int64_t* point3d_ids);
/* points3D with track_len >= min_track_length (the reference's default 3): ids [n] u64, xyz [n,3] f64, rgb [n,3] u8,
 * err [n] f64, track_offsets [n+1] into tracks [t,2] u32 (image_id, point2D_idx). */
int dg_colmap_points3d(const char* path, int min_track_length, uint64_t* n, uint64_t* n_track, uint64_t* ids,
                       double* xyz, uint8_t* rgb, double* err, uint64_t* track_offsets, uint32_t* tracks);

const char* dg_last_error(void);
int dg_version(void);
/* Cumulative host time (ns, process-wide) the forward has spent waiting for its one counter read-back (phase 1's
 * num_rendered / cut / error flag, dg_rasterize_forward): the part of a caller's host time per step that is waiting
 * for the GPU rather than work.  Introspection for the bench; no reference counterpart. */
uint64_t dg_host_wait_ns(void);
/* Explicit teardown of the library's process-wide device state before interpreter / runtime exit: waits for the
 * streams it created (the overlapped SH update's side streams), destroys them and their events, frees the adaptive-
 * capacity probes, the pinned counter buffers and the profiling events.  Idempotent; any later call re-creates what it
 * needs.  No reference counterpart (the reference's extension holds no such state); dogs_amd._lib registers it with
 * Python's atexit so nothing of it is alive when the HIP runtime or a profiler tool finalises. */
int dg_shutdown(void);

#ifdef __cplusplus
}
#endif
#endif /* DOGS_HIP_H */
