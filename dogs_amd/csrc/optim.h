// optim.h -- the optimizer side of a training view:
//   * SparseGaussianAdam over all parameter groups in one launch (adam.cu:10-38 per group), with the densification
//     statistics of the same view (gaussian_trainer.py:433-438, gaussian_splat_model.py:533-541) folded in;
//   * densify_and_prune (gaussian_splat_model.py:434-531) as GPU stream compaction: selection, one candidate pass
//     over [originals not split | clones | split children], one gather of every parameter and Adam moment.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gs {

constexpr int MAX_ADAM_GROUPS = 8;

struct AdamGroup {
    float* param;
    const float* grad;
    float* m;
    float* v;
    float lr, eps;
    uint32_t M;       // floats per Gaussian
    uint32_t vec;     // 1: param/grad/m/v (and u/z) 16-byte aligned (float4 path)
    // optional ADMM proximal term 0.5 rho mse(x + u, z): gradient coef ((x + u) - z), coef = rho / numel
    const float* u;
    const float* z;
    float coef;
    // optional activation backward folded in (the native training step): grad is dL/d(activated parameter) and the
    // update sees dL/d(raw parameter) -- 0: grad as given; 1: sigmoid (act = sigmoid(raw), M = 1); 2: exp plus the
    // scale regulariser reg * prod(scaling) (act = exp(raw), M = 3); 3: F.normalize (the raw quaternion is param, M = 4)
    int gmode;
    const float* act;
    float reg;
    // gmode 2: *zero_stamp == stamp when any scaling of the step is exactly 0 (written by the activation pass); torch's
    // prod backward then takes its zero-safe form for EVERY row, so the regulariser's gradient does too
    const uint64_t* zero_stamp;
    uint64_t stamp;
};

struct AdamMultiArgs {
    AdamGroup g[MAX_ADAM_GROUPS];
    uint32_t start[MAX_ADAM_GROUPS + 2];  // first work item of group k (items = 4-float chunks); start[n] = stats
    int n;
    const uint8_t* visible;  // [N]; NULL: visible = vis_radii > 0
    const int* vis_radii;    // [N]
    uint32_t N;
    float b1, b2;
    // densification statistics (optional: radii == nullptr)
    const int* radii;          // [N]
    const float* dmeans2D;     // [N, stride] screen-space gradient (x, y used)
    uint32_t dm_stride;
    float* max_radii2D;        // [N]
    float* grad_accum;         // [N]
    float* denom;              // [N]
    // optional (depth_thr > 0): geometry.depth_threshold -- the screen-space gradient the statistics read is scaled by
    // min(1, (depth[i] / depth_thr)^2) first (_RasterizeGaussians.backward's scale_tensor, gaussian_trainer.py:376)
    const float* depth;        // [N] view-space depth (the rasterizer backward's depth output)
    float depth_thr;
    // optional: hot[i] != 0 marks the rows that may carry a rasterizer gradient (the binned Gaussians, rcnt > 0);
    // a 4-float chunk touching no hot row takes its incoming gradient as zero without reading it (the native step,
    // where the activation fold supplies the regulariser's gradient of every row)
    const uint32_t* hot;
    // optional (the native step's overlapped update, dg_train_step_args::sh_status): status_out[i] = visible | hot << 1
    // written for every row by the row blocks; a launch given `status` reads its rows' visibility and hot flag there
    // instead of visible / vis_radii / hot (the next step's forward overwrites those while the launch may still run)
    uint8_t* status_out;
    const uint8_t* status;
    uint32_t grid_cap;   // optional: at most this many blocks, striding over the work (0: one block per work block)
    uint32_t nblocks;    // set by launch_adam_multi
};
void launch_adam_multi(const AdamMultiArgs& a, hipStream_t s);
uint32_t clamp_l1_blocks(uint32_t n);
void launch_clamp_l1_fwd(uint32_t n, const float* img, const float* gt, float* out, float* partial, hipStream_t s);
void launch_row_prod_fwd(uint32_t N, uint32_t M, const float* x, float* prod, uint32_t* zero_stamp, uint32_t stamp,
                         hipStream_t s);
void launch_row_prod_bwd(uint32_t N, uint32_t M, const float* x, const float* prod, const float* dprod,
                         const uint32_t* zero_stamp, uint32_t stamp, float* dx, hipStream_t s);
void launch_clamp_l1_bwd(uint32_t n, const float* img, const float* clamped, const float* gt, const float* g_img,
                         const float* g_l1, float* d_img, hipStream_t s, float g_l1_value = 0.0f);
uint32_t block_sum_blocks(uint32_t n);
void launch_block_sum(const float* x, uint32_t n, int mode, float* partial, hipStream_t s);
void launch_loss_final(const float* p_l1, uint32_t n_l1, const float* p_ssim, uint32_t n_ssim, const float* p_sc,
                       uint32_t n_sc, uint32_t n_img, uint32_t P, float* loss, hipStream_t s);
void launch_activate_fwd(uint32_t N, const float* ro, const float* rs, const float* rq, float* o, float* sc, float* q,
                         uint64_t* zero_stamp, uint64_t stamp,
                         hipStream_t s);
void launch_activate_bwd(uint32_t N, const float* o, const float* sc, const float* rq, const float* go,
                         const float* gsc, const float* gq, float* dro, float* drs, float* drq, hipStream_t s,
                         float scale_reg = 0.0f, const uint64_t* zero_stamp = nullptr, uint64_t stamp = 0);

// ---- densify_and_prune
struct DensifyArgs {
    uint32_t N;
    // parameters (raw, as stored by the model) and their Adam moments (m/v may be null: no optimizer state)
    const float *xyz, *f_dc, *f_rest, *opacity, *scaling, *rot;
    const float *m[6], *v[6];
    uint32_t width[6];         // floats per Gaussian: xyz 3, f_dc 3*, f_rest 3*(M), opacity 1, scaling 3, rot 4
    const float* grad_accum;   // [N]
    const float* denom;        // [N]
    float grad_threshold, dense_extent;  // max_grad, percent_dense * extent
    // selection outputs (device scratch, 0/1 per original)
    uint32_t* clone_flag;      // [N]
    uint32_t* split_flag;      // [N]
};
struct RebuildArgs {
    DensifyArgs d;
    uint32_t nc, ns, replicas;
    const uint32_t* clone_idx;  // [nc]
    const uint32_t* split_idx;  // [ns]
    const float* samples;       // [replicas * ns, 3]
    float min_opacity;
    int use_bbox;
    float bbox_z;
    int use_screen;             // max_screen_size is not None
    float max_screen, big_extent;  // max_screen_size, 0.1 * extent
    uint32_t* keep;             // [C] 0/1 per candidate row
    // outputs: [Nf, width] each
    float* out_p[6];
    float* out_m[6];
    float* out_v[6];
};
// clone/split flags (0/1) of every original Gaussian
void launch_densify_select(const DensifyArgs& a, hipStream_t s);
// clone_idx / split_idx from the scanned flags
void launch_densify_lists(const DensifyArgs& a, const uint32_t* clone_pos, const uint32_t* split_pos,
                          uint32_t* clone_idx, uint32_t* split_idx, hipStream_t s);
// keep flags of the candidates (C = N + nc + replicas * ns)
void launch_densify_keep(const RebuildArgs& a, hipStream_t s);
// gather of the kept candidates into out_* (positions = scanned keep)
void launch_densify_gather(const RebuildArgs& a, const uint32_t* keep_pos, hipStream_t s);

}  // namespace gs
