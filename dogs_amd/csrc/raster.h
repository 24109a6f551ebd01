// raster.h -- kernel argument blocks and launchers of the gfx950 rasterizer (raster_fwd.hip, raster_bwd.hip)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gs {

// Splat record: everything binning and compositing read per Gaussian, in ONE 32-B record so a
// depth-ordered or instance-ordered gather touches one cache line instead of one per array.
//   sp[2g]     = {mean2D.x, mean2D.y, conic.a, conic.b}
//   sp[2g + 1] = {conic.c, opacity * AA scale, bits(x0 | x1 << 16), bits(y0 | y1 << 16)}   (tile rect)
__device__ __forceinline__ void sp_rect(const float4& s1, int& x0, int& y0, int& x1, int& y1) {
    const uint32_t rx = __float_as_uint(s1.z), ry = __float_as_uint(s1.w);
    x0 = (int)(rx & 0xffffu); x1 = (int)(rx >> 16); y0 = (int)(ry & 0xffffu); y1 = (int)(ry >> 16);
}

struct PreArgs {
    int P, D, M, W, H, tiles_x, tiles_y;
    int antialiasing, prefiltered;
    float tanfovx, tanfovy, focal_x, focal_y, scale_mod;
    const float *means3D, *scales, *rotations, *opacities, *dc, *sh, *colors, *cov3D_precomp;
    const float *view, *proj, *campos;
    int* radii;
    float4* sp;         // splat record, 2 x float4 per Gaussian (see SP_* below)
    float4* rgbi;       // rgb, 1 / view z
    uint32_t* depthkey; // float bits of view z, 0xffffffff when no tile survives the precise cull
    uint32_t* cnt;      // precise tile count
    unsigned long long* rect_sum;  // num_rendered of the reference (sum of rect areas)
    uint32_t* err;
};

struct RenderArgs {
    int W, H, tiles_x, num_tiles;
    uint32_t K, P;          // bounds of s_e/eg and of the geometry arrays
    const uint2* ranges;
    const uint32_t* s_e;   // sorted instance -> emission index
    const uint32_t* eg;    // emission index -> Gaussian
    const float4* sp;
    const float4* rgbi;
    const float* bg;
    float *out_color, *out_invd, *final_T, *img_color, *img_invd;
    uint32_t *n_contrib, *max_contrib;
};

struct RenderBwdArgs {
    int W, H, tiles_x, num_tiles;
    uint32_t K, P;
    const uint2* ranges;
    const uint32_t* max_contrib;
    const uint32_t* s_e;
    const uint32_t* eg;
    const float4* sp;
    const float4* rgbi;
    const float* bg;
    const float *final_T, *img_color, *img_invd;
    const uint32_t* n_contrib;
    const float* dL_dpix;
    const float* dL_dinvd;   // may be null
    float* rec;              // [K][12] per-instance gradient record
    uint8_t* flag;           // [K] record written
    const uint32_t* invd_nonzero;  // device flag: any(dL_dinvd != 0)
};

struct GaussBwdArgs {
    int P, D, M, W, H, antialiasing;
    uint32_t K;
    float tanfovx, tanfovy, focal_x, focal_y, scale_mod;
    const float *means3D, *scales, *rotations, *opacities, *dc, *sh, *cov3D_precomp;
    const float *view, *proj, *campos;
    const int* radii;
    const uint32_t* cnt;
    const uint32_t* first_e;
    const float4* sp;        // splat records (conic + AA-scaled opacity)
    const float* rec;
    const uint8_t* flag;
    float4* sums;            // [P][3] record sums (k_record_sum -> k_gauss_bwd)
    float *dmeans2D, *dcolors, *dopacity, *dmeans3D, *dcov3D, *ddc, *dsh, *dscales, *drot, *depth;
};

void launch_preprocess(const PreArgs& a, hipStream_t s);
void launch_emit(int P, const uint32_t* order, const uint32_t* skey, const uint32_t* off, const float4* sp,
                 int tiles_x, uint32_t* first_e, uint32_t* tilekey, uint32_t* eg, hipStream_t s);
void launch_ranges(uint32_t K, const uint32_t* keys, uint2* ranges, uint32_t num_tiles, hipStream_t s);
void launch_render_fwd(const RenderArgs& a, hipStream_t s);
void launch_mark_visible(int P, const float* means3D, const float* view, bool* present, hipStream_t s);
void launch_filter(const PreArgs& a, hipStream_t s);
void launch_render_bwd(const RenderBwdArgs& a, uint32_t* invd_flag, hipStream_t s);
void launch_record_sum(const GaussBwdArgs& a, hipStream_t s);
void launch_gauss_bwd(const GaussBwdArgs& a, hipStream_t s);

}  // namespace gs
