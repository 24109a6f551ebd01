/*
 * gs_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A plain-C restatement of the reference Taming-3DGS tile rasterizer shipped in
 *   /root/reference/submodules/diff-gaussian-rasterization/cuda_rasterizer/
 * forward and backward, line by line.  It is imported only by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg; the product path
 * (dogs_amd/) never links or calls it.
 *
 * Arithmetic conventions (shared, by construction, with the HIP kernels so that
 * tile/key indexing is bit-exact):
 *   - built with -ffp-contract=off; every a*b+c that nvcc's default --fmad=true
 *     would contract is written as an explicit fmaf() here, innermost product
 *     first, left to right (glm's mat3 product order, type_mat3x3.inl);
 *   - glm matrices are column-major: m[col][row];
 *   - division and sqrt are IEEE correctly rounded (hipcc's default
 *     -fhip-fp32-correctly-rounded-divide-sqrt matches);
 *   - logf() in the precise tile cull (rasterizer_impl.cu:151) is gs_crlogf()
 *     below: the correctly rounded logf, the closest stand-in for CUDA's logf
 *     (<= 1 ulp), evaluated in double by the same operation sequence as the HIP
 *     kernels' (gs_common.h), so oracle and kernels agree bit for bit and both
 *     are correctly rounded on the cull's whole domain (all opacities, checked
 *     exhaustively: gso_crlogf_check, tests/test_oracle_logf.py).  Until round 5
 *     both used a float polynomial (gs_logf_r5 below, kept for the census
 *     gso_logf_census) that is up to 3 ulp off on 7.7% of the opacities;
 *   - float->int conversions saturate (GPU v_cvt_i32_f32 semantics);
 *   - ndc2Pix is evaluated in double, as the reference's double literals imply
 *     (auxiliary.h:40-43).
 * The one non-reproducible op is exp() in compositing (GPU v_exp_f32 vs libm
 * expf); it is the only source of forward image differences.
 *
 * Threads (OpenMP, gso_set_threads): every parallel loop writes disjoint
 * outputs, and every floating-point sum that crosses a parallel loop's items is
 * re-done afterwards in the sequential order (per-instance backward records
 * summed in sorted-instance order, the count-mode score as repeated adds), so
 * the results are bit-identical for any thread count.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#include <limits.h>
#include <omp.h>

#define BLOCK_X 16
#define BLOCK_Y 16
#define BLOCK_SIZE 256
#define NUM_CH 3

/* auxiliary.h:21-38 */
static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;
typedef struct { float m[3][3]; } mat3; /* glm column-major: m[col][row] */

/* ------------------------------------------------------------------ */
/* logf of the precise tile cull                                        */
/* ------------------------------------------------------------------ */
/* Round 5's deterministic float logf (the HIP kernels evaluated the same polynomial).  It is not the reference's:
   on 7.7% of the opacities o in (2^-24, 1] its value of logf(o / (1/255)) is 1-3 ulp away from the correctly
   rounded one.  Kept only for the flip census (gso_logf_census). */
static float gs_logf_r5(float a) {
    if (!(a > 0.0f)) return (a == 0.0f) ? -INFINITY : NAN;
    if (a == INFINITY) return INFINITY;
    uint32_t u; memcpy(&u, &a, 4);
    int e = 0;
    if (u < 0x00800000u) { /* subnormal */
        float b = a * 8388608.0f; memcpy(&u, &b, 4); e = -23;
    }
    e += (int)((u >> 23) & 0xff) - 127;
    uint32_t mu = (u & 0x007fffffu) | 0x3f800000u;
    float m; memcpy(&m, &mu, 4);
    if (m > 1.41421356f) { m = m * 0.5f; e += 1; }
    float s = (m - 1.0f) / (m + 1.0f);
    float s2 = s * s;
    float p = fmaf(s2, 0.22222222f, 0.28571429f);
    p = fmaf(s2, p, 0.4f);
    p = fmaf(s2, p, 0.66666669f);
    p = fmaf(s2, p, 2.0f);
    float lm = s * p;
    return fmaf((float)e, 0.693147182f, lm);
}

/* Correctly rounded logf on the cull's domain (rasterizer_impl.cu:151: logf(co.w / (1/255)), co.w an opacity).
   log(a) = e ln2 + 2 atanh(s), s = (m - 1)/(m + 1), m in [sqrt(1/2), sqrt(2)), in double: the atanh series to
   s^19 (|s| <= 0.1716, truncation < 2^-60 relative), ln2 split hi/lo so e*ln2_hi is exact, then one rounding to
   float.  Every operation is an IEEE double op (+, *, /, fma), so the GPU (gs_common.h, the same sequence) returns
   the same bits.  The double result is within a few double ulps of log(a); on every float a in [2^-20, 256)
   (2.35e8 inputs, a superset of the cull's o * 255) that rounds correctly except for the two inputs below, whose
   exact logarithm lies within 3e-16 of a float midpoint (arbitrated at 80 digits, tests/test_oracle_logf.py). */
float gs_crlogf(float a) {
    if (!(a > 0.0f)) return (a == 0.0f) ? -INFINITY : NAN;
    if (a == INFINITY) return INFINITY;
    if (a == 0x1.827a74p-7f) return -0x1.1c2b1ep+2f;
    if (a == 0x1.2f1fd6p+3f) return 0x1.1fcbcep+1f;
    uint32_t u; memcpy(&u, &a, 4);
    int e = 0;
    if (u < 0x00800000u) { float b = a * 8388608.0f; memcpy(&u, &b, 4); e = -23; }
    e += (int)((u >> 23) & 0xff) - 127;
    uint32_t mu = (u & 0x007fffffu) | 0x3f800000u;
    if (mu > 0x3fb504f3u) { mu -= 0x00800000u; e += 1; }   /* m in [sqrt(1/2), sqrt(2)) */
    float mf; memcpy(&mf, &mu, 4);
    const double m = (double)mf;
    const double s = (m - 1.0) / (m + 1.0);
    const double s2 = s * s;
    double p = fma(s2, 0.10526315789473684, 0.11764705882352941);   /* 2/19, 2/17 */
    p = fma(s2, p, 0.13333333333333333);                            /* 2/15 */
    p = fma(s2, p, 0.15384615384615385);                            /* 2/13 */
    p = fma(s2, p, 0.18181818181818182);                            /* 2/11 */
    p = fma(s2, p, 0.22222222222222222);                            /* 2/9 */
    p = fma(s2, p, 0.2857142857142857);                             /* 2/7 */
    p = fma(s2, p, 0.4);                                            /* 2/5 */
    p = fma(s2, p, 0.6666666666666666);                             /* 2/3 */
    const double lm = fma(s * s2, p, 2.0 * s);
    const double ed = (double)e;
    return (float)fma(ed, 0x1.62e42fefa3800p-1, fma(ed, 0x1.ef35793c76730p-45, lm));
}

/* the cull threshold of n opacities (rasterizer_impl.cu:149-151), the oracle side of dg_cull_log_threshold */
void gso_cull_log_threshold(int64_t n, const float* opacity, float* thr) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) thr[i] = gs_crlogf(opacity[i] / (1.0f / 255.0f));
}

/* Exhaustive check of gs_crlogf against logl (x87 80-bit, rounded once to float) over the float bit patterns
   [lo, hi): returns the number of disagreements and writes up to max_bad of the disagreeing inputs (the caller
   arbitrates them at high precision: logl's own error can misround within ~2^-40 of a midpoint). */
int64_t gso_crlogf_check(uint32_t lo, uint32_t hi, float* bad, int64_t max_bad) {
    int64_t nbad = 0;
#pragma omp parallel for schedule(static, 65536) reduction(+ : nbad)
    for (int64_t i = lo; i < (int64_t)hi; i++) {
        const uint32_t u = (uint32_t)i;
        float x; memcpy(&x, &u, 4);
        if (gs_crlogf(x) != (float)logl((long double)x)) nbad++;
    }
    if (nbad > 0 && max_bad > 0) {   /* second, sequential pass for the (few) inputs themselves, in order */
        int64_t k = 0;
        for (uint32_t u = lo; u < hi && k < max_bad; u++) {
            float x; memcpy(&x, &u, 4);
            if (gs_crlogf(x) != (float)logl((long double)x)) bad[k++] = x;
        }
    }
    return nbad;
}

/* threads of the parallel loops (OpenMP); <= 0 -> all cores.  Results do not depend on it. */
void gso_set_threads(int n) { omp_set_num_threads(n > 0 ? n : omp_get_num_procs()); }
int gso_get_threads(void) { return omp_get_max_threads(); }

/* saturating float -> int, NaN -> 0 (GPU cvt semantics) */
static inline int sat_f2i(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return INT_MAX;
    if (f <= -2147483648.0f) return INT_MIN;
    return (int)f;
}

/* CUDA min()/max() on floats are fminf/fmaxf (NaN-ignoring), as are gfx950 v_min/v_max_f32 */
#define minf_ fminf
#define maxf_ fmaxf

/* ------------------------------------------------------------------ */
/* glm restatements                                                    */
/* ------------------------------------------------------------------ */
static mat3 mat3_cols(float a0, float a1, float a2, float a3, float a4, float a5, float a6,
                      float a7, float a8) {
    mat3 r;
    r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
    r.m[1][0] = a3; r.m[1][1] = a4; r.m[1][2] = a5;
    r.m[2][0] = a6; r.m[2][1] = a7; r.m[2][2] = a8;
    return r;
}
/* glm operator*(mat3, mat3): R[j][i] = A[0][i]*B[j][0] + A[1][i]*B[j][1] + A[2][i]*B[j][2] */
static mat3 mat3_mul(const mat3* A, const mat3* B) {
    mat3 R;
    for (int j = 0; j < 3; j++)
        for (int i = 0; i < 3; i++)
            R.m[j][i] = fmaf(A->m[2][i], B->m[j][2], fmaf(A->m[1][i], B->m[j][1], A->m[0][i] * B->m[j][0]));
    return R;
}
static mat3 mat3_T(const mat3* A) {
    mat3 R;
    for (int j = 0; j < 3; j++)
        for (int i = 0; i < 3; i++) R.m[j][i] = A->m[i][j];
    return R;
}

/* auxiliary.h:69-108 */
static inline v3 tp4x3(v3 p, const float* m) {
    v3 r = {fmaf(m[8], p.z, fmaf(m[4], p.y, m[0] * p.x)) + m[12],
            fmaf(m[9], p.z, fmaf(m[5], p.y, m[1] * p.x)) + m[13],
            fmaf(m[10], p.z, fmaf(m[6], p.y, m[2] * p.x)) + m[14]};
    return r;
}
static inline v4 tp4x4(v3 p, const float* m) {
    v4 r = {fmaf(m[8], p.z, fmaf(m[4], p.y, m[0] * p.x)) + m[12],
            fmaf(m[9], p.z, fmaf(m[5], p.y, m[1] * p.x)) + m[13],
            fmaf(m[10], p.z, fmaf(m[6], p.y, m[2] * p.x)) + m[14],
            fmaf(m[11], p.z, fmaf(m[7], p.y, m[3] * p.x)) + m[15]};
    return r;
}
static inline v3 tv4x3T(v3 p, const float* m) {
    v3 r = {fmaf(m[2], p.z, fmaf(m[1], p.y, m[0] * p.x)),
            fmaf(m[6], p.z, fmaf(m[5], p.y, m[4] * p.x)),
            fmaf(m[10], p.z, fmaf(m[9], p.y, m[8] * p.x))};
    return r;
}
static inline float ndc2Pix(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

/* auxiliary.h:110-143 */
static v3 dnormvdv3(v3 v, v3 dv) {
    float sum2 = fmaf(v.z, v.z, fmaf(v.y, v.y, v.x * v.x));
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    v3 r;
    r.x = ((sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32;
    r.y = (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32;
    r.z = (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32;
    return r;
}

/* ------------------------------------------------------------------ */
/* parameters / state                                                  */
/* ------------------------------------------------------------------ */
typedef struct {
    int P, D, M, W, H;
    int prefiltered, antialiasing;
    float scale_modifier, tanfovx, tanfovy;
    const float* bg;             /* [3] */
    const float* means3D;        /* [P,3] */
    const float* colors;         /* [P,3] or NULL */
    const float* opacities;      /* [P] */
    const float* scales;         /* [P,3] or NULL */
    const float* rotations;      /* [P,4] or NULL */
    const float* cov3D_precomp;  /* [P,6] or NULL */
    const float* viewmatrix;     /* [16] */
    const float* projmatrix;     /* [16] */
    const float* dc;             /* [P,3] */
    const float* sh;             /* [P,M,3] or NULL */
    const float* campos;         /* [3] */
} gso_params;

typedef struct {
    gso_params p;
    int tiles_x, tiles_y, num_tiles;
    float focal_x, focal_y;
    /* geometry (GeometryState, rasterizer_impl.h) */
    float* depths; int* radii; float* means2D; float* cov3D; float* conic_opacity; float* rgb;
    unsigned char* clamped; uint32_t* tiles_touched;
    /* binning */
    int64_t num_rendered; int64_t num_valid;
    uint64_t* keys; uint32_t* vals; /* sorted valid instances */
    uint32_t* ranges;              /* [num_tiles][2] */
    /* image */
    float* final_T; uint32_t* n_contrib; uint32_t* max_contrib; float* pix_color; float* pix_invdepth;
    /* LightGaussian count mode (old forward.cu:481-487): contributing pixels and sum of opacity per Gaussian */
    int32_t* gcount; float* gscore;
    /* samples (SampleState) */
    uint32_t* bucket_offsets; int64_t num_buckets;
    float* sT; float* sar; float* sard;
} gso_ctx;

/* ------------------------------------------------------------------ */
/* forward preprocess (forward.cu:24-276)                               */
/* ------------------------------------------------------------------ */
static v3 sh_to_rgb(int idx, int deg, int max_coeffs, const float* means, v3 campos, const float* dc,
                    const float* shs, unsigned char* clamped) {
    v3 pos = {means[3 * idx], means[3 * idx + 1], means[3 * idx + 2]};
    v3 dir = {pos.x - campos.x, pos.y - campos.y, pos.z - campos.z};
    float len = sqrtf(fmaf(dir.z, dir.z, fmaf(dir.y, dir.y, dir.x * dir.x)));
    dir.x = dir.x / len; dir.y = dir.y / len; dir.z = dir.z / len;
    const float* d0 = dc + 3 * idx;
    const float* sh = shs ? shs + (size_t)idx * max_coeffs * 3 : NULL;
    float basis[15];
    int nb = 0;
    if (deg > 0) {
        float x = dir.x, y = dir.y, z = dir.z;
        basis[0] = -SH_C1 * y; basis[1] = SH_C1 * z; basis[2] = -SH_C1 * x; nb = 3;
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            basis[3] = SH_C2[0] * xy;
            basis[4] = SH_C2[1] * yz;
            basis[5] = SH_C2[2] * (2.0f * zz - xx - yy);
            basis[6] = SH_C2[3] * xz;
            basis[7] = SH_C2[4] * (xx - yy);
            nb = 8;
            if (deg > 2) {
                basis[8] = SH_C3[0] * y * (3.0f * xx - yy);
                basis[9] = SH_C3[1] * xy * z;
                basis[10] = SH_C3[2] * y * (4.0f * zz - xx - yy);
                basis[11] = SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
                basis[12] = SH_C3[4] * x * (4.0f * zz - xx - yy);
                basis[13] = SH_C3[5] * z * (xx - yy);
                basis[14] = SH_C3[6] * x * (xx - 3.0f * yy);
                nb = 15;
            }
        }
    }
    float res[3];
    for (int c = 0; c < 3; c++) {
        float r = SH_C0 * d0[c];
        for (int k = 0; k < nb; k++) r = fmaf(basis[k], sh[3 * k + c], r);
        res[c] = r + 0.5f;
    }
    clamped[3 * idx + 0] = res[0] < 0;
    clamped[3 * idx + 1] = res[1] < 0;
    clamped[3 * idx + 2] = res[2] < 0;
    v3 out = {maxf_(res[0], 0.0f), maxf_(res[1], 0.0f), maxf_(res[2], 0.0f)};
    return out;
}

static void cov3d_fwd(v3 scale, float mod, v4 rot, float* cov3D) {
    mat3 S = mat3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * scale.x; S.m[1][1] = mod * scale.y; S.m[2][2] = mod * scale.z;
    float r = rot.x, x = rot.y, y = rot.z, z = rot.w;
    mat3 R = mat3_cols(fmaf(-2.f, fmaf(y, y, z * z), 1.f), 2.f * fmaf(x, y, -(r * z)), 2.f * fmaf(x, z, r * y),
                       2.f * fmaf(x, y, r * z), fmaf(-2.f, fmaf(x, x, z * z), 1.f), 2.f * fmaf(y, z, -(r * x)),
                       2.f * fmaf(x, z, -(r * y)), 2.f * fmaf(y, z, r * x), fmaf(-2.f, fmaf(x, x, y * y), 1.f));
    mat3 M = mat3_mul(&S, &R);
    mat3 Mt = mat3_T(&M);
    mat3 Sig = mat3_mul(&Mt, &M);
    cov3D[0] = Sig.m[0][0]; cov3D[1] = Sig.m[0][1]; cov3D[2] = Sig.m[0][2];
    cov3D[3] = Sig.m[1][1]; cov3D[4] = Sig.m[1][2]; cov3D[5] = Sig.m[2][2];
}

/* returns T (2 used cols) and cov2D entries, forward.cu:79-114 */
static v3 cov2d_fwd(v3 mean, float fx, float fy, float tfx, float tfy, const float* cov3D,
                    const float* vm, mat3* Tout, mat3* Wout, mat3* Vout, v3* tout, float* xgm, float* ygm) {
    v3 t = tp4x3(mean, vm);
    const float limx = 1.3f * tfx, limy = 1.3f * tfy;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = minf_(limx, maxf_(-limx, txtz)) * t.z;
    t.y = minf_(limy, maxf_(-limy, tytz)) * t.z;
    if (xgm) *xgm = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
    if (ygm) *ygm = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
    float tz2 = t.z * t.z;
    mat3 J = mat3_cols(fx / t.z, 0.0f, -(fx * t.x) / tz2, 0.0f, fy / t.z, -(fy * t.y) / tz2, 0, 0, 0);
    mat3 W = mat3_cols(vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]);
    mat3 T = mat3_mul(&W, &J);
    mat3 V = mat3_cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4], cov3D[5]);
    mat3 Tt = mat3_T(&T), Vt = mat3_T(&V);
    mat3 A = mat3_mul(&Tt, &Vt);
    mat3 cov = mat3_mul(&A, &T);
    if (Tout) *Tout = T;
    if (Wout) *Wout = W;
    if (Vout) *Vout = V;
    if (tout) *tout = t;
    v3 r = {cov.m[0][0], cov.m[0][1], cov.m[1][1]};
    return r;
}

static void get_rect(float px, float py, int r, uint32_t* rmin, uint32_t* rmax, int gx, int gy) {
    /* auxiliary.h:45-55 */
    int a;
    a = sat_f2i((px - (float)r) / (float)BLOCK_X); a = a > 0 ? a : 0; rmin[0] = (uint32_t)(a < gx ? a : gx);
    a = sat_f2i((py - (float)r) / (float)BLOCK_Y); a = a > 0 ? a : 0; rmin[1] = (uint32_t)(a < gy ? a : gy);
    a = sat_f2i((((px + (float)r) + (float)BLOCK_X) - 1.0f) / (float)BLOCK_X); a = a > 0 ? a : 0;
    rmax[0] = (uint32_t)(a < gx ? a : gx);
    a = sat_f2i((((py + (float)r) + (float)BLOCK_Y) - 1.0f) / (float)BLOCK_Y); a = a > 0 ? a : 0;
    rmax[1] = (uint32_t)(a < gy ? a : gy);
}

static int preprocess_one(gso_ctx* c, int idx) {
    const gso_params* p = &c->p;
    c->radii[idx] = 0;
    c->tiles_touched[idx] = 0;
    v3 po = {p->means3D[3 * idx], p->means3D[3 * idx + 1], p->means3D[3 * idx + 2]};
    /* in_frustum, auxiliary.h:150-175 */
    v3 p_view = tp4x3(po, p->viewmatrix);
    if (p_view.z <= 0.2f) return p->prefiltered ? -1 : 0;
    v4 ph = tp4x4(po, p->projmatrix);
    float pw = 1.0f / (ph.w + 0.0000001f);
    v3 pp = {ph.x * pw, ph.y * pw, ph.z * pw};
    const float* cov3D;
    if (p->cov3D_precomp) cov3D = p->cov3D_precomp + 6 * idx;
    else {
        v3 s = {p->scales[3 * idx], p->scales[3 * idx + 1], p->scales[3 * idx + 2]};
        v4 q = {p->rotations[4 * idx], p->rotations[4 * idx + 1], p->rotations[4 * idx + 2], p->rotations[4 * idx + 3]};
        cov3d_fwd(s, p->scale_modifier, q, c->cov3D + 6 * idx);
        cov3D = c->cov3D + 6 * idx;
    }
    v3 cov = cov2d_fwd(po, c->focal_x, c->focal_y, p->tanfovx, p->tanfovy, cov3D, p->viewmatrix, NULL, NULL, NULL,
                       NULL, NULL, NULL);
    const float h_var = 0.3f;
    const float det_cov = fmaf(cov.x, cov.z, -(cov.y * cov.y));
    cov.x += h_var; cov.z += h_var;
    const float det_cov_plus_h_cov = fmaf(cov.x, cov.z, -(cov.y * cov.y));
    float h_scale = 1.0f;
    if (p->antialiasing) h_scale = sqrtf(maxf_(0.000025f, det_cov / det_cov_plus_h_cov));
    const float det = det_cov_plus_h_cov;
    if (det == 0.0f) return 0;
    float det_inv = 1.f / det;
    v3 conic = {cov.z * det_inv, -cov.y * det_inv, cov.x * det_inv};
    float mid = 0.5f * (cov.x + cov.z);
    float disc = sqrtf(maxf_(0.1f, fmaf(mid, mid, -det)));
    float lambda1 = mid + disc, lambda2 = mid - disc;
    float my_radius = ceilf(3.f * sqrtf(maxf_(lambda1, lambda2)));
    float pix_x = ndc2Pix(pp.x, p->W), pix_y = ndc2Pix(pp.y, p->H);
    uint32_t rmin[2], rmax[2];
    get_rect(pix_x, pix_y, sat_f2i(my_radius), rmin, rmax, c->tiles_x, c->tiles_y);
    if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) return 0;
    if (p->colors == NULL) {
        v3 cp = {p->campos[0], p->campos[1], p->campos[2]};
        v3 col = sh_to_rgb(idx, p->D, p->M, p->means3D, cp, p->dc, p->sh, c->clamped);
        c->rgb[3 * idx + 0] = col.x; c->rgb[3 * idx + 1] = col.y; c->rgb[3 * idx + 2] = col.z;
    }
    c->depths[idx] = p_view.z;
    c->radii[idx] = sat_f2i(my_radius);
    c->means2D[2 * idx] = pix_x; c->means2D[2 * idx + 1] = pix_y;
    c->conic_opacity[4 * idx + 0] = conic.x;
    c->conic_opacity[4 * idx + 1] = conic.y;
    c->conic_opacity[4 * idx + 2] = conic.z;
    c->conic_opacity[4 * idx + 3] = p->opacities[idx] * h_scale;
    c->tiles_touched[idx] = (rmax[1] - rmin[1]) * (rmax[0] - rmin[0]);
    return 0;
}

/* rasterizer_impl.cu:52-100 */
static float max_contrib_power_rect(v4 co, float mx, float my, float rminx, float rminy, float rmaxx, float rmaxy) {
    const float PW = 15.0f, PH = 15.0f;
    const float x_min_diff = rminx - mx;
    const float x_left = x_min_diff > 0.0f ? 1.0f : 0.0f;
    const float not_in_x = x_left + (mx > rmaxx ? 1.0f : 0.0f);
    const float y_min_diff = rminy - my;
    const float y_above = y_min_diff > 0.0f ? 1.0f : 0.0f;
    const float not_in_y = y_above + (my > rmaxy ? 1.0f : 0.0f);
    float power = 0.0f;
    if ((not_in_y + not_in_x) > 0.0f) {
        const float px = x_left > 0.0f ? rminx : rmaxx;
        const float py = y_above > 0.0f ? rminy : rmaxy;
        const float dx = copysignf(PW, x_min_diff);
        const float dy = copysignf(PH, y_min_diff);
        const float diffx = mx - px, diffy = my - py;
        const float rcx = 1.0f / (225.0f * co.x);
        const float rcz = 1.0f / (225.0f * co.z);
        float ax = fmaf(dx * co.y, diffy, (dx * co.x) * diffx) * rcx;
        float ay = fmaf(dy * co.z, diffy, (dy * co.y) * diffx) * rcz;
        ax = (ax != ax) ? 0.0f : minf_(maxf_(ax, 0.0f), 1.0f);
        ay = (ay != ay) ? 0.0f : minf_(maxf_(ay, 0.0f), 1.0f);
        const float tx = not_in_y * ax, ty = not_in_x * ay;
        const float qx = fmaf(tx, dx, px), qy = fmaf(ty, dy, py);
        const float ddx = mx - qx, ddy = my - qy;
        /* evaluate_opacity_factor: 0.5*(co.x dx^2 + co.z dy^2) + co.y dx dy */
        power = fmaf(co.y * ddx, ddy, 0.5f * fmaf(co.z * ddy, ddy, (co.x * ddx) * ddx));
    }
    return power;
}

typedef struct { uint64_t key; uint32_t val; } kv_t;
static int kv_cmp(const void* a, const void* b) {
    const kv_t* x = (const kv_t*)a; const kv_t* y = (const kv_t*)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->val < y->val ? -1 : (x->val > y->val);
}

/* ------------------------------------------------------------------ */
/* public API                                                           */
/* ------------------------------------------------------------------ */
void gso_free(gso_ctx* c) {
    if (!c) return;
    free(c->depths); free(c->radii); free(c->means2D); free(c->cov3D); free(c->conic_opacity); free(c->rgb);
    free(c->clamped); free(c->tiles_touched); free(c->keys); free(c->vals); free(c->ranges); free(c->final_T);
    free(c->n_contrib); free(c->max_contrib); free(c->pix_color); free(c->pix_invdepth); free(c->bucket_offsets);
    free(c->gcount); free(c->gscore);
    free(c->sT); free(c->sar); free(c->sard);
    free(c);
}

/* The logf census: preprocess the view as gso_forward does, then walk every rendered
   Gaussian's getRect tiles with the precise cull test (rasterizer_impl.cu:151, 171) under both thresholds: round 5's
   gs_logf_r5 and the correctly rounded gs_crlogf.  out[0] (tile, Gaussian) pairs tested, out[1] kept under gs_crlogf,
   out[2] kept only under gs_logf_r5, out[3] kept only under gs_crlogf, out[4] rendered Gaussians, out[5] of them with a
   different threshold.  Returns 0, or 2 on OOM. */
int gso_logf_census(const gso_params* prm, int64_t* out) {
    gso_ctx* c = (gso_ctx*)calloc(1, sizeof(gso_ctx));
    if (!c) return 2;
    c->p = *prm;
    const int P = prm->P;
    c->focal_y = prm->H / (2.0f * prm->tanfovy);
    c->focal_x = prm->W / (2.0f * prm->tanfovx);
    c->tiles_x = (prm->W + BLOCK_X - 1) / BLOCK_X;
    c->tiles_y = (prm->H + BLOCK_Y - 1) / BLOCK_Y;
    c->num_tiles = c->tiles_x * c->tiles_y;
    size_t Pn = P > 0 ? (size_t)P : 1;
    c->depths = calloc(Pn, 4); c->radii = calloc(Pn, 4); c->means2D = calloc(Pn * 2, 4); c->cov3D = calloc(Pn * 6, 4);
    c->conic_opacity = calloc(Pn * 4, 4); c->rgb = calloc(Pn * 3, 4); c->clamped = calloc(Pn * 3, 1);
    c->tiles_touched = calloc(Pn, 4);
    if (!c->depths || !c->radii || !c->means2D || !c->cov3D || !c->conic_opacity || !c->rgb || !c->clamped ||
        !c->tiles_touched) { gso_free(c); return 2; }
#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; i++) preprocess_one(c, i);
    int64_t tested = 0, kept = 0, only_r5 = 0, only_cr = 0, rendered = 0, thr_diff = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : tested, kept, only_r5, only_cr, rendered, thr_diff)
    for (int idx = 0; idx < P; idx++) {
        if (!(c->radii[idx] > 0)) continue;
        rendered++;
        uint32_t rmin[2], rmax[2];
        const float mx = c->means2D[2 * idx], my = c->means2D[2 * idx + 1];
        get_rect(mx, my, c->radii[idx], rmin, rmax, c->tiles_x, c->tiles_y);
        v4 co = {c->conic_opacity[4 * idx], c->conic_opacity[4 * idx + 1], c->conic_opacity[4 * idx + 2],
                 c->conic_opacity[4 * idx + 3]};
        const float t_cr = gs_crlogf(co.w / (1.0f / 255.0f)), t_r5 = gs_logf_r5(co.w / (1.0f / 255.0f));
        thr_diff += t_cr != t_r5;
        for (uint32_t y = rmin[1]; y < rmax[1]; y++)
            for (uint32_t x = rmin[0]; x < rmax[0]; x++) {
                const float p = max_contrib_power_rect(co, mx, my, (float)(x * BLOCK_X), (float)(y * BLOCK_Y),
                                                       (float)((x + 1) * BLOCK_X - 1), (float)((y + 1) * BLOCK_Y - 1));
                const int a = p <= t_cr, b = p <= t_r5;
                tested++; kept += a; only_r5 += b && !a; only_cr += a && !b;
            }
    }
    out[0] = tested; out[1] = kept; out[2] = only_r5; out[3] = only_cr; out[4] = rendered; out[5] = thr_diff;
    gso_free(c);
    return 0;
}

/* Rasterizer::forward, rasterizer_impl.cu:334-498.  out_color [3,H,W], out_invdepth [H,W], radii [P].
   Returns NULL on error (*err set: 1 = prefiltered violation, 2 = OOM). */
gso_ctx* gso_forward(const gso_params* prm, float* out_color, float* out_invdepth, int* radii_out, int* err) {
    *err = 0;
    gso_ctx* c = (gso_ctx*)calloc(1, sizeof(gso_ctx));
    if (!c) { *err = 2; return NULL; }
    c->p = *prm;
    const int P = prm->P, W = prm->W, H = prm->H;
    c->focal_y = H / (2.0f * prm->tanfovy);
    c->focal_x = W / (2.0f * prm->tanfovx);
    c->tiles_x = (W + BLOCK_X - 1) / BLOCK_X;
    c->tiles_y = (H + BLOCK_Y - 1) / BLOCK_Y;
    c->num_tiles = c->tiles_x * c->tiles_y;
    size_t Pn = P > 0 ? (size_t)P : 1;
    c->depths = calloc(Pn, 4); c->radii = calloc(Pn, 4); c->means2D = calloc(Pn * 2, 4); c->cov3D = calloc(Pn * 6, 4);
    c->conic_opacity = calloc(Pn * 4, 4); c->rgb = calloc(Pn * 3, 4); c->clamped = calloc(Pn * 3, 1);
    c->tiles_touched = calloc(Pn, 4);
    const size_t HW = (size_t)W * H;
    c->final_T = calloc(HW ? HW : 1, 4); c->n_contrib = calloc(HW ? HW : 1, 4);
    c->gcount = calloc(prm->P ? prm->P : 1, 4); c->gscore = calloc(prm->P ? prm->P : 1, 4);
    c->max_contrib = calloc(c->num_tiles ? c->num_tiles : 1, 4);
    c->pix_color = calloc(3 * HW + 1, 4); c->pix_invdepth = calloc(HW + 1, 4);
    c->ranges = calloc(2 * (size_t)(c->num_tiles ? c->num_tiles : 1), 4);
    c->bucket_offsets = calloc(c->num_tiles ? c->num_tiles : 1, 4);

    int pre_err = 0;
#pragma omp parallel for schedule(static) reduction(| : pre_err)
    for (int i = 0; i < P; i++)
        if (preprocess_one(c, i) < 0) pre_err |= 1;
    if (pre_err) { *err = 1; gso_free(c); return NULL; }

    /* inclusive scan of tiles_touched -> num_rendered (rect bound) */
    int64_t total = 0;
    for (int i = 0; i < P; i++) total += c->tiles_touched[i];
    c->num_rendered = total;

    /* duplicateWithKeys (rasterizer_impl.cu:120-190): only valid instances are kept;
       the reference's invalid padding sorts after every valid key and is never read.
       Two passes over the Gaussians (precise count, then emit at the scanned offsets) keep the sequential
       emission order (Gaussian-major, tile rows then columns) whatever the thread count. */
    uint32_t* vcount = (uint32_t*)calloc(Pn, 4);
    int64_t* voff = (int64_t*)malloc(8 * (Pn + 1));
    for (int pass = 0; pass < 2; pass++) {
        if (pass == 1) {
            voff[0] = 0;
            for (int i = 0; i < P; i++) voff[i + 1] = voff[i] + vcount[i];
        }
#pragma omp parallel for schedule(dynamic, 256)
        for (int idx = 0; idx < P; idx++) {
            if (!(c->radii[idx] > 0)) continue;
            uint32_t rmin[2], rmax[2];
            float mx = c->means2D[2 * idx], my = c->means2D[2 * idx + 1];
            get_rect(mx, my, c->radii[idx], rmin, rmax, c->tiles_x, c->tiles_y);
            v4 co = {c->conic_opacity[4 * idx], c->conic_opacity[4 * idx + 1], c->conic_opacity[4 * idx + 2],
                     c->conic_opacity[4 * idx + 3]};
            const float thr = gs_crlogf(co.w / (1.0f / 255.0f));
            uint32_t dbits; memcpy(&dbits, &c->depths[idx], 4);
            int64_t o = pass ? voff[idx] : 0;
            uint32_t cnt = 0;
            for (uint32_t y = rmin[1]; y < rmax[1]; y++)
                for (uint32_t x = rmin[0]; x < rmax[0]; x++) {
                    float p = max_contrib_power_rect(co, mx, my, (float)(x * BLOCK_X), (float)(y * BLOCK_Y),
                                                     (float)((x + 1) * BLOCK_X - 1), (float)((y + 1) * BLOCK_Y - 1));
                    if (p <= thr) {
                        if (pass) {
                            uint64_t key = (uint64_t)(y * c->tiles_x + x);
                            c->keys[o] = (key << 32) | dbits;
                            c->vals[o] = (uint32_t)idx;
                            o++;
                        }
                        cnt++;
                    }
                }
            if (!pass) vcount[idx] = cnt;
        }
        if (pass == 0) {
            int64_t t = 0;
            for (int i = 0; i < P; i++) t += vcount[i];
            c->keys = (uint64_t*)malloc(8 * (size_t)(t ? t : 1));
            c->vals = (uint32_t*)malloc(4 * (size_t)(t ? t : 1));
            c->num_valid = t;
        }
    }
    free(vcount); free(voff);
    const int64_t nv = c->num_valid;
    /* stable LSD sort == lexicographic (tile, depth bits, idx) order: a stable counting sort by tile
       (emission order within a tile is ascending idx), then each tile's run sorted by (depth bits, idx) */
    {
        const int NT = c->num_tiles;
        int64_t* tstart = (int64_t*)calloc((size_t)NT + 1, 8);
        for (int64_t i = 0; i < nv; i++) tstart[(c->keys[i] >> 32) + 1]++;
        for (int t = 0; t < NT; t++) tstart[t + 1] += tstart[t];
        int64_t* fill = (int64_t*)malloc(8 * (size_t)(NT ? NT : 1));
        memcpy(fill, tstart, 8 * (size_t)NT);
        kv_t* kv = (kv_t*)malloc(sizeof(kv_t) * (size_t)(nv ? nv : 1));
        for (int64_t i = 0; i < nv; i++) {
            const int64_t d = fill[c->keys[i] >> 32]++;
            kv[d].key = c->keys[i]; kv[d].val = c->vals[i];
        }
#pragma omp parallel for schedule(dynamic, 16)
        for (int t = 0; t < NT; t++)
            qsort(kv + tstart[t], (size_t)(tstart[t + 1] - tstart[t]), sizeof(kv_t), kv_cmp);
        for (int64_t i = 0; i < nv; i++) { c->keys[i] = kv[i].key; c->vals[i] = kv[i].val; }
        free(kv); free(fill); free(tstart);
    }
    /* identifyTileRanges (rasterizer_impl.cu:195-220), valid keys only */
    for (int64_t i = 0; i < nv; i++) {
        uint32_t t = (uint32_t)(c->keys[i] >> 32);
        if (i == 0 || (uint32_t)(c->keys[i - 1] >> 32) != t) c->ranges[2 * t] = (uint32_t)i;
        if (i == nv - 1 || (uint32_t)(c->keys[i + 1] >> 32) != t) c->ranges[2 * t + 1] = (uint32_t)(i + 1);
    }
    /* perTileBucketCount + scan (rasterizer_impl.cu:223-232, 464-469) */
    int64_t bsum = 0;
    for (int t = 0; t < c->num_tiles; t++) {
        uint32_t n = c->ranges[2 * t + 1] - c->ranges[2 * t];
        bsum += (n + 31) / 32;
        c->bucket_offsets[t] = (uint32_t)bsum;
    }
    c->num_buckets = bsum;
    c->sT = (float*)malloc(4 * (size_t)BLOCK_SIZE * (size_t)(bsum ? bsum : 1));
    c->sar = (float*)malloc(4 * (size_t)BLOCK_SIZE * 3 * (size_t)(bsum ? bsum : 1));
    c->sard = (float*)malloc(4 * (size_t)BLOCK_SIZE * (size_t)(bsum ? bsum : 1));
    if (!c->sT || !c->sar || !c->sard) { *err = 2; gso_free(c); return NULL; }

    /* renderCUDA (forward.cu:349-501): tiles in parallel, pixels of a tile in thread-rank order */
    const float* feat = prm->colors ? prm->colors : c->rgb;
#pragma omp parallel for schedule(dynamic, 4)
    for (int tile = 0; tile < c->num_tiles; tile++) {
        {
            const int ty = tile / c->tiles_x, tx = tile % c->tiles_x;
            const uint32_t r0 = c->ranges[2 * tile], r1 = c->ranges[2 * tile + 1];
            const uint32_t n = r1 - r0;
            const uint32_t bbm0 = tile == 0 ? 0 : c->bucket_offsets[tile - 1];
            uint32_t tile_max = 0;
            for (int tid = 0; tid < BLOCK_SIZE; tid++) {
                const int px = tx * BLOCK_X + (tid % BLOCK_X), py = ty * BLOCK_Y + (tid / BLOCK_X);
                const int inside = px < W && py < H;
                if (!inside) continue;
                const float pfx = (float)px, pfy = (float)py;
                float T = 1.0f, C[3] = {0, 0, 0}, ed = 0.0f;
                uint32_t contributor = 0, last = 0, bbm = bbm0;
                for (uint32_t j = 0; j < n; j++) {
                    if (j % 32 == 0) {
                        c->sT[(size_t)bbm * BLOCK_SIZE + tid] = T;
                        for (int ch = 0; ch < 3; ch++)
                            c->sar[(size_t)bbm * BLOCK_SIZE * 3 + ch * BLOCK_SIZE + tid] = C[ch];
                        c->sard[(size_t)bbm * BLOCK_SIZE + tid] = ed;
                        ++bbm;
                    }
                    contributor++;
                    const uint32_t g = c->vals[r0 + j];
                    const float dx = c->means2D[2 * g] - pfx, dy = c->means2D[2 * g + 1] - pfy;
                    const float* co = c->conic_opacity + 4 * g;
                    const float power = fmaf(-0.5f, fmaf(co[2] * dy, dy, (co[0] * dx) * dx), -((co[1] * dx) * dy));
                    if (power > 0.0f) continue;
                    const float alpha = minf_(0.99f, co[3] * expf(power));
                    if (alpha < 1.0f / 255.0f) continue;
                    const float test_T = T * (1 - alpha);
                    if (test_T < 0.0001f) break; /* done = true */
                    for (int ch = 0; ch < 3; ch++) C[ch] = fmaf(feat[3 * g + ch] * alpha, T, C[ch]);
                    ed = fmaf((1.f / c->depths[g]) * alpha, T, ed);
                    T = test_T;
                    last = contributor;
#pragma omp atomic
                    c->gcount[g]++;            /* gaussian_count[collected_id[j]]++ */
                }
                const size_t pid = (size_t)W * py + px;
                c->final_T[pid] = T;
                c->n_contrib[pid] = last;
                for (int ch = 0; ch < 3; ch++) {
                    float v = fmaf(T, prm->bg[ch], C[ch]);
                    out_color[ch * HW + pid] = v;
                    c->pix_color[ch * HW + pid] = v;
                }
                out_invdepth[pid] = ed;
                c->pix_invdepth[pid] = ed;
                if (last > tile_max) tile_max = last;
            }
            c->max_contrib[tile] = tile_max;
        }
    }
    /* important_score[g] += con_o.w once per contributing pixel: every term of the sum is the same float, so repeated
       adds give the sequential (tile, pixel) order's result exactly */
#pragma omp parallel for schedule(static)
    for (int g = 0; g < P; g++) {
        float sc = 0.0f;
        const float o = c->conic_opacity[4 * g + 3];
        for (int32_t k = 0; k < c->gcount[g]; k++) sc += o;
        c->gscore[g] = sc;
    }
    if (radii_out) memcpy(radii_out, c->radii, 4 * (size_t)P);
    return c;
}

/* ------------------------------------------------------------------ */
/* backward                                                             */
/* ------------------------------------------------------------------ */
typedef struct {
    const float* dL_dpix; const float* dL_dinvdepth;
    float* dmeans2D;  /* [P,3] */
    float* dconic;    /* [P,4] (x,y,-,w) as the reference's float4 view of [P,2,2] */
    float* dopacity;  /* [P] */
    float* dcolors;   /* [P,3] */
    float* dinvdepth; /* [P] */
    float* dmeans3D;  /* [P,3] */
    float* dcov3D;    /* [P,6] */
    float* ddc;       /* [P,3] */
    float* dsh;       /* [P,M,3] */
    float* dscales;   /* [P,3] */
    float* drot;      /* [P,4] */
    float* depth;     /* [P] */
} gso_grads;

/* PerGaussianRenderCUDA (backward.cu:455-658): buckets of 32 splats, per-pixel state from the
   forward samples; lanes visit pixels in order so the per-splat sums run over pixels 0..255. */
static int render_bwd(gso_ctx* c, const gso_grads* g) {
    const gso_params* p = &c->p;
    const int W = p->W, H = p->H;
    const size_t HW = (size_t)W * H;
    const float* colors = p->colors ? p->colors : c->rgb;
    const float ddelx_dx = (float)(0.5 * W), ddely_dy = (float)(0.5 * H);
    /* the 10 sums of each (tile, splat) instance; added into the per-Gaussian gradients below in the sequential
       (tile, bucket, splat) order */
    float* rec = (float*)malloc(sizeof(float) * 10 * (size_t)(c->num_valid ? c->num_valid : 1));
    if (!rec) return 2;
#pragma omp parallel for schedule(dynamic, 4)
    for (int tile = 0; tile < c->num_tiles; tile++) {
        const uint32_t r0 = c->ranges[2 * tile], r1 = c->ranges[2 * tile + 1];
        const int n = (int)(r1 - r0);
        const uint32_t bbm = tile == 0 ? 0 : c->bucket_offsets[tile - 1];
        const int nb = (n + 31) / 32;
        const int tx = tile % c->tiles_x, ty = tile / c->tiles_x;
        for (int b = 0; b < nb; b++) {
            if ((uint32_t)(b * 32) >= c->max_contrib[tile]) break;
            const uint32_t gb = bbm + b;
            float acc[32][10];
            memset(acc, 0, sizeof(acc));
            for (int pix = 0; pix < BLOCK_SIZE; pix++) {
                const int px = tx * BLOCK_X + pix % BLOCK_X, py = ty * BLOCK_Y + pix / BLOCK_X;
                if (px >= W || py >= H) continue;
                const size_t pid = (size_t)W * py + px;
                const uint32_t last = c->n_contrib[pid];
                if ((uint32_t)(b * 32) >= last) continue;
                float T = c->sT[(size_t)gb * BLOCK_SIZE + pix];
                float ar[3], dLp[3];
                for (int ch = 0; ch < 3; ch++) {
                    ar[ch] = -c->pix_color[ch * HW + pid] + c->sar[(size_t)gb * BLOCK_SIZE * 3 + ch * BLOCK_SIZE + pix];
                    dLp[ch] = g->dL_dpix[ch * HW + pid];
                }
                float ard = -c->pix_invdepth[pid] + c->sard[(size_t)gb * BLOCK_SIZE + pix];
                const float T_final = c->final_T[pid];
                const float dLid = g->dL_dinvdepth ? g->dL_dinvdepth[pid] : 0.0f;
                const float pfx = (float)px, pfy = (float)py;
                for (int k = 0; k < 32; k++) {
                    const int sidx = b * 32 + k;
                    if (sidx >= n) break;
                    if ((uint32_t)sidx >= last) break;
                    const uint32_t gi = c->vals[r0 + sidx];
                    const float* co = c->conic_opacity + 4 * gi;
                    const float dx = c->means2D[2 * gi] - pfx, dy = c->means2D[2 * gi + 1] - pfy;
                    const float power = fmaf(-0.5f, fmaf(co[2] * dy, dy, (co[0] * dx) * dx), -((co[1] * dx) * dy));
                    if (power > 0.0f) continue;
                    const float G = expf(power);
                    const float alpha = minf_(0.99f, co[3] * G);
                    if (alpha < 1.0f / 255.0f) continue;
                    const float weight = alpha * T;
                    const float oma_inv = 1.0f / (1.0f - alpha);
                    float bg_dot = 0.0f, dL_dalpha = 0.0f;
                    for (int ch = 0; ch < 3; ch++) {
                        const float cc = colors[3 * gi + ch];
                        ar[ch] = fmaf(weight, cc, ar[ch]);
                        acc[k][6 + ch] = fmaf(weight, dLp[ch], acc[k][6 + ch]);
                        dL_dalpha = fmaf(fmaf(cc, T, oma_inv * ar[ch]), dLp[ch], dL_dalpha);
                        bg_dot = fmaf(p->bg[ch], dLp[ch], bg_dot);
                    }
                    const float invd = 1.f / c->depths[gi];
                    ard = fmaf(weight, invd, ard);
                    acc[k][9] = fmaf(weight, dLid, acc[k][9]);
                    dL_dalpha = fmaf(fmaf(invd, T, oma_inv * ard), dLid, dL_dalpha);
                    dL_dalpha = fmaf(-T_final / (1.0f - alpha), bg_dot, dL_dalpha);
                    T = T * (1.0f - alpha);
                    const float dL_dG = co[3] * dL_dalpha;
                    const float gdx = G * dx, gdy = G * dy;
                    const float dG_ddelx = fmaf(-gdx, co[0], -(gdy * co[1]));
                    const float dG_ddely = fmaf(-gdy, co[2], -(gdx * co[1]));
                    acc[k][0] = fmaf(dL_dG * dG_ddelx, ddelx_dx, acc[k][0]);
                    acc[k][1] = fmaf(dL_dG * dG_ddely, ddely_dy, acc[k][1]);
                    acc[k][2] = fmaf(-0.5f * gdx * dx, dL_dG, acc[k][2]);
                    acc[k][3] = fmaf(-0.5f * gdx * dy, dL_dG, acc[k][3]);
                    acc[k][4] = fmaf(-0.5f * gdy * dy, dL_dG, acc[k][4]);
                    acc[k][5] = fmaf(G, dL_dalpha, acc[k][5]);
                }
            }
            for (int k = 0; k < 32; k++) {
                const int sidx = b * 32 + k;
                if (sidx >= n) break;
                memcpy(rec + 10 * ((size_t)r0 + sidx), acc[k], sizeof(acc[k]));
            }
        }
    }
    for (int tile = 0; tile < c->num_tiles; tile++) {
        const uint32_t r0 = c->ranges[2 * tile], r1 = c->ranges[2 * tile + 1];
        /* the buckets the loop above visited: up to the first that starts at or past the tile's max contributor */
        const uint32_t nbv = (c->max_contrib[tile] + 31) / 32;
        const uint32_t end = r0 + (nbv * 32 < r1 - r0 ? nbv * 32 : r1 - r0);
        for (uint32_t i = r0; i < end; i++) {
            const uint32_t gi = c->vals[i];
            const float* a = rec + 10 * (size_t)i;
            g->dmeans2D[3 * gi + 0] += a[0];
            g->dmeans2D[3 * gi + 1] += a[1];
            g->dconic[4 * gi + 0] += a[2];
            g->dconic[4 * gi + 1] += a[3];
            g->dconic[4 * gi + 3] += a[4];
            g->dopacity[gi] += a[5];
            for (int ch = 0; ch < 3; ch++) g->dcolors[3 * gi + ch] += a[6 + ch];
            g->dinvdepth[gi] += a[9];
        }
    }
    free(rec);
    return 0;
}

static inline float sq(float x) { return x * x; }

/* computeCov2DCUDA (backward.cu:149-326) */
static void cov2d_bwd(gso_ctx* c, const gso_grads* g, int idx) {
    const gso_params* p = &c->p;
    const float* cov3D = p->cov3D_precomp ? p->cov3D_precomp + 6 * idx : c->cov3D + 6 * idx;
    v3 mean = {p->means3D[3 * idx], p->means3D[3 * idx + 1], p->means3D[3 * idx + 2]};
    const float h_x = c->focal_x, h_y = c->focal_y;
    v3 dL_dconic = {g->dconic[4 * idx], g->dconic[4 * idx + 1], g->dconic[4 * idx + 3]};
    mat3 T, W, Vrk; v3 t; float xgm, ygm;
    v3 cv = cov2d_fwd(mean, h_x, h_y, p->tanfovx, p->tanfovy, cov3D, p->viewmatrix, &T, &W, &Vrk, &t, &xgm, &ygm);
    g->depth[idx] = tp4x3(mean, p->viewmatrix).z;
    float c_xx = cv.x, c_xy = cv.y, c_yy = cv.z;
    const float h_var = 0.3f;
    float d_inside_root = 0.f;
    if (p->antialiasing) {
        const float det_cov = fmaf(c_xx, c_yy, -(c_xy * c_xy));
        c_xx += h_var; c_yy += h_var;
        const float det_cov_plus = fmaf(c_xx, c_yy, -(c_xy * c_xy));
        const float hs = sqrtf(maxf_(0.000025f, det_cov / det_cov_plus));
        const float dLo = g->dopacity[idx];
        const float dhs = dLo * p->opacities[idx];
        g->dopacity[idx] = dLo * hs;
        d_inside_root = (det_cov / det_cov_plus) <= 0.000025f ? 0.f : dhs / (2 * hs);
    } else {
        c_xx += h_var; c_yy += h_var;
    }
    float dcxx = 0, dcxy = 0, dcyy = 0;
    if (p->antialiasing) {
        const float x = c_xx, y = c_yy, z = c_xy, w = h_var;
        const float denom_f = d_inside_root / sq(w * w + w * (x + y) + x * y - z * z);
        dcxx = w * (w * y + y * y + z * z) * denom_f;
        dcyy = w * (w * x + x * x + z * z) * denom_f;
        dcxy = -2.f * w * z * (w + x + y) * denom_f;
    }
    const float denom = c_xx * c_yy - c_xy * c_xy;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    float* dcov = g->dcov3D + 6 * idx;
    /* glm T[col][row] */
    const float T00 = T.m[0][0], T01 = T.m[0][1], T02 = T.m[0][2], T10 = T.m[1][0], T11 = T.m[1][1], T12 = T.m[1][2];
    if (denom2inv != 0) {
        dcxx += denom2inv * (-c_yy * c_yy * dL_dconic.x + 2 * c_xy * c_yy * dL_dconic.y + (denom - c_xx * c_yy) * dL_dconic.z);
        dcyy += denom2inv * (-c_xx * c_xx * dL_dconic.z + 2 * c_xx * c_xy * dL_dconic.y + (denom - c_xx * c_yy) * dL_dconic.x);
        dcxy += denom2inv * 2 * (c_xy * c_yy * dL_dconic.x - (denom + 2 * c_xy * c_xy) * dL_dconic.y + c_xx * c_xy * dL_dconic.z);
        dcov[0] = (T00 * T00 * dcxx + T00 * T10 * dcxy + T10 * T10 * dcyy);
        dcov[3] = (T01 * T01 * dcxx + T01 * T11 * dcxy + T11 * T11 * dcyy);
        dcov[5] = (T02 * T02 * dcxx + T02 * T12 * dcxy + T12 * T12 * dcyy);
        dcov[1] = 2 * T00 * T01 * dcxx + (T00 * T11 + T01 * T10) * dcxy + 2 * T10 * T11 * dcyy;
        dcov[2] = 2 * T00 * T02 * dcxx + (T00 * T12 + T02 * T10) * dcxy + 2 * T10 * T12 * dcyy;
        dcov[4] = 2 * T02 * T01 * dcxx + (T01 * T12 + T02 * T11) * dcxy + 2 * T11 * T12 * dcyy;
    } else {
        for (int i = 0; i < 6; i++) dcov[i] = 0;
    }
    const float (*V)[3] = (const float (*)[3])Vrk.m;
    float dT00 = 2 * (T00 * V[0][0] + T01 * V[0][1] + T02 * V[0][2]) * dcxx + (T10 * V[0][0] + T11 * V[0][1] + T12 * V[0][2]) * dcxy;
    float dT01 = 2 * (T00 * V[1][0] + T01 * V[1][1] + T02 * V[1][2]) * dcxx + (T10 * V[1][0] + T11 * V[1][1] + T12 * V[1][2]) * dcxy;
    float dT02 = 2 * (T00 * V[2][0] + T01 * V[2][1] + T02 * V[2][2]) * dcxx + (T10 * V[2][0] + T11 * V[2][1] + T12 * V[2][2]) * dcxy;
    float dT10 = 2 * (T10 * V[0][0] + T11 * V[0][1] + T12 * V[0][2]) * dcyy + (T00 * V[0][0] + T01 * V[0][1] + T02 * V[0][2]) * dcxy;
    float dT11 = 2 * (T10 * V[1][0] + T11 * V[1][1] + T12 * V[1][2]) * dcyy + (T00 * V[1][0] + T01 * V[1][1] + T02 * V[1][2]) * dcxy;
    float dT12 = 2 * (T10 * V[2][0] + T11 * V[2][1] + T12 * V[2][2]) * dcyy + (T00 * V[2][0] + T01 * V[2][1] + T02 * V[2][2]) * dcxy;
    const float (*Wm)[3] = (const float (*)[3])W.m;
    float dJ00 = Wm[0][0] * dT00 + Wm[0][1] * dT01 + Wm[0][2] * dT02;
    float dJ02 = Wm[2][0] * dT00 + Wm[2][1] * dT01 + Wm[2][2] * dT02;
    float dJ11 = Wm[1][0] * dT10 + Wm[1][1] * dT11 + Wm[1][2] * dT12;
    float dJ12 = Wm[2][0] * dT10 + Wm[2][1] * dT11 + Wm[2][2] * dT12;
    float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    float dtx = xgm * -h_x * tz2 * dJ02;
    float dty = ygm * -h_y * tz2 * dJ12;
    float dLid = g->dinvdepth[idx];
    float dtz = -h_x * tz2 * dJ00 - h_y * tz2 * dJ11 + (2 * h_x * t.x) * tz3 * dJ02 + (2 * h_y * t.y) * tz3 * dJ12 - dLid * tz2;
    v3 dm = tv4x3T((v3){dtx, dty, dtz}, p->viewmatrix);
    g->dmeans3D[3 * idx + 0] = dm.x; g->dmeans3D[3 * idx + 1] = dm.y; g->dmeans3D[3 * idx + 2] = dm.z;
}

/* computeColorFromSH backward (backward.cu:23-144) */
static void sh_bwd(gso_ctx* c, const gso_grads* g, int idx) {
    const gso_params* p = &c->p;
    const int deg = p->D, M = p->M;
    v3 pos = {p->means3D[3 * idx], p->means3D[3 * idx + 1], p->means3D[3 * idx + 2]};
    v3 dir_orig = {pos.x - p->campos[0], pos.y - p->campos[1], pos.z - p->campos[2]};
    float len = sqrtf(fmaf(dir_orig.z, dir_orig.z, fmaf(dir_orig.y, dir_orig.y, dir_orig.x * dir_orig.x)));
    v3 dir = {dir_orig.x / len, dir_orig.y / len, dir_orig.z / len};
    const float* sh = p->sh + (size_t)idx * M * 3;
    float dRGB[3];
    for (int ch = 0; ch < 3; ch++) dRGB[ch] = c->clamped[3 * idx + ch] ? 0.0f : g->dcolors[3 * idx + ch];
    float dx[3] = {0, 0, 0}, dy[3] = {0, 0, 0}, dz[3] = {0, 0, 0};
    const float x = dir.x, y = dir.y, z = dir.z;
    float* ddc = g->ddc + 3 * idx;
    float* dsh = g->dsh + (size_t)idx * M * 3;
    for (int ch = 0; ch < 3; ch++) ddc[ch] = SH_C0 * dRGB[ch];
#define SHV(k, ch) sh[3 * (k) + (ch)]
    if (deg > 0) {
        float b1 = -SH_C1 * y, b2 = SH_C1 * z, b3 = -SH_C1 * x;
        for (int ch = 0; ch < 3; ch++) {
            dsh[0 + ch] = b1 * dRGB[ch]; dsh[3 + ch] = b2 * dRGB[ch]; dsh[6 + ch] = b3 * dRGB[ch];
            dx[ch] = -SH_C1 * SHV(2, ch); dy[ch] = -SH_C1 * SHV(0, ch); dz[ch] = SH_C1 * SHV(1, ch);
        }
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            float b4 = SH_C2[0] * xy, b5 = SH_C2[1] * yz, b6 = SH_C2[2] * (2.f * zz - xx - yy), b7 = SH_C2[3] * xz,
                  b8 = SH_C2[4] * (xx - yy);
            for (int ch = 0; ch < 3; ch++) {
                dsh[9 + ch] = b4 * dRGB[ch]; dsh[12 + ch] = b5 * dRGB[ch]; dsh[15 + ch] = b6 * dRGB[ch];
                dsh[18 + ch] = b7 * dRGB[ch]; dsh[21 + ch] = b8 * dRGB[ch];
                dx[ch] += SH_C2[0] * y * SHV(3, ch) + SH_C2[2] * 2.f * -x * SHV(5, ch) + SH_C2[3] * z * SHV(6, ch) + SH_C2[4] * 2.f * x * SHV(7, ch);
                dy[ch] += SH_C2[0] * x * SHV(3, ch) + SH_C2[1] * z * SHV(4, ch) + SH_C2[2] * 2.f * -y * SHV(5, ch) + SH_C2[4] * 2.f * -y * SHV(7, ch);
                dz[ch] += SH_C2[1] * y * SHV(4, ch) + SH_C2[2] * 2.f * 2.f * z * SHV(5, ch) + SH_C2[3] * x * SHV(6, ch);
            }
            if (deg > 2) {
                float b9 = SH_C3[0] * y * (3.f * xx - yy), b10 = SH_C3[1] * xy * z, b11 = SH_C3[2] * y * (4.f * zz - xx - yy),
                      b12 = SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy), b13 = SH_C3[4] * x * (4.f * zz - xx - yy),
                      b14 = SH_C3[5] * z * (xx - yy), b15 = SH_C3[6] * x * (xx - 3.f * yy);
                for (int ch = 0; ch < 3; ch++) {
                    dsh[24 + ch] = b9 * dRGB[ch]; dsh[27 + ch] = b10 * dRGB[ch]; dsh[30 + ch] = b11 * dRGB[ch];
                    dsh[33 + ch] = b12 * dRGB[ch]; dsh[36 + ch] = b13 * dRGB[ch]; dsh[39 + ch] = b14 * dRGB[ch];
                    dsh[42 + ch] = b15 * dRGB[ch];
                    dx[ch] += (SH_C3[0] * SHV(8, ch) * 3.f * 2.f * xy + SH_C3[1] * SHV(9, ch) * yz + SH_C3[2] * SHV(10, ch) * -2.f * xy +
                               SH_C3[3] * SHV(11, ch) * -3.f * 2.f * xz + SH_C3[4] * SHV(12, ch) * (-3.f * xx + 4.f * zz - yy) +
                               SH_C3[5] * SHV(13, ch) * 2.f * xz + SH_C3[6] * SHV(14, ch) * 3.f * (xx - yy));
                    dy[ch] += (SH_C3[0] * SHV(8, ch) * 3.f * (xx - yy) + SH_C3[1] * SHV(9, ch) * xz +
                               SH_C3[2] * SHV(10, ch) * (-3.f * yy + 4.f * zz - xx) + SH_C3[3] * SHV(11, ch) * -3.f * 2.f * yz +
                               SH_C3[4] * SHV(12, ch) * -2.f * xy + SH_C3[5] * SHV(13, ch) * -2.f * yz + SH_C3[6] * SHV(14, ch) * -3.f * 2.f * xy);
                    dz[ch] += (SH_C3[1] * SHV(9, ch) * xy + SH_C3[2] * SHV(10, ch) * 4.f * 2.f * yz +
                               SH_C3[3] * SHV(11, ch) * 3.f * (2.f * zz - xx - yy) + SH_C3[4] * SHV(12, ch) * 4.f * 2.f * xz +
                               SH_C3[5] * SHV(13, ch) * (xx - yy));
                }
            }
        }
    }
#undef SHV
    v3 dL_ddir = {dx[0] * dRGB[0] + dx[1] * dRGB[1] + dx[2] * dRGB[2], dy[0] * dRGB[0] + dy[1] * dRGB[1] + dy[2] * dRGB[2],
                  dz[0] * dRGB[0] + dz[1] * dRGB[1] + dz[2] * dRGB[2]};
    v3 dm = dnormvdv3(dir_orig, dL_ddir);
    g->dmeans3D[3 * idx + 0] += dm.x; g->dmeans3D[3 * idx + 1] += dm.y; g->dmeans3D[3 * idx + 2] += dm.z;
}

/* computeCov3D backward (backward.cu:330-393) */
static void cov3d_bwd(gso_ctx* c, const gso_grads* g, int idx) {
    const gso_params* p = &c->p;
    const float mod = p->scale_modifier;
    const float* q = p->rotations + 4 * idx;
    float r = q[0], x = q[1], y = q[2], z = q[3];
    mat3 R = mat3_cols(fmaf(-2.f, fmaf(y, y, z * z), 1.f), 2.f * fmaf(x, y, -(r * z)), 2.f * fmaf(x, z, r * y),
                       2.f * fmaf(x, y, r * z), fmaf(-2.f, fmaf(x, x, z * z), 1.f), 2.f * fmaf(y, z, -(r * x)),
                       2.f * fmaf(x, z, -(r * y)), 2.f * fmaf(y, z, r * x), fmaf(-2.f, fmaf(x, x, y * y), 1.f));
    v3 s = {mod * p->scales[3 * idx], mod * p->scales[3 * idx + 1], mod * p->scales[3 * idx + 2]};
    mat3 S = mat3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = s.x; S.m[1][1] = s.y; S.m[2][2] = s.z;
    mat3 M = mat3_mul(&S, &R);
    const float* dc = g->dcov3D + 6 * idx;
    mat3 dSig = mat3_cols(dc[0], 0.5f * dc[1], 0.5f * dc[2], 0.5f * dc[1], dc[3], 0.5f * dc[4], 0.5f * dc[2], 0.5f * dc[4], dc[5]);
    mat3 dM = mat3_mul(&M, &dSig);
    for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) dM.m[i][j] *= 2.0f;
    mat3 Rt = mat3_T(&R), dMt = mat3_T(&dM);
    float* dsc = g->dscales + 3 * idx;
    for (int k = 0; k < 3; k++)
        dsc[k] = fmaf(Rt.m[k][2], dMt.m[k][2], fmaf(Rt.m[k][1], dMt.m[k][1], Rt.m[k][0] * dMt.m[k][0]));
    for (int j = 0; j < 3; j++) { dMt.m[0][j] *= s.x; dMt.m[1][j] *= s.y; dMt.m[2][j] *= s.z; }
    const float (*D)[3] = (const float (*)[3])dMt.m;
    float* dq = g->drot + 4 * idx;
    dq[0] = 2 * z * (D[0][1] - D[1][0]) + 2 * y * (D[2][0] - D[0][2]) + 2 * x * (D[1][2] - D[2][1]);
    dq[1] = 2 * y * (D[1][0] + D[0][1]) + 2 * z * (D[2][0] + D[0][2]) + 2 * r * (D[1][2] - D[2][1]) - 4 * x * (D[2][2] + D[1][1]);
    dq[2] = 2 * x * (D[1][0] + D[0][1]) + 2 * r * (D[2][0] - D[0][2]) + 2 * z * (D[1][2] + D[2][1]) - 4 * y * (D[2][2] + D[0][0]);
    dq[3] = 2 * r * (D[0][1] - D[1][0]) + 2 * x * (D[2][0] + D[0][2]) + 2 * y * (D[1][2] + D[2][1]) - 4 * z * (D[1][1] + D[0][0]);
}

/* BACKWARD::preprocessCUDA (backward.cu:399-451) minus SH/cov3D parts */
static void mean2d_bwd(gso_ctx* c, const gso_grads* g, int idx) {
    const float* proj = c->p.projmatrix;
    v3 m = {c->p.means3D[3 * idx], c->p.means3D[3 * idx + 1], c->p.means3D[3 * idx + 2]};
    v4 mh = tp4x4(m, proj);
    float m_w = 1.0f / (mh.w + 0.0000001f);
    float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
    float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
    float gx = g->dmeans2D[3 * idx], gy = g->dmeans2D[3 * idx + 1];
    g->dmeans3D[3 * idx + 0] += (proj[0] * m_w - proj[3] * mul1) * gx + (proj[1] * m_w - proj[3] * mul2) * gy;
    g->dmeans3D[3 * idx + 1] += (proj[4] * m_w - proj[7] * mul1) * gx + (proj[5] * m_w - proj[7] * mul2) * gy;
    g->dmeans3D[3 * idx + 2] += (proj[8] * m_w - proj[11] * mul1) * gx + (proj[9] * m_w - proj[11] * mul2) * gy;
}

/* Rasterizer::backward (rasterizer_impl.cu:555-676).  All gradient arrays must be zeroed by the caller. */
int gso_backward(gso_ctx* c, const float* dL_dpix, const float* dL_dinvdepth, float* dmeans2D, float* dconic,
                 float* dopacity, float* dcolors, float* dinvdepth, float* dmeans3D, float* dcov3D, float* ddc,
                 float* dsh, float* dscales, float* drot, float* depth) {
    gso_grads g = {dL_dpix, dL_dinvdepth, dmeans2D, dconic, dopacity, dcolors, dinvdepth, dmeans3D,
                   dcov3D, ddc, dsh, dscales, drot, depth};
    if (render_bwd(c, &g)) return 2;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < c->p.P; i++) {
        if (!(c->radii[i] > 0)) continue;
        cov2d_bwd(c, &g, i);
    }
#pragma omp parallel for schedule(static)
    for (int i = 0; i < c->p.P; i++) {
        if (!(c->radii[i] > 0)) continue;
        mean2d_bwd(c, &g, i);
        if (c->p.sh) sh_bwd(c, &g, i);
        if (c->p.scales) cov3d_bwd(c, &g, i);
    }
    return 0;
}

/* ---- accessors ---- */
int64_t gso_num_rendered(const gso_ctx* c) { return c->num_rendered; }
int64_t gso_num_valid(const gso_ctx* c) { return c->num_valid; }
int64_t gso_num_buckets(const gso_ctx* c) { return c->num_buckets; }
int gso_num_tiles(const gso_ctx* c) { return c->num_tiles; }
void gso_copy_list(const gso_ctx* c, uint32_t* tiles, uint32_t* idx, uint32_t* depth_bits) {
    for (int64_t i = 0; i < c->num_valid; i++) {
        tiles[i] = (uint32_t)(c->keys[i] >> 32);
        idx[i] = c->vals[i];
        if (depth_bits) depth_bits[i] = (uint32_t)(c->keys[i] & 0xffffffffu);
    }
}
/* count mode outputs (CountGaussiansCUDA, old rasterize_points.cu:148-233): per-Gaussian contributing pixels and
 * the opacity summed over them, in this restatement's sequential (tile, pixel, splat) order */
void gso_copy_counts(const gso_ctx* c, int32_t* count, float* score) {
    memcpy(count, c->gcount, 4 * (size_t)c->p.P);
    memcpy(score, c->gscore, 4 * (size_t)c->p.P);
}
void gso_copy_ranges(const gso_ctx* c, uint32_t* ranges) { memcpy(ranges, c->ranges, 8 * (size_t)c->num_tiles); }
void gso_copy_geom(const gso_ctx* c, float* depths, float* means2D, float* conic, float* rgb, float* cov3D,
                   uint8_t* clamped, uint32_t* tiles_touched) {
    size_t P = (size_t)c->p.P;
    if (depths) memcpy(depths, c->depths, 4 * P);
    if (means2D) memcpy(means2D, c->means2D, 8 * P);
    if (conic) memcpy(conic, c->conic_opacity, 16 * P);
    if (rgb) memcpy(rgb, c->rgb, 12 * P);
    if (cov3D) memcpy(cov3D, c->cov3D, 24 * P);
    if (clamped) memcpy(clamped, c->clamped, 3 * P);
    if (tiles_touched) memcpy(tiles_touched, c->tiles_touched, 4 * P);
}
void gso_copy_image_state(const gso_ctx* c, float* final_T, uint32_t* n_contrib, uint32_t* max_contrib) {
    size_t HW = (size_t)c->p.W * c->p.H;
    if (final_T) memcpy(final_T, c->final_T, 4 * HW);
    if (n_contrib) memcpy(n_contrib, c->n_contrib, 4 * HW);
    if (max_contrib) memcpy(max_contrib, c->max_contrib, 4 * (size_t)c->num_tiles);
}

/* checkFrustum (rasterizer_impl.cu:104-116) */
void gso_mark_visible(int P, const float* means3D, const float* view, const float* proj, uint8_t* present) {
    (void)proj;
    for (int i = 0; i < P; i++) {
        v3 po = {means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]};
        present[i] = tp4x3(po, view).z > 0.2f;
    }
}

/* filter_preprocessCUDA (forward.cu:279-344): radii only, no low-pass */
void gso_filter_radii(const gso_params* p, int* radii) {
    const float fy = p->H / (2.0f * p->tanfovy), fx = p->W / (2.0f * p->tanfovx);
    const int gx = (p->W + BLOCK_X - 1) / BLOCK_X, gy = (p->H + BLOCK_Y - 1) / BLOCK_Y;
    for (int idx = 0; idx < p->P; idx++) {
        radii[idx] = 0;
        v3 po = {p->means3D[3 * idx], p->means3D[3 * idx + 1], p->means3D[3 * idx + 2]};
        if (tp4x3(po, p->viewmatrix).z <= 0.2f) continue;
        v4 ph = tp4x4(po, p->projmatrix);
        float pw = 1.0f / (ph.w + 0.0000001f);
        float cov3[6];
        const float* cov3D;
        if (p->cov3D_precomp) cov3D = p->cov3D_precomp + 6 * idx;
        else {
            v3 s = {p->scales[3 * idx], p->scales[3 * idx + 1], p->scales[3 * idx + 2]};
            v4 q = {p->rotations[4 * idx], p->rotations[4 * idx + 1], p->rotations[4 * idx + 2], p->rotations[4 * idx + 3]};
            cov3d_fwd(s, p->scale_modifier, q, cov3);
            cov3D = cov3;
        }
        v3 cov = cov2d_fwd(po, fx, fy, p->tanfovx, p->tanfovy, cov3D, p->viewmatrix, NULL, NULL, NULL, NULL, NULL, NULL);
        float det = fmaf(cov.x, cov.z, -(cov.y * cov.y));
        if (det == 0.0f) continue;
        float mid = 0.5f * (cov.x + cov.z);
        float disc = sqrtf(maxf_(0.1f, fmaf(mid, mid, -det)));
        float my_radius = ceilf(3.f * sqrtf(maxf_(mid + disc, mid - disc)));
        uint32_t rmin[2], rmax[2];
        get_rect(ndc2Pix(ph.x * pw, p->W), ndc2Pix(ph.y * pw, p->H), sat_f2i(my_radius), rmin, rmax, gx, gy);
        if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) continue;
        radii[idx] = sat_f2i(my_radius);
    }
}

/* adamUpdateCUDA (adam.cu:10-38) */
void gso_adam(float* param, const float* grad, float* m, float* v, const uint8_t* visible, float lr, float b1, float b2,
              float eps, uint32_t N, uint32_t M) {
#pragma omp parallel for schedule(static)
    for (uint64_t i = 0; i < (uint64_t)N * M; i++) {
        if (!visible[i / M]) continue;
        float gr = grad[i];
        float em = fmaf(b1, m[i], (1.0f - b1) * gr);
        float ev = fmaf(b2, v[i], ((1.0f - b2) * gr) * gr);
        float step = -lr * em / (sqrtf(ev) + eps);
        param[i] += step;
        m[i] = em; v[i] = ev;
    }
}
