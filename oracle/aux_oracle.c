/*
 * aux_oracle.c -- TEST INFRASTRUCTURE ONLY.
 * CPU restatements of the two satellite kernels of the hot path:
 *   fused-ssim      /root/reference/submodules/fused-ssim/ssim.cu:36-307
 *   simple-knn      /root/reference/submodules/simple-knn/simple_knn.cu:45-221
 * Same arithmetic conventions as gs_oracle.c (-ffp-contract=off, explicit fmaf where
 * nvcc contracts a*b+c).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

/* ssim.cu:9-19 */
static const float GW[11] = {0.001028380123898387f, 0.0075987582094967365f, 0.036000773310661316f,
                             0.10936068743467331f, 0.21300552785396576f, 0.26601171493530273f,
                             0.21300552785396576f, 0.10936068743467331f, 0.036000773310661316f,
                             0.0075987582094967365f, 0.001028380123898387f};

/* get_pix_value (ssim.cu:36-42): zero outside the image */
static inline float pix(const float* img, int y, int x, int H, int W) {
    return (x >= W || y >= H || x < 0 || y < 0) ? 0.0f : img[(size_t)y * W + x];
}

/* separable 11x11 conv of f(img) at (y,x): x-pass per source row then y-pass, the kernel's order
   (do_separable_conv_x / do_separable_conv_y). mode 0: a, 1: a*a, 2: a*b */
static float conv2(const float* a, const float* b, int mode, int y, int x, int H, int W) {
    float v = 0.0f;
    for (int ky = 0; ky < 11; ky++) {
        const int yy = y - 5 + ky;
        float h = 0.0f;
        for (int kx = 0; kx < 11; kx++) {
            const int xx = x - 5 + kx;
            float s = pix(a, yy, xx, H, W);
            if (mode == 1) s = s * s;
            else if (mode == 2) s = s * pix(b, yy, xx, H, W);
            h = fmaf(GW[kx], s, h);
        }
        v = fmaf(GW[ky], h, v);
    }
    return v;
}

/* fusedssimCUDA (ssim.cu:187-286). img [B,CH,H,W]; dm_* may be NULL (train=false). */
void aux_ssim_fwd(int B, int CH, int H, int W, float C1, float C2, const float* img1, const float* img2,
                  float* map, float* dm_dmu1, float* dm_dsigma1_sq, float* dm_dsigma12) {
    const size_t HW = (size_t)H * W;
    for (int b = 0; b < B; b++)
        for (int c = 0; c < CH; c++) {
            const float* i1 = img1 + ((size_t)b * CH + c) * HW;
            const float* i2 = img2 + ((size_t)b * CH + c) * HW;
            for (int y = 0; y < H; y++)
                for (int x = 0; x < W; x++) {
                    const float mu1 = conv2(i1, NULL, 0, y, x, H, W);
                    const float sigma1_sq = fmaf(-mu1, mu1, conv2(i1, NULL, 1, y, x, H, W));
                    const float mu2 = conv2(i2, NULL, 0, y, x, H, W);
                    const float sigma2_sq = fmaf(-mu2, mu2, conv2(i2, NULL, 1, y, x, H, W));
                    const float sigma12 = fmaf(-mu1, mu2, conv2(i1, i2, 2, y, x, H, W));
                    const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
                    const float Cc = fmaf(2.0f, mu1_mu2, C1);
                    const float D = fmaf(2.0f, sigma12, C2);
                    const float A = (mu1_sq + mu2_sq) + C1;
                    const float Bb = (sigma1_sq + sigma2_sq) + C2;
                    const float m = (Cc * D) / (A * Bb);
                    const size_t gi = ((size_t)b * CH + c) * HW + (size_t)y * W + x;
                    map[gi] = m;
                    if (dm_dmu1) {
                        dm_dmu1[gi] = ((mu2 * 2.0f * D) / (A * Bb) - (mu2 * 2.0f * Cc) / (A * Bb) -
                                       (mu1 * 2.0f * Cc * D) / (A * A * Bb) + (mu1 * 2.0f * Cc * D) / (A * Bb * Bb));
                        dm_dsigma1_sq[gi] = ((-Cc * D) / (A * Bb * Bb));
                        dm_dsigma12[gi] = ((2 * Cc) / (A * Bb));
                    }
                }
        }
}

/* fusedssim_backwardCUDA (ssim.cu:288-366) */
void aux_ssim_bwd(int B, int CH, int H, int W, const float* img1, const float* img2, const float* dL_dmap,
                  const float* dm_dmu1, const float* dm_dsigma1_sq, const float* dm_dsigma12, float* dL_dimg1) {
    const size_t HW = (size_t)H * W;
    for (int b = 0; b < B; b++)
        for (int c = 0; c < CH; c++) {
            const size_t off = ((size_t)b * CH + c) * HW;
            const float *dl = dL_dmap + off, *a = dm_dmu1 + off, *s = dm_dsigma1_sq + off, *x12 = dm_dsigma12 + off;
            for (int y = 0; y < H; y++)
                for (int x = 0; x < W; x++) {
                    const float p1 = img1[off + (size_t)y * W + x], p2 = img2[off + (size_t)y * W + x];
                    float d = conv2(a, dl, 2, y, x, H, W);
                    d += (p1 * 2.0f) * conv2(s, dl, 2, y, x, H, W);
                    d += p2 * conv2(x12, dl, 2, y, x, H, W);
                    dL_dimg1[off + (size_t)y * W + x] = d;
                }
        }
}

/* ---------------- simple-knn ---------------- */
static uint32_t prepMorton(uint32_t x) {
    x = (x | (x << 16)) & 0x030000FF;
    x = (x | (x << 8)) & 0x0300F00F;
    x = (x | (x << 4)) & 0x030C30C3;
    x = (x | (x << 2)) & 0x09249249;
    return x;
}
/* float -> uint32 with GPU cvt_u32 semantics: NaN/negative -> 0, saturate high */
static inline uint32_t sat_f2u(float f) {
    if (!(f > 0.0f)) return 0;
    if (f >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)f;
}
uint32_t aux_morton(const float* p, const float* mn, const float* mx) {
    uint32_t c[3];
    for (int k = 0; k < 3; k++) c[k] = prepMorton(sat_f2u(((p[k] - mn[k]) / (mx[k] - mn[k])) * 1023.0f));
    return c[0] | (c[1] << 1) | (c[2] << 2);
}

typedef struct { uint32_t code, idx; } mc_t;
static int mc_cmp(const void* a, const void* b) {
    const mc_t* x = (const mc_t*)a; const mc_t* y = (const mc_t*)b;
    if (x->code != y->code) return x->code < y->code ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}
static inline void update3(const float* ref, const float* pt, float* best) {
    float dx = pt[0] - ref[0], dy = pt[1] - ref[1], dz = pt[2] - ref[2];
    float dist = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
    for (int j = 0; j < 3; j++)
        if (best[j] > dist) { float t = best[j]; best[j] = dist; dist = t; }
}
static inline float box_dist(const float* mn, const float* mx, const float* p) {
    float d[3] = {0, 0, 0};
    for (int k = 0; k < 3; k++)
        if (p[k] < mn[k] || p[k] > mx[k]) {
            float a = fabsf(p[k] - mn[k]), b = fabsf(p[k] - mx[k]);
            d[k] = a < b ? a : b;
        }
    return fmaf(d[2], d[2], fmaf(d[1], d[1], d[0] * d[0]));
}

/* SimpleKNN::knn (simple_knn.cu:185-221); out[P]; also returns the sorted order if order != NULL */
int aux_knn(int P, const float* pts, float* out, uint32_t* order) {
    const int BOX = 1024;
    float mn[3] = {0, 0, 0}, mx[3] = {0, 0, 0}; /* reduction init {0,0,0} (:191) */
    for (int i = 0; i < P; i++)
        for (int k = 0; k < 3; k++) {
            float v = pts[3 * i + k];
            if (v < mn[k]) mn[k] = v;
            if (v > mx[k]) mx[k] = v;
        }
    mc_t* mc = (mc_t*)malloc(sizeof(mc_t) * (size_t)(P ? P : 1));
    if (!mc) return -1;
    for (int i = 0; i < P; i++) { mc[i].code = aux_morton(pts + 3 * i, mn, mx); mc[i].idx = (uint32_t)i; }
    qsort(mc, (size_t)P, sizeof(mc_t), mc_cmp);
    const int nb = (P + BOX - 1) / BOX;
    float* bmin = (float*)malloc(sizeof(float) * 3 * (size_t)(nb ? nb : 1));
    float* bmax = (float*)malloc(sizeof(float) * 3 * (size_t)(nb ? nb : 1));
    for (int b = 0; b < nb; b++) {
        for (int k = 0; k < 3; k++) { bmin[3 * b + k] = FLT_MAX; bmax[3 * b + k] = -FLT_MAX; }
        for (int i = b * BOX; i < P && i < (b + 1) * BOX; i++)
            for (int k = 0; k < 3; k++) {
                float v = pts[3 * mc[i].idx + k];
                if (v < bmin[3 * b + k]) bmin[3 * b + k] = v;
                if (v > bmax[3 * b + k]) bmax[3 * b + k] = v;
            }
    }
    /* every point's search is independent and writes its own slot: threads change nothing in the result */
#pragma omp parallel for schedule(dynamic, 256)
    for (int idx = 0; idx < P; idx++) {
        const float* pt = pts + 3 * mc[idx].idx;
        float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
        int lo = idx - 3 > 0 ? idx - 3 : 0, hi = idx + 3 < P - 1 ? idx + 3 : P - 1;
        for (int i = lo; i <= hi; i++) if (i != idx) update3(pt, pts + 3 * mc[i].idx, best);
        const float reject = best[2];
        best[0] = best[1] = best[2] = FLT_MAX;
        for (int b = 0; b < nb; b++) {
            float d = box_dist(bmin + 3 * b, bmax + 3 * b, pt);
            if (d > reject || d > best[2]) continue;
            for (int i = b * BOX; i < P && i < (b + 1) * BOX; i++)
                if (i != idx) update3(pt, pts + 3 * mc[i].idx, best);
        }
        out[mc[idx].idx] = (best[0] + best[1] + best[2]) / 3.0f;
    }
    if (order) for (int i = 0; i < P; i++) order[i] = mc[i].idx;
    free(mc); free(bmin); free(bmax);
    return 0;
}
