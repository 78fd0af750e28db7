/*
 * vr_oracle.c -- CPU restatement of the reference d_render path
 * (ykou/Volume-Rendering-Based-on-Distribution-Data, volumeRender_kernel.cu = K,
 * volumeRender.cpp = C).
 *
 * TEST INFRASTRUCTURE ONLY -- see vr_oracle.h.  Never linked into the product.
 *
 * Evaluation rules ("canonical arithmetic"):
 *  - every expression is evaluated with ISO C semantics exactly as written in
 *    the reference source: float/double promotions as the source implies,
 *    left-to-right association, NO fused multiply-add (built with
 *    -ffp-contract=off);
 *  - rsqrtf(x) is taken as 1.0f/sqrtf(x) (both correctly rounded);
 *  - the float overload log(float) is taken as (float)log((double)x);
 *  - texture fetches follow the CUDA texture-fetch rules: point sampling
 *    i = floor(u*N); linear sampling xB = u*N - 0.5, i = floor(xB),
 *    alpha = frac(xB) held in 9-bit fixed point with 8 fractional bits
 *    (rounded to nearest even); clamp addressing (coordinate clamped to
 *    [0,1] first, which gives the same texels as index clamping and a
 *    defined answer for NaN);  1-D/3-D linear blends are
 *    (1-a)*t0 + a*t1, x first, then y, then z.
 */
#include "vr_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* log(2.0) in double, correctly rounded (K:766 `log(2.0)`) */
#define LN2_D 0x1.62e42fefa39efp-1

typedef struct { float x, y, z; } f3;
typedef struct { float x, y, z, w; } f4;

/* transfer function, K:2323-2326 */
static const f4 TF[9] = {
    {0.0f, 0.0f, 0.0f, 0.0f}, {1.0f, 0.0f, 0.0f, 1.0f}, {1.0f, 0.5f, 0.0f, 1.0f},
    {1.0f, 1.0f, 0.0f, 1.0f}, {0.0f, 1.0f, 0.0f, 1.0f}, {0.0f, 1.0f, 1.0f, 1.0f},
    {0.0f, 0.0f, 1.0f, 1.0f}, {1.0f, 0.0f, 1.0f, 1.0f}, {0.0f, 0.0f, 0.0f, 0.0f},
};

static inline float logf_cr(float x) { return (float)log((double)x); }

/* Alternative readings of the arithmetic the reference leaves open, for the
 * parity-margin study only (orc_set_reading, tools/parity_margin.py, DESIGN.md
 * section 3.1); all zero = the canonical reading every test pins:
 *   g_w_trunc    1: texture filter weights truncated to 8 fractional bits
 *                (K:601/619/683) instead of rounded to nearest;
 *   g_rsqrt_ulps rsqrtf of helper_math normalize (K:295) moved this many ulps
 *                from the correctly rounded 1/sqrtf;
 *   g_log_ulps   the per-bin float log of the entropy (K:766) moved this many
 *                ulps from (float)log((double)x). */
static int g_w_trunc = 0, g_rsqrt_ulps = 0, g_log_ulps = 0;

void orc_set_reading(int w_trunc, int rsqrt_ulps, int log_ulps) {
    g_w_trunc = w_trunc;
    g_rsqrt_ulps = rsqrt_ulps;
    g_log_ulps = log_ulps;
}

static inline float ulp_step(float x, int k) {
    for (; k > 0; k--) x = nextafterf(x, INFINITY);
    for (; k < 0; k++) x = nextafterf(x, -INFINITY);
    return x;
}

/* rsqrtf(dot(v, v)) of normalize (K:295) */
static inline float rsqrt_read(float x) {
    const float r = 1.0f / sqrtf(x);
    return g_rsqrt_ulps ? ulp_step(r, g_rsqrt_ulps) : r;
}

/* log(pr) of the entropy's per-bin term (K:766) */
static inline float logf_bin(float x) {
    const float r = logf_cr(x);
    return (g_log_ulps && r != 0.0f) ? ulp_step(r, g_log_ulps) : r;
}

/* 9-bit fixed point weight with 8 fractional bits */
static inline float q8(float a) {
    return (g_w_trunc ? floorf(a * 256.0f) : rintf(a * 256.0f)) * (1.0f / 256.0f);
}

static inline float clamp01(float u) { return fminf(fmaxf(u, 0.0f), 1.0f); }

/* linear-filter texel pair + quantised weight for one axis */
static inline void lin_axis(float u, int n, int *i0, int *i1, float *a) {
    u = clamp01(u);
    float xb = u * (float)n - 0.5f;
    float fl = floorf(xb);
    float fr = xb - fl;
    int i = (int)fl;
    int j = i + 1;
    *a = q8(fr);
    *i0 = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
    *i1 = j < 0 ? 0 : (j > n - 1 ? n - 1 : j);
}

/* point-filter texel, normalised coordinates, clamp (tex, K:62, 2161-2165) */
static inline int point_axis(float u, int n) {
    u = clamp01(u);
    int i = (int)floorf(u * (float)n);
    return i > n - 1 ? n - 1 : i;
}

static inline float lerpq(float a, float b, float t) { return (1.0f - t) * a + t * b; }

void orc_transfer(float x, float out[4]) {
    int i0, i1;
    float a;
    lin_axis(x, 9, &i0, &i1, &a);
    out[0] = lerpq(TF[i0].x, TF[i1].x, a);
    out[1] = lerpq(TF[i0].y, TF[i1].y, a);
    out[2] = lerpq(TF[i0].z, TF[i1].z, a);
    out[3] = lerpq(TF[i0].w, TF[i1].w, a);
}

/* __saturatef: clamp to [0,1], NaN -> 0 */
static inline float sat(float x) {
    if (!(x > 0.0f)) return 0.0f;
    return x > 1.0f ? 1.0f : x;
}

/* rgbaFloatToInt, K:186-193 (truncating float->uint) */
uint32_t orc_pack(const float rgba[4]) {
    float r = sat(rgba[0]), g = sat(rgba[1]), b = sat(rgba[2]), a = sat(rgba[3]);
    return ((uint32_t)(a * 255.0f) << 24) | ((uint32_t)(b * 255.0f) << 16) |
           ((uint32_t)(g * 255.0f) << 8) | (uint32_t)(r * 255.0f);
}

/* K:736-738: float MaxHistogram = 0.0217; binWidth = (Max - Min) / (float)nBins */
static inline float bin_width(int nbins) {
    const float maxh = (float)0.0217;
    const float minh = 0.0f;
    return (maxh - minh) / (float)nbins;
}

/* K:742-747 (also K:359-366): mean += p * (binWidth * i + binWidth / 2.0) */
static inline float raw_mean(const float *p, int nbins) {
    const float bw = bin_width(nbins);
    float mean = 0.0f;
    for (int i = 0; i < nbins; i++) {
        double c = (double)(bw * (float)i) + (double)bw / 2.0;
        mean = (float)((double)mean + (double)p[i] * c);
    }
    return mean;
}

float orc_corner_mean(const float *rec, int nbins) { return raw_mean(rec, nbins); }

static inline float entropy_norm(int nbins) {
    /* K:769: log((float)nBins) / log(2.0f), both float overloads */
    return logf_cr((float)nbins) / logf_cr(2.0f);
}

/* d_basicDataProcessing statistics, K:742-773 */
static void stats3(const float *p, int nbins, float enorm, int want, float out[3]) {
    const float maxh = (float)0.0217;
    float mean = raw_mean(p, nbins);
    float var = 0.0f;
    if (want & 2) {
        for (int i = 0; i < nbins; i++) { /* K:750-755 */
            float d = ((float)i / (float)nbins) * maxh - mean;
            var = var + p[i] * d * d;
        }
    }
    out[0] = (float)((double)mean / 0.0217);   /* K:758 */
    out[1] = (float)((double)var / 0.000021);  /* K:759 */
    float ent = 0.0f;
    if (want & 4) {
        for (int i = 0; i < nbins; i++) { /* K:762-767 */
            float pr = p[i];
            double t = pr <= 0 ? 0.0 : ((double)logf_bin(pr) / LN2_D);
            ent = (float)((double)ent + (double)pr * t);
        }
        ent = -ent;          /* K:768 */
        ent = ent / enorm;   /* K:769 */
    }
    out[2] = ent;
}

void orc_record_stats(const float *rec, int nbins, float out[3]) {
    stats3(rec, nbins, entropy_norm(nbins), 7, out);
}

/* ------------------------------------------------------------------------ */
/* per-ray march, K:272-717                                                  */
/* ------------------------------------------------------------------------ */

typedef struct {
    const float *vol;
    int nx, ny, nz, nb;
    float enorm;
    uint64_t *mark; /* optional footprint bitset */
    const orc_codec *codec; /* methods 4/5/6 */
    const float *flex;      /* methods 8/9/0: block statistics, nflex^3 float4 */
    int nflex;
} vol_t;

static inline const float *rec_at(const vol_t *v, int x, int y, int z) {
    size_t idx = ((size_t)z * (size_t)v->ny + (size_t)y) * (size_t)v->nx + (size_t)x;
    return v->vol + idx * (size_t)v->nb;
}

static inline void mark_voxel(const vol_t *v, int x, int y, int z) {
    size_t idx = ((size_t)z * (size_t)v->ny + (size_t)y) * (size_t)v->nx + (size_t)x;
    __atomic_fetch_or(&v->mark[idx >> 6], (uint64_t)1 << (idx & 63), __ATOMIC_RELAXED);
}

/* Fractal/template codec record (d_basicDataProcessing K:775-871 with
 * fractalDecoding K:195-222), restated with these choices for the reference's
 * undefined behaviour: fractalDecoding's result is the decoded array (K:221
 * returns a pointer to a local), error entries whose bin id is outside
 * [0, nbins) are skipped (K:810 admits == nbins, an out-of-bounds write), and
 * the inputs are validated (template id, 0 <= shift < nbins, NE <= slots), so
 * the wrap `m - nBins` of K:204-206 is exact. */
void orc_codec_decode(const orc_codec *c, int nbins, size_t vidx, float *dec) {
    const int32_t *cb = c->codebook + 4 * vidx;
    const int tid = cb[0], shift = cb[1], flip = cb[2] != 0, ne = cb[3];
    const float *orig = c->templates + (size_t)tid * (size_t)nbins;
    for (int i = 0; i < nbins; i++) { /* K:199-219 */
        int m = i + shift;
        if (m >= nbins) m = m - nbins;
        dec[m] = flip ? orig[nbins - 1 - i] : orig[i];
    }
    const float *err = c->errors + 2 * vidx * (size_t)c->err_slots;
    for (int j = 0; j < ne; j++) { /* K:805-823 */
        int idx = (int)err[2 * j];
        if (idx < 0 || idx >= nbins) continue;
        dec[idx] = dec[idx] + err[2 * j + 1];
        if (dec[idx] < 0) dec[idx] = 0;
    }
    float total = 0.0f; /* K:826-835 */
    for (int i = 0; i < nbins; i++) total = total + dec[i];
    for (int i = 0; i < nbins; i++)
        if (total > 0) dec[i] = dec[i] / total;
}

/* statistics of a decoded codec record, K:837-868: the bin centre is used in
 * both mean and variance (unlike K:750-755) */
static void codec_stats3(const orc_codec *c, int nbins, float enorm, size_t vidx, float out[3]) {
    float dec[256];
    orc_codec_decode(c, nbins, vidx, dec);
    const float bw = bin_width(nbins);
    float mean = raw_mean(dec, nbins);
    float var = 0.0f;
    for (int i = 0; i < nbins; i++) {
        double d = ((double)(bw * (float)i) + (double)bw / 2.0) - (double)mean;
        var = (float)((double)var + (double)dec[i] * d * d);
    }
    out[0] = (float)((double)mean / 0.0217);
    out[1] = (float)((double)var / 0.000021);
    float ent = 0.0f;
    for (int i = 0; i < nbins; i++) {
        float pr = dec[i];
        double t = pr <= 0 ? 0.0 : ((double)logf_bin(pr) / LN2_D);
        ent = (float)((double)ent + (double)pr * t);
    }
    ent = -ent;
    out[2] = ent / enorm;
}

void orc_codec_stats(const orc_codec *c, int nbins, size_t vidx, float out[3]) {
    codec_stats3(c, nbins, entropy_norm(nbins), vidx, out);
}

/* methods 1/2/3: tex3D(originalQueryTex, p) with hardware trilinear (K:601, 619,
 * 635; texture set up K:1864-1869), the statistic decoded from the 8 corner
 * records instead of a pre-baked float4 volume (algebraically identical). */
static float sample_stat(const vol_t *v, f3 pos, int comp) {
    float px = pos.x * 0.5f + 0.5f;
    float py = pos.y * 0.5f + 0.5f;
    float pz = pos.z * 0.5f + 0.5f;
    int x0, x1, y0, y1, z0, z1;
    float ax, ay, az;
    lin_axis(px, v->nx, &x0, &x1, &ax);
    lin_axis(py, v->ny, &y0, &y1, &ay);
    lin_axis(pz, v->nz, &z0, &z1, &az);
    if (v->mark) {
        mark_voxel(v, x0, y0, z0); mark_voxel(v, x1, y0, z0);
        mark_voxel(v, x0, y1, z0); mark_voxel(v, x1, y1, z0);
        mark_voxel(v, x0, y0, z1); mark_voxel(v, x1, y0, z1);
        mark_voxel(v, x0, y1, z1); mark_voxel(v, x1, y1, z1);
    }
    float s[8][3];
    if (comp >= 3) { /* methods 4/5/6: fractalQueryTex, K:639-652 */
        const int xs[2] = {x0, x1}, ys[2] = {y0, y1}, zs[2] = {z0, z1};
        for (int j = 0; j < 8; j++) {
            size_t idx = ((size_t)zs[j >> 2] * (size_t)v->ny + (size_t)ys[(j >> 1) & 1]) *
                             (size_t)v->nx + (size_t)xs[j & 1];
            codec_stats3(v->codec, v->nb, v->enorm, idx, s[j]);
        }
        comp -= 3;
        float c00 = lerpq(s[0][comp], s[1][comp], ax);
        float c10 = lerpq(s[2][comp], s[3][comp], ax);
        float c01 = lerpq(s[4][comp], s[5][comp], ax);
        float c11 = lerpq(s[6][comp], s[7][comp], ax);
        float c0 = lerpq(c00, c10, ay);
        float c1 = lerpq(c01, c11, ay);
        return lerpq(c0, c1, az);
    }
    const int want = comp == 0 ? 1 : (comp == 1 ? 3 : 4);
    stats3(rec_at(v, x0, y0, z0), v->nb, v->enorm, want, s[0]);
    stats3(rec_at(v, x1, y0, z0), v->nb, v->enorm, want, s[1]);
    stats3(rec_at(v, x0, y1, z0), v->nb, v->enorm, want, s[2]);
    stats3(rec_at(v, x1, y1, z0), v->nb, v->enorm, want, s[3]);
    stats3(rec_at(v, x0, y0, z1), v->nb, v->enorm, want, s[4]);
    stats3(rec_at(v, x1, y0, z1), v->nb, v->enorm, want, s[5]);
    stats3(rec_at(v, x0, y1, z1), v->nb, v->enorm, want, s[6]);
    stats3(rec_at(v, x1, y1, z1), v->nb, v->enorm, want, s[7]);
    float c00 = lerpq(s[0][comp], s[1][comp], ax);
    float c10 = lerpq(s[2][comp], s[3][comp], ax);
    float c01 = lerpq(s[4][comp], s[5][comp], ax);
    float c11 = lerpq(s[6][comp], s[7][comp], ax);
    float c0 = lerpq(c00, c10, ay);
    float c1 = lerpq(c01, c11, ay);
    return lerpq(c0, c1, az);
}

/* Flexible-block sample, K:654-680: tex3D(flexBlockTex, (p*0.5+0.5)*nFlexBlock*)
 * with an unnormalised coordinate, linear filter and clamp addressing on the
 * 500^3 float4 array of bindToTex (K:1691-1714), which holds the block
 * statistics at [0, nblk) per axis and zeros elsewhere. */
#define FLEX_TEX 500 /* nMaxBlockDim, K:93 */
static inline void lin_axis_unnorm(float u, int *i0, int *i1, float *a) {
    float xb = u - 0.5f;
    float fl = floorf(xb);
    float fr = xb - fl;
    int i = (int)fl;
    *a = q8(fr);
    *i0 = i < 0 ? 0 : (i > FLEX_TEX - 1 ? FLEX_TEX - 1 : i);
    *i1 = i + 1 < 0 ? 0 : (i + 1 > FLEX_TEX - 1 ? FLEX_TEX - 1 : i + 1);
}

static inline float flex_texel(const vol_t *v, int x, int y, int z, int comp) {
    const int n = v->nflex;
    if (x >= n || y >= n || z >= n) return 0.0f;
    return v->flex[(((size_t)z * n + y) * n + x) * 4 + comp];
}

static float sample_flex(const vol_t *v, f3 pos, int comp) {
    const float nf = (float)v->nflex;
    int x0, x1, y0, y1, z0, z1;
    float ax, ay, az;
    lin_axis_unnorm((pos.x * 0.5f + 0.5f) * nf, &x0, &x1, &ax);
    lin_axis_unnorm((pos.y * 0.5f + 0.5f) * nf, &y0, &y1, &ay);
    lin_axis_unnorm((pos.z * 0.5f + 0.5f) * nf, &z0, &z1, &az);
    float c00 = lerpq(flex_texel(v, x0, y0, z0, comp), flex_texel(v, x1, y0, z0, comp), ax);
    float c10 = lerpq(flex_texel(v, x0, y1, z0, comp), flex_texel(v, x1, y1, z0, comp), ax);
    float c01 = lerpq(flex_texel(v, x0, y0, z1, comp), flex_texel(v, x1, y0, z1, comp), ax);
    float c11 = lerpq(flex_texel(v, x0, y1, z1, comp), flex_texel(v, x1, y1, z1, comp), ax);
    float c0 = lerpq(c00, c10, ay);
    float c1 = lerpq(c01, c11, ay);
    return lerpq(c0, c1, az);
}

/* method 7 corner state, K:320-367 / K:398-463 */
typedef struct {
    f3 ip[8];
    float mean[8];
} m7_t;

static void m7_refresh(const vol_t *v, const int N[3], f3 pos, m7_t *m) {
    float qx = pos.x * 0.5f + 0.5f, qy = pos.y * 0.5f + 0.5f, qz = pos.z * 0.5f + 0.5f;
    float fx = floorf(qx * (float)N[0]) / (float)N[0];
    float cx = ceilf(qx * (float)N[0]) / (float)N[0];
    float fy = floorf(qy * (float)N[1]) / (float)N[1];
    float cy = ceilf(qy * (float)N[1]) / (float)N[1];
    float fz = floorf(qz * (float)N[2]) / (float)N[2];
    float cz = ceilf(qz * (float)N[2]) / (float)N[2];
    for (int j = 0; j < 8; j++) {
        m->ip[j].x = (j & 1) ? cx : fx;
        m->ip[j].y = (j & 2) ? cy : fy;
        m->ip[j].z = (j & 4) ? cz : fz;
        int ix = point_axis(m->ip[j].x, v->nx);
        int iy = point_axis(m->ip[j].y, v->ny);
        int iz = point_axis(m->ip[j].z, v->nz);
        m->mean[j] = raw_mean(rec_at(v, ix, iy, iz), v->nb);
    }
}

/* inInterpolation, K:253-270 */
static inline int m7_inside(f3 pos, const m7_t *m) {
    float qx = pos.x * 0.5f + 0.5f, qy = pos.y * 0.5f + 0.5f, qz = pos.z * 0.5f + 0.5f;
    if (qx < m->ip[0].x || qy < m->ip[0].y || qz < m->ip[0].z || qx > m->ip[7].x ||
        qy > m->ip[7].y || qz > m->ip[7].z)
        return 0;
    return 1;
}

/* K:466-479 */
static float m7_sample(f3 pos, const m7_t *m) {
    float xd = (pos.x * 0.5f + 0.5f - m->ip[0].x) / (m->ip[1].x - m->ip[0].x);
    float yd = (pos.y * 0.5f + 0.5f - m->ip[0].y) / (m->ip[2].y - m->ip[0].y);
    float zd = (pos.z * 0.5f + 0.5f - m->ip[0].z) / (m->ip[4].z - m->ip[0].z);
    const float *mn = m->mean;
    float m00 = (float)((double)mn[0] * (1.0 - (double)xd) + (double)(mn[1] * xd));
    float m10 = (float)((double)mn[2] * (1.0 - (double)xd) + (double)(mn[3] * xd));
    float m01 = (float)((double)mn[4] * (1.0 - (double)xd) + (double)(mn[5] * xd));
    float m11 = (float)((double)mn[6] * (1.0 - (double)xd) + (double)(mn[7] * xd));
    float m0 = (float)((double)m00 * (1.0 - (double)yd) + (double)(m10 * yd));
    float m1 = (float)((double)m01 * (1.0 - (double)yd) + (double)(m11 * yd));
    float im = (float)((double)m0 * (1.0 - (double)zd) + (double)(m1 * zd));
    return im * 50.0f; /* K:479 */
}

static inline float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

/* one pixel; returns samples taken, -1 on a miss */
static int render_pixel(const vol_t *v, const orc_render_params *p, int x, int y,
                        float rgba[4]) {
    const int maxSteps = 500;          /* K:276 */
    const float tstep = 0.01f;         /* K:277 */
    const float opacityThreshold = 0.95f;
    const float *M = p->inv_view;

    float u = ((float)x / (float)p->width) * 2.0f - 1.0f;  /* K:288 */
    float vv = ((float)y / (float)p->height) * 2.0f - 1.0f; /* K:289 */

    /* K:293-296 */
    f3 o;
    o.x = 0.0f * M[0] + 0.0f * M[1] + 0.0f * M[2] + 1.0f * M[3];
    o.y = 0.0f * M[4] + 0.0f * M[5] + 0.0f * M[6] + 1.0f * M[7];
    o.z = 0.0f * M[8] + 0.0f * M[9] + 0.0f * M[10] + 1.0f * M[11];
    f3 d0 = {u, vv, -2.0f};
    float inv = rsqrt_read(dot3(d0, d0));
    d0.x = d0.x * inv; d0.y = d0.y * inv; d0.z = d0.z * inv;
    f3 d;
    d.x = d0.x * M[0] + d0.y * M[1] + d0.z * M[2];
    d.y = d0.x * M[4] + d0.y * M[5] + d0.z * M[6];
    d.z = d0.x * M[8] + d0.y * M[9] + d0.z * M[10];

    /* intersectBox, K:136-156 */
    f3 invR = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    f3 tbot = {invR.x * (-1.0f - o.x), invR.y * (-1.0f - o.y), invR.z * (-1.0f - o.z)};
    f3 ttop = {invR.x * (1.0f - o.x), invR.y * (1.0f - o.y), invR.z * (1.0f - o.z)};
    f3 tmin = {fminf(ttop.x, tbot.x), fminf(ttop.y, tbot.y), fminf(ttop.z, tbot.z)};
    f3 tmax = {fmaxf(ttop.x, tbot.x), fmaxf(ttop.y, tbot.y), fmaxf(ttop.z, tbot.z)};
    float tnear = fmaxf(fmaxf(tmin.x, tmin.y), fmaxf(tmin.x, tmin.z));
    float tfar = fminf(fminf(tmax.x, tmax.y), fminf(tmax.x, tmax.z));
    if (!(tfar > tnear)) return -1; /* K:302-303: no write */
    if (tnear < 0.0f) tnear = 0.0f;

    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = tnear;
    f3 pos = {o.x + d.x * tnear, o.y + d.y * tnear, o.z + d.z * tnear};
    f3 step = {d.x * tstep, d.y * tstep, d.z * tstep};

    m7_t m7;
    const int method = p->query_method;
    if (method == 7) m7_refresh(v, p->m7_dims, pos, &m7); /* K:320-367 */

    int n = 0;
    for (int i = 0; i < maxSteps; i++) {
        float sample = 0.5f; /* K:383 */
        if (method == 7) {
            if (!m7_inside(pos, &m7)) m7_refresh(v, p->m7_dims, pos, &m7);
            sample = m7_sample(pos, &m7);
        } else if (method == 1) {
            sample = sample_stat(v, pos, 0);
        } else if (method == 2) {
            sample = sample_stat(v, pos, 1);
        } else if (method == 3) {
            sample = sample_stat(v, pos, 2);
        } else if (method >= 4 && method <= 6 && v->codec) {
            sample = sample_stat(v, pos, method - 1);
        } else if (v->flex && (method == 8 || method == 9 || method == 0)) {
            /* K:654-680: .z entropy (8), .x mean (9), .y variance (0) */
            sample = sample_flex(v, pos, method == 8 ? 2 : (method == 9 ? 0 : 1));
        }
        n = i + 1;
        float col[4];
        orc_transfer((sample - p->transfer_offset) * p->transfer_scale, col); /* K:683 */
        col[3] = col[3] * p->density;   /* K:685 */
        col[0] = col[0] * col[3];       /* K:691-693 */
        col[1] = col[1] * col[3];
        col[2] = col[2] * col[3];
        float om = 1.0f - sw;           /* K:695 */
        sx = sx + col[0] * om;
        sy = sy + col[1] * om;
        sz = sz + col[2] * om;
        sw = sw + col[3] * om;
        if (sw > opacityThreshold) break; /* K:698 */
        t = t + tstep;                    /* K:701 */
        if (t > tfar) break;              /* K:703 */
        pos.x = pos.x + step.x;           /* K:706 */
        pos.y = pos.y + step.y;
        pos.z = pos.z + step.z;
    }
    rgba[0] = sx * p->brightness; /* K:713 */
    rgba[1] = sy * p->brightness;
    rgba[2] = sz * p->brightness;
    rgba[3] = sw * p->brightness;
    return n;
}

static void run_rows(const vol_t *v, const orc_render_params *p, uint32_t *out,
                     float *out_f, int32_t *out_n, int row_start, int row_stride,
                     int nthreads, int64_t *total) {
    if (row_stride < 1) row_stride = 1;
    int nrows = row_start < p->height ? (p->height - 1 - row_start) / row_stride + 1 : 0;
    int64_t acc = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(+ : acc)
#endif
    for (int r = 0; r < nrows; r++) {
        int y = row_start + r * row_stride;
        for (int x = 0; x < p->width; x++) {
            float rgba[4];
            int n = render_pixel(v, p, x, y, rgba);
            size_t pix = (size_t)y * (size_t)p->width + (size_t)x;
            if (out_n) out_n[pix] = n;
            if (n < 0) continue;
            acc += n;
            if (out) out[pix] = orc_pack(rgba);
            if (out_f) {
                out_f[pix * 4 + 0] = sat(rgba[0]);
                out_f[pix * 4 + 1] = sat(rgba[1]);
                out_f[pix * 4 + 2] = sat(rgba[2]);
                out_f[pix * 4 + 3] = sat(rgba[3]);
            }
        }
    }
    (void)nthreads;
    *total = acc;
}

int64_t orc_render(const float *vol, int nx, int ny, int nz, int nbins,
                   const orc_render_params *p, uint32_t *out, float *out_f,
                   int32_t *out_n, int row_start, int row_stride, int nthreads) {
    vol_t v = {vol, nx, ny, nz, nbins, entropy_norm(nbins), NULL, NULL, NULL, 0};
    int64_t total = 0;
    run_rows(&v, p, out, out_f, out_n, row_start, row_stride, nthreads, &total);
    return total;
}

int64_t orc_render_codec(const orc_codec *codec, int nx, int ny, int nz, int nbins,
                         const orc_render_params *p, uint32_t *out, float *out_f,
                         int32_t *out_n, int row_start, int row_stride, int nthreads) {
    vol_t v = {NULL, nx, ny, nz, nbins, entropy_norm(nbins), NULL, codec, NULL, 0};
    int64_t total = 0;
    run_rows(&v, p, out, out_f, out_n, row_start, row_stride, nthreads, &total);
    return total;
}

int64_t orc_count_footprint(const float *vol, int nx, int ny, int nz, int nbins,
                            const orc_render_params *p, int nthreads) {
    size_t nvox = (size_t)nx * (size_t)ny * (size_t)nz;
    size_t nwords = (nvox + 63) / 64;
    uint64_t *mark = (uint64_t *)calloc(nwords, sizeof(uint64_t));
    if (!mark) return -1;
    vol_t v = {vol, nx, ny, nz, nbins, entropy_norm(nbins), mark, NULL, NULL, 0};
    int64_t total = 0;
    run_rows(&v, p, NULL, NULL, NULL, 0, 1, nthreads, &total);
    int64_t u = 0;
    for (size_t i = 0; i < nwords; i++) u += __builtin_popcountll(mark[i]);
    free(mark);
    return u;
}

/* ------------------------------------------------------------------------ */
/* synthetic distribution volume                       */
/* ------------------------------------------------------------------------ */

/* omp_get_max_threads() of this process (bench.py reports it beside the
 * threads the CPU baseline uses) */
int orc_max_threads(void) { return omp_get_max_threads(); }

uint64_t orc_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline double u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }

#define SYN_K 8
#define SYN_G 16
#define SYN_Q 4096

static void axis_table(int n, double c, double s, float *out) {
    for (int i = 0; i < n; i++) {
        double q = ((double)i + 0.5) / (double)n;
        out[i] = (float)exp(-(q - c) * (q - c) / (2.0 * s * s));
    }
}

void orc_synth_fill(int nx, int ny, int nz, int nbins, uint64_t seed, float *vol,
                    int nthreads) {
    float amp[SYN_K];
    float *gx = (float *)malloc(sizeof(float) * SYN_K * (size_t)nx);
    float *gy = (float *)malloc(sizeof(float) * SYN_K * (size_t)ny);
    float *gz = (float *)malloc(sizeof(float) * SYN_K * (size_t)nz);
    for (int k = 0; k < SYN_K; k++) {
        double r[5];
        for (int j = 0; j < 5; j++) r[j] = u01(orc_splitmix64(seed + 0x100u + 8u * (uint64_t)k + (uint64_t)j));
        amp[k] = (float)(0.3 + 0.7 * r[0]);
        double s = 0.05 + 0.15 * r[4];
        axis_table(nx, 0.2 + 0.6 * r[1], s, gx + (size_t)k * nx);
        axis_table(ny, 0.2 + 0.6 * r[2], s, gy + (size_t)k * ny);
        axis_table(nz, 0.2 + 0.6 * r[3], s, gz + (size_t)k * nz);
    }
    float *tab = NULL;
    if (nbins > 1) {
        tab = (float *)malloc(sizeof(float) * SYN_G * SYN_Q * (size_t)nbins);
        double *e = (double *)malloc(sizeof(double) * (size_t)nbins);
        for (int g = 0; g < SYN_G; g++) {
            double sig = 0.02 + 0.1 * (double)g / 15.0;
            for (int q = 0; q < SYN_Q; q++) {
                double mu = ((double)q + 0.5) / (double)SYN_Q;
                double sum = 0.0;
                for (int b = 0; b < nbins; b++) {
                    double dd = ((double)b + 0.5) / (double)nbins - mu;
                    e[b] = exp(-dd * dd / (2.0 * sig * sig));
                    sum += e[b];
                }
                float *row = tab + ((size_t)g * SYN_Q + (size_t)q) * (size_t)nbins;
                for (int b = 0; b < nbins; b++) row[b] = (float)(e[b] / sum);
            }
        }
        free(e);
    }
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
    for (int z = 0; z < nz; z++) {
        for (int y = 0; y < ny; y++) {
            for (int x = 0; x < nx; x++) {
                float f = 0.0f;
                for (int k = 0; k < SYN_K; k++)
                    f = f + ((amp[k] * gx[(size_t)k * nx + x]) * gy[(size_t)k * ny + y]) *
                                gz[(size_t)k * nz + z];
                if (f > 1.0f) f = 1.0f;
                uint64_t vidx = ((uint64_t)z * (uint64_t)ny + (uint64_t)y) * (uint64_t)nx + (uint64_t)x;
                float *rec = vol + vidx * (uint64_t)nbins;
                if (nbins == 1) {
                    rec[0] = f;
                } else {
                    int q = (int)(f * 4096.0f);
                    if (q > SYN_Q - 1) q = SYN_Q - 1;
                    int g = (int)(orc_splitmix64(seed ^ vidx) & (SYN_G - 1));
                    memcpy(rec, tab + ((size_t)g * SYN_Q + (size_t)q) * (size_t)nbins,
                           sizeof(float) * (size_t)nbins);
                }
            }
        }
    }
    (void)nthreads;
    free(tab);
    free(gx);
    free(gy);
    free(gz);
}

/* Synthetic codec volume: the section-5 field encoded
 * against ntpl templates; mirrors k_synth_codec bit for bit. */
void orc_synth_codec(int nx, int ny, int nz, int nbins, int ntpl, int slots, uint64_t seed,
                     int32_t *cb, float *tpl, float *err) {
    float amp[SYN_K];
    float *gx = (float *)malloc(sizeof(float) * SYN_K * (size_t)nx);
    float *gy = (float *)malloc(sizeof(float) * SYN_K * (size_t)ny);
    float *gz = (float *)malloc(sizeof(float) * SYN_K * (size_t)nz);
    for (int k = 0; k < SYN_K; k++) {
        double r[5];
        for (int j = 0; j < 5; j++) r[j] = u01(orc_splitmix64(seed + 0x100u + 8u * (uint64_t)k + (uint64_t)j));
        amp[k] = (float)(0.3 + 0.7 * r[0]);
        double s = 0.05 + 0.15 * r[4];
        axis_table(nx, 0.2 + 0.6 * r[1], s, gx + (size_t)k * nx);
        axis_table(ny, 0.2 + 0.6 * r[2], s, gy + (size_t)k * ny);
        axis_table(nz, 0.2 + 0.6 * r[3], s, gz + (size_t)k * nz);
    }
    double *e = (double *)malloc(sizeof(double) * (size_t)nbins);
    for (int t = 0; t < ntpl; t++) {
        double mu = ((double)t + 0.5) / (double)ntpl, sum = 0.0;
        for (int b = 0; b < nbins; b++) {
            double dd = ((double)b + 0.5) / (double)nbins - mu;
            e[b] = exp(-dd * dd / (2.0 * 0.06 * 0.06));
            sum += e[b];
        }
        for (int b = 0; b < nbins; b++) tpl[(size_t)t * nbins + b] = (float)(e[b] / sum);
    }
    free(e);
    const int nemax = (slots < 3 ? slots : 3) + 1;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int z = 0; z < nz; z++)
        for (int y = 0; y < ny; y++)
            for (int x = 0; x < nx; x++) {
                float f = 0.0f;
                for (int k = 0; k < SYN_K; k++)
                    f = f + ((amp[k] * gx[(size_t)k * nx + x]) * gy[(size_t)k * ny + y]) *
                                gz[(size_t)k * nz + z];
                if (f > 1.0f) f = 1.0f;
                int t = (int)(f * (float)ntpl);
                if (t > ntpl - 1) t = ntpl - 1;
                uint64_t v = ((uint64_t)z * (uint64_t)ny + (uint64_t)y) * (uint64_t)nx + (uint64_t)x;
                uint64_t h = orc_splitmix64(seed ^ v);
                int32_t *c = cb + 4 * v;
                c[0] = t;
                c[1] = (int)((h >> 8) & 1) % nbins;
                c[2] = ((h >> 16) & 7) == 0 ? 1 : 0;
                c[3] = (int)((h >> 24) % (uint64_t)nemax);
                for (int j = 0; j < slots; j++) {
                    uint64_t h2 = orc_splitmix64(seed + 0x5bd1e995ull + v * (uint64_t)slots + (uint64_t)j);
                    err[2 * (v * (uint64_t)slots + (uint64_t)j)] = (float)(h2 % (uint64_t)nbins);
                    err[2 * (v * (uint64_t)slots + (uint64_t)j) + 1] =
                        (float)(((double)(h2 >> 11) * 0x1.0p-53 - 0.5) / 10.0);
                }
            }
    free(gx);
    free(gy);
    free(gz);
}

/* ------------------------------------------------------------------------ */
/* flexible blocks: the dataProcessing pre-pass, K:892-1126, 1142-1544       */
/* ------------------------------------------------------------------------ */
/*
 * Choices for the reference's undefined / unordered behaviour:
 *  - the per-corner sum runs over the sub-spans in their index order
 *    i*ny*nz + j*nz + k (the reference adds them with shared-memory float
 *    atomics in whatever order the threads arrive, K:1402, 1520);
 *  - a sub-span is looked up as the linear scan of K:1352-1372 finds it: the
 *    scan's `break` leaves only the x loop, so among equal spans the LAST
 *    64-entry row holding one wins, and the first entry of that row; a span with
 *    no entry is an error (the reference reads an uninitialised codebook entry);
 *  - flexibleFractalDecoding's result is the decoded array (K:249 returns a
 *    pointer to a local); templates come from layer 0 (K:1389 reads layer 1 of
 *    a one-layer array); error and simple-histogram bin ids outside [0, nbins)
 *    are skipped (K:1407 admits == flexNBin, an out-of-bounds write);
 *  - only cubic volumes (d_divideBlock loops x over nz and z over nx, K:1013-1015,
 *    and fills the span arrays of all three axes in each pass, K:935-1011).
 */
static int flex_find(const int32_t *low, const int32_t *high, int n, const int l[3],
                     const int h[3]) {
    int best = -1, best_row = -1;
    for (int i = 0; i < n; i++) {
        const int32_t *a = low + 4 * (size_t)i, *b = high + 4 * (size_t)i;
        if (a[0] == l[0] && a[1] == l[1] && a[2] == l[2] && b[0] == h[0] && b[1] == h[1] &&
            b[2] == h[2]) {
            if (i / 64 != best_row) {
                best = i;
                best_row = i / 64;
            }
        }
    }
    return best;
}

/* K:1248-1282: [1, x] as dyadic spans, lowest set bit first */
static int flex_split(int x, int lo[8], int hi[8]) {
    int n = 0;
    for (int i = 0; i <= 6; i++) {
        if ((x & ~(1 << i)) != x) {
            hi[n] = x;
            x &= ~(1 << i);
            lo[n] = x + 1;
            n++;
        }
        if (x == 0) break;
    }
    return n;
}

/* histogram of one span (K:1349-1437 fractal, K:1438-1531 simple), unweighted */
static int flex_span_hist_uncached(const orc_flex *f, const int l[3], const int h[3], float *out);

/* memo of span histograms per (low, high): block corners share most sub-spans,
 * so each distinct span is looked up (linear scan) and decoded once */
typedef struct {
    int key[6];
    int w;      /* weight, or -1 for a missing span; 0 = empty slot */
    float *hist;
} flex_memo_slot;
static flex_memo_slot *g_memo = NULL;
static size_t g_memo_cap = 0;
static const orc_flex *g_memo_f = NULL;

static void flex_memo_reset(const orc_flex *f) {
    for (size_t i = 0; i < g_memo_cap; i++) free(g_memo[i].hist);
    free(g_memo);
    g_memo_cap = 1u << 18;
    g_memo = calloc(g_memo_cap, sizeof(flex_memo_slot));
    g_memo_f = f;
}

static int flex_span_hist(const orc_flex *f, const int l[3], const int h[3], float *out) {
    if (g_memo_f != f) return flex_span_hist_uncached(f, l, h, out);
    uint64_t k = 1469598103934665603ull;
    const int key[6] = {l[0], l[1], l[2], h[0], h[1], h[2]};
    for (int q = 0; q < 6; q++) k = (k ^ (uint64_t)(uint32_t)key[q]) * 1099511628211ull;
    size_t i = (size_t)(k & (g_memo_cap - 1));
    for (;; i = (i + 1) & (g_memo_cap - 1)) {
        flex_memo_slot *s = &g_memo[i];
        if (s->w == 0) {
            memcpy(s->key, key, sizeof key);
            s->hist = malloc(sizeof(float) * (size_t)f->nbins);
            s->w = flex_span_hist_uncached(f, l, h, s->hist);
            if (s->w == 0) s->w = -2; /* cannot happen: spans hold >= 1 voxel */
            break;
        }
        if (memcmp(s->key, key, sizeof key) == 0) break;
    }
    if (g_memo[i].w < 0) return -1;
    memcpy(out, g_memo[i].hist, sizeof(float) * (size_t)f->nbins);
    return g_memo[i].w;
}

static int flex_span_hist_uncached(const orc_flex *f, const int l[3], const int h[3], float *out) {
    const int nb = f->nbins;
    const int size = (h[0] - l[0] + 1) * (h[1] - l[1] + 1) * (h[2] - l[2] + 1);
    if (size >= 8) { /* K:1349 */
        const int e = flex_find(f->fractal_low, f->fractal_high, f->n_fractal, l, h);
        if (e < 0) return -1;
        const int32_t *cb = f->fractal_code + 4 * (size_t)e;
        const int tid = cb[0], shift = cb[1], flip = cb[2] != 0, ne = cb[3];
        const float *orig = f->templates + (size_t)tid * (size_t)nb;
        for (int i = 0; i < nb; i++) { /* flexibleFractalDecoding, K:225-250 */
            int m = i + shift;
            if (m >= nb) m = m - nb;
            out[m] = flip ? orig[nb - 1 - i] : orig[i];
        }
        const float *err = f->fractal_err + 2 * (size_t)e * (size_t)nb;
        for (int j = 0; j < ne; j++) { /* K:1400-1418 */
            int idx = (int)err[2 * j];
            if (idx < 0 || idx >= nb) continue;
            out[idx] = out[idx] + err[2 * j + 1];
            if (out[idx] < 0) out[idx] = 0;
        }
        float total = 0.0f; /* K:1420-1431 */
        for (int i = 0; i < nb; i++) total = total + out[i];
        for (int i = 0; i < nb; i++) out[i] = out[i] / total;
    } else {
        const int l0[3] = {l[0] - 1, l[1] - 1, l[2] - 1}; /* K:1444-1449 */
        const int h0[3] = {h[0] - 1, h[1] - 1, h[2] - 1};
        const int e = flex_find(f->simple_low, f->simple_high, f->n_simple, l0, h0);
        if (e < 0) return -1;
        for (int i = 0; i < nb; i++) out[i] = 0.0f;
        const float *pr = f->simple_hist + 2 * (size_t)e * (size_t)nb;
        for (int j = 0; j < f->simple_count[e]; j++) { /* K:1510-1514 */
            int idx = (int)pr[2 * j];
            if (idx < 0 || idx >= nb) continue;
            out[idx] = pr[2 * j + 1];
        }
    }
    return size;
}

int orc_flex_corner(const orc_flex *f, int x, int y, int z, float *hist) {
    int xl[8], xh[8], yl[8], yh[8], zl[8], zh[8];
    const int nx = flex_split(x, xl, xh), ny = flex_split(y, yl, yh), nz = flex_split(z, zl, zh);
    float sp[256];
    for (int b = 0; b < f->nbins; b++) hist[b] = 0.0f;
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < ny; j++)
            for (int k = 0; k < nz; k++) {
                const int l[3] = {xl[i], yl[j], zl[k]}, h[3] = {xh[i], yh[j], zh[k]};
                const int w = flex_span_hist(f, l, h, sp);
                if (w < 0) return -1 - (i * ny * nz + j * nz + k);
                for (int b = 0; b < f->nbins; b++) hist[b] = hist[b] + sp[b] * (float)w;
            }
    return nx * ny * nz;
}

int orc_flex_process(const orc_flex *f, float *blocks) {
    const int D = f->dim, bs = f->block, nb = f->nbins;
    if (D < 1 || D > 126 || bs < 1 || bs > D || nb < 1 || nb > 256) return -1000000;
    const int nblk = (D + bs - 1) / bs; /* K:906-931 */
    flex_memo_reset(f);
    const float bw = (255.0f - 0.0f) / (float)nb; /* K:1084-1087 */
    const float enorm = entropy_norm(nb);
    int rc = nblk;
    for (int n = 0; n < nblk * nblk * nblk; n++) {
        const int bx = n % nblk, by = (n / nblk) % nblk, bz = n / (nblk * nblk);
        /* span of block n, K:935-1024: [1 + i*bs, (i+1)*bs], the last cut at D */
        const int lo[3] = {1 + bx * bs, 1 + by * bs, 1 + bz * bs};
        const int hi[3] = {bx == nblk - 1 ? D : (bx + 1) * bs, by == nblk - 1 ? D : (by + 1) * bs,
                           bz == nblk - 1 ? D : (bz + 1) * bs};
        float c[8][256];
        for (int k = 0; k < 8; k++) { /* corners, K:1151-1228 */
            const int x = (k & 1) ? hi[0] : lo[0], y = (k & 2) ? hi[1] : lo[1],
                      z = (k & 4) ? hi[2] : lo[2];
            if (orc_flex_corner(f, x, y, z, c[k]) < 0) rc = -1 - n;
        }
        float h[256], total = 0.0f;
        for (int s = 0; s < nb; s++) { /* K:1041-1051 */
            h[s] = c[0][s] + c[3][s] + c[4][s] + c[7][s] - c[1][s] - c[2][s] - c[5][s] - c[6][s];
            if (h[s] < 0) h[s] = 0;
        }
        for (int s = 0; s < nb; s++) total += h[s]; /* K:1059-1062 */
        if (!(total <= 0)) {
            for (int s = 0; s < nb; s++) { /* K:1072-1080 */
                h[s] = h[s] / total;
                if (h[s] < 0) h[s] = 0;
                if (h[s] > 1) h[s] = 1;
            }
        }
        float mean = 0.0f; /* K:1086-1090 */
        for (int i = 0; i < nb; i++)
            mean = (float)((double)mean + (double)h[i] * ((double)(bw * (float)i) + (double)bw / 2.0));
        float var = 0.0f; /* K:1094-1098 */
        for (int i = 0; i < nb; i++) {
            const double d = ((double)(bw * (float)i) + (double)bw / 2.0) - (double)mean;
            var = (float)((double)var + (double)h[i] * d * d);
        }
        float ent = 0.0f; /* K:1106-1115 */
        for (int i = 0; i < nb; i++) {
            const float pr = h[i];
            const double t = pr <= 0 ? 0.0 : ((double)logf_bin(pr) / LN2_D);
            ent = (float)((double)ent + (double)pr * t);
        }
        ent = -ent;
        ent = ent / enorm;
        float *o = blocks + 4 * (size_t)n; /* flexBlockData[n], K:1117-1119 */
        o[0] = mean;
        o[1] = var;
        o[2] = ent;
        o[3] = 0.0f;
    }
    g_memo_f = NULL;
    return rc;
}

int64_t orc_render_flex(const float *blocks, int nblk, const orc_render_params *p,
                        uint32_t *out, float *out_f, int32_t *out_n, int row_start,
                        int row_stride, int nthreads) {
    vol_t v = {NULL, 1, 1, 1, 1, 0.0f, NULL, NULL, blocks, nblk};
    int64_t total = 0;
    run_rows(&v, p, out, out_f, out_n, row_start, row_stride, nthreads, &total);
    return total;
}

/* ------------------------------------------------------------------------ */
/* GMM distribution volumes (config 5)                 */
/* ------------------------------------------------------------------------ */

/* T(p) over the L = K/4 lane partials, in the order k_march_gmm's DPP steps
 * (quad_perm xor 1, xor 2, row_half_mirror) complete them:
 * L = 2: p0 + p1;  L = 4: (p0 + p1) + (p2 + p3);
 * L = 8: ((p0 + p1) + (p2 + p3)) + ((p4 + p5) + (p6 + p7)) */
static inline float gmm_tree(const float *p, int L) {
    if (L == 2) return p[0] + p[1];
    const float a = (p[0] + p[1]) + (p[2] + p[3]);
    if (L == 4) return a;
    return a + ((p[4] + p[5]) + (p[6] + p[7]));
}

/* lane s of a ray's group holds components 4s .. 4s + 3 */
float orc_gmm_stat(const float *wm, const float *sg, int K, int method) {
    const int L = K / 4;
    float pm[8] = {0}, pq[8] = {0};
    for (int l = 0; l < L; l++) {
        const int k0 = 4 * l;
        pm[l] = wm[2 * k0] * wm[2 * k0 + 1];
        for (int j = 1; j < 4; j++) pm[l] = fmaf(wm[2 * (k0 + j)], wm[2 * (k0 + j) + 1], pm[l]);
    }
    const float m = gmm_tree(pm, L);
    if (method == 1) return m;
    for (int l = 0; l < L; l++) {
        const int k0 = 4 * l;
        pq[l] = wm[2 * k0] * fmaf(sg[k0], sg[k0], wm[2 * k0 + 1] * wm[2 * k0 + 1]);
        for (int j = 1; j < 4; j++) {
            const int k = k0 + j;
            pq[l] = fmaf(wm[2 * k], fmaf(sg[k], sg[k], wm[2 * k + 1] * wm[2 * k + 1]), pq[l]);
        }
    }
    const float q = gmm_tree(pq, L);
    const float mm = m * m;
    return (q - mm) * 16.0f;
}

/* the generator's per-axis Gaussian tables; one voxel's
 * records follow from them and the voxel index alone (gmm_voxel), so the
 * resident slices and the procedural source below give identical records */
struct orc_gmm_proc {
    int nx, ny, nz, K;
    uint64_t seed;
    float amp[SYN_K];
    float *gx, *gy, *gz;
};

orc_gmm_proc *orc_gmm_proc_new(int nx, int ny, int nz, int K, uint64_t seed) {
    orc_gmm_proc *g = (orc_gmm_proc *)calloc(1, sizeof *g);
    if (!g) return NULL;
    g->nx = nx; g->ny = ny; g->nz = nz; g->K = K; g->seed = seed;
    g->gx = (float *)malloc(sizeof(float) * SYN_K * (size_t)nx);
    g->gy = (float *)malloc(sizeof(float) * SYN_K * (size_t)ny);
    g->gz = (float *)malloc(sizeof(float) * SYN_K * (size_t)nz);
    if (!g->gx || !g->gy || !g->gz) {
        orc_gmm_proc_free(g);
        return NULL;
    }
    for (int k = 0; k < SYN_K; k++) {
        double r[5];
        for (int j = 0; j < 5; j++) r[j] = u01(orc_splitmix64(seed + 0x100u + 8u * (uint64_t)k + (uint64_t)j));
        g->amp[k] = (float)(0.3 + 0.7 * r[0]);
        double sd = 0.05 + 0.15 * r[4];
        axis_table(nx, 0.2 + 0.6 * r[1], sd, g->gx + (size_t)k * nx);
        axis_table(ny, 0.2 + 0.6 * r[2], sd, g->gy + (size_t)k * ny);
        axis_table(nz, 0.2 + 0.6 * r[3], sd, g->gz + (size_t)k * nz);
    }
    return g;
}

void orc_gmm_proc_free(orc_gmm_proc *g) {
    if (!g) return;
    free(g->gx);
    free(g->gy);
    free(g->gz);
    free(g);
}

/* records of voxel (x, y, z): wm[K][2] (w, mu), sg[K] */
static void gmm_voxel(const orc_gmm_proc *g, int x, int y, int z, float *wm, float *sg) {
    const int nx = g->nx, ny = g->ny, K = g->K;
    float f = 0.0f;
    for (int k = 0; k < SYN_K; k++)
        f = f + ((g->amp[k] * g->gx[(size_t)k * nx + x]) * g->gy[(size_t)k * ny + y]) *
                    g->gz[(size_t)k * g->nz + z];
    if (f > 1.0f) f = 1.0f;
    const uint64_t v = ((uint64_t)z * (uint64_t)ny + (uint64_t)y) * (uint64_t)nx + (uint64_t)x;
    float sum = 0.0f;
    for (int k = 0; k < K; k++) {
        uint64_t h = orc_splitmix64(g->seed ^ 0x6A09E667F3BCC909ull ^ (v * (uint64_t)K + (uint64_t)k));
        sum = sum + (0.05f + (float)((h >> 16) & 0xFFFFFFull) * 0x1p-24f);
    }
    for (int k = 0; k < K; k++) {
        uint64_t h = orc_splitmix64(g->seed ^ 0x6A09E667F3BCC909ull ^ (v * (uint64_t)K + (uint64_t)k));
        const float u = (float)(h >> 40) * 0x1p-24f;
        const float r = 0.05f + (float)((h >> 16) & 0xFFFFFFull) * 0x1p-24f;
        float mu = (f * 0.8f + 0.1f) + (u - 0.5f) * 0.2f;
        mu = fminf(fmaxf(mu, 0.0f), 1.0f);
        wm[2 * k] = r / sum;
        wm[2 * k + 1] = mu;
        sg[k] = ((float)(h & 0xFFFFull) * 0x1p-16f) * 0.05f + 0.005f;
    }
}

void orc_synth_gmm(int nx, int ny, int nz, int K, uint64_t seed, int z_base, int nzs, float *wm,
                   float *sg, int nthreads) {
    orc_gmm_proc *g = orc_gmm_proc_new(nx, ny, nz, K, seed);
    if (!g) return;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
    for (int zl = 0; zl < nzs; zl++) {
        for (int y = 0; y < ny; y++) {
            for (int x = 0; x < nx; x++) {
                const uint64_t lv = ((uint64_t)zl * (uint64_t)ny + (uint64_t)y) * (uint64_t)nx + (uint64_t)x;
                gmm_voxel(g, x, y, zl + z_base, wm + lv * 2 * (uint64_t)K, sg + lv * (uint64_t)K);
            }
        }
    }
    (void)nthreads;
    orc_gmm_proc_free(g);
}

/* eye ray + intersectBox (K:288-306), as render_pixel */
static int gmm_ray(const orc_render_params *p, int x, int y, f3 *o, f3 *d, float *tnear,
                   float *tfar) {
    const float *M = p->inv_view;
    float u = ((float)x / (float)p->width) * 2.0f - 1.0f;
    float vv = ((float)y / (float)p->height) * 2.0f - 1.0f;
    o->x = 0.0f * M[0] + 0.0f * M[1] + 0.0f * M[2] + 1.0f * M[3];
    o->y = 0.0f * M[4] + 0.0f * M[5] + 0.0f * M[6] + 1.0f * M[7];
    o->z = 0.0f * M[8] + 0.0f * M[9] + 0.0f * M[10] + 1.0f * M[11];
    f3 d0 = {u, vv, -2.0f};
    float inv = rsqrt_read(dot3(d0, d0));
    d0.x = d0.x * inv; d0.y = d0.y * inv; d0.z = d0.z * inv;
    d->x = d0.x * M[0] + d0.y * M[1] + d0.z * M[2];
    d->y = d0.x * M[4] + d0.y * M[5] + d0.z * M[6];
    d->z = d0.x * M[8] + d0.y * M[9] + d0.z * M[10];
    f3 invR = {1.0f / d->x, 1.0f / d->y, 1.0f / d->z};
    f3 tbot = {invR.x * (-1.0f - o->x), invR.y * (-1.0f - o->y), invR.z * (-1.0f - o->z)};
    f3 ttop = {invR.x * (1.0f - o->x), invR.y * (1.0f - o->y), invR.z * (1.0f - o->z)};
    f3 tmin = {fminf(ttop.x, tbot.x), fminf(ttop.y, tbot.y), fminf(ttop.z, tbot.z)};
    f3 tmax = {fmaxf(ttop.x, tbot.x), fmaxf(ttop.y, tbot.y), fmaxf(ttop.z, tbot.z)};
    *tnear = fmaxf(fmaxf(tmin.x, tmin.y), fmaxf(tmin.x, tmin.z));
    *tfar = fminf(fminf(tmax.x, tmax.y), fminf(tmax.x, tmax.z));
    if (!(*tfar > *tnear)) return 0;
    if (*tnear < 0.0f) *tnear = 0.0f;
    return 1;
}

static inline const float *gmm_wm(const orc_gmm *v, int x, int y, int z) {
    size_t i = ((size_t)(z - v->z_base) * (size_t)v->ny + (size_t)y) * (size_t)v->nx + (size_t)x;
    return v->wm + i * 2 * (size_t)v->K;
}
static inline const float *gmm_sg(const orc_gmm *v, int x, int y, int z) {
    size_t i = ((size_t)(z - v->z_base) * (size_t)v->ny + (size_t)y) * (size_t)v->nx + (size_t)x;
    return v->sg + i * (size_t)v->K;
}
static inline void gmm_mark(const orc_gmm *v, uint64_t *mark, int x, int y, int z) {
    size_t idx = ((size_t)z * (size_t)v->ny + (size_t)y) * (size_t)v->nx + (size_t)x;
    __atomic_fetch_or(&mark[idx >> 6], (uint64_t)1 << (idx & 63), __ATOMIC_RELAXED);
}

/* march one ray (state in/out) through the slab; returns 1 if it leaves the
 * slab alive, 0 if it ended (early exit, tfar, 500 samples) */
static int gmm_march(const orc_gmm *v, const orc_gmm_proc *proc, const orc_render_params *p,
                     int z_lo, int z_hi, int slab, f3 d, float tfar, orc_gmm_ray *s,
                     uint64_t *mark) {
    float pwm[64], psg[32]; /* proc: one voxel's records, K <= 32 */
    const f3 step = {d.x * 0.01f, d.y * 0.01f, d.z * 0.01f};
    for (;;) {
        int x0, x1, y0, y1, z0, z1;
        float ax, ay, az;
        lin_axis(s->pos[0] * 0.5f + 0.5f, v->nx, &x0, &x1, &ax);
        lin_axis(s->pos[1] * 0.5f + 0.5f, v->ny, &y0, &y1, &ay);
        lin_axis(s->pos[2] * 0.5f + 0.5f, v->nz, &z0, &z1, &az);
        if (slab && (z0 < z_lo || z0 >= z_hi)) return 1;
        const int xs[2] = {x0, x1}, ys[2] = {y0, y1}, zs[2] = {z0, z1};
        float sv[8];
        for (int j = 0; j < 8; j++) {
            const int X = xs[j & 1], Y = ys[(j >> 1) & 1], Z = zs[j >> 2];
            if (mark) gmm_mark(v, mark, X, Y, Z);
            if (proc) {
                gmm_voxel(proc, X, Y, Z, pwm, psg);
                sv[j] = orc_gmm_stat(pwm, psg, v->K, p->query_method);
            } else {
                sv[j] = orc_gmm_stat(gmm_wm(v, X, Y, Z), gmm_sg(v, X, Y, Z), v->K, p->query_method);
            }
        }
        float c00 = lerpq(sv[0], sv[1], ax), c10 = lerpq(sv[2], sv[3], ax);
        float c01 = lerpq(sv[4], sv[5], ax), c11 = lerpq(sv[6], sv[7], ax);
        float c0 = lerpq(c00, c10, ay), c1 = lerpq(c01, c11, ay);
        const float sample = lerpq(c0, c1, az);
        s->n = s->n + 1;
        float col[4];
        orc_transfer((sample - p->transfer_offset) * p->transfer_scale, col); /* K:683 */
        col[3] = col[3] * p->density;
        col[0] = col[0] * col[3];
        col[1] = col[1] * col[3];
        col[2] = col[2] * col[3];
        const float om = 1.0f - s->sum[3];
        s->sum[0] = s->sum[0] + col[0] * om;
        s->sum[1] = s->sum[1] + col[1] * om;
        s->sum[2] = s->sum[2] + col[2] * om;
        s->sum[3] = s->sum[3] + col[3] * om;
        if (s->sum[3] > 0.95f) return 0;    /* K:698 */
        s->t = s->t + 0.01f;                /* K:701 */
        const int end = s->t > tfar || s->n >= 500; /* K:703, K:381 */
        s->pos[0] = s->pos[0] + step.x;     /* K:706 */
        s->pos[1] = s->pos[1] + step.y;
        s->pos[2] = s->pos[2] + step.z;
        if (end) return 0;
    }
}

/* alive-list entries: 9 words, pix | n << 23 in the last (vr_gmm.hip GmmRay) */
static orc_gmm_ray gmm_unpack(const uint32_t *w) {
    orc_gmm_ray s;
    memcpy(s.sum, w, 4 * sizeof(float));
    memcpy(&s.t, w + 4, sizeof(float));
    memcpy(s.pos, w + 5, 3 * sizeof(float));
    s.pix = w[8] & ((1u << 23) - 1u);
    s.n = w[8] >> 23;
    return s;
}

static void gmm_pack(const orc_gmm_ray *s, uint32_t *w) {
    memcpy(w, s->sum, 4 * sizeof(float));
    memcpy(w + 4, &s->t, sizeof(float));
    memcpy(w + 5, s->pos, 3 * sizeof(float));
    w[8] = s->pix | (s->n << 23);
}

int64_t orc_render_gmm(const orc_gmm *v, const orc_render_params *p, int z_lo, int z_hi,
                       const uint32_t *rays_in, uint32_t n_in, uint32_t *rays_out,
                       uint32_t *n_out, uint32_t *out, float *out_f, int32_t *out_n,
                       uint64_t *mark) {
    const int slab = rays_out != NULL;
    const uint64_t n = rays_in ? (uint64_t)n_in : (uint64_t)p->width * (uint64_t)p->height;
    int64_t samples = 0;
    uint32_t k_out = 0;
    for (uint64_t i = 0; i < n; i++) {
        orc_gmm_ray s;
        memset(&s, 0, sizeof s);
        f3 o, d;
        float tnear, tfar;
        int x, y;
        if (rays_in) {
            s = gmm_unpack(rays_in + i * ORC_GMM_RAY_WORDS);
            x = (int)(s.pix % (uint32_t)p->width);
            y = (int)(s.pix / (uint32_t)p->width);
            if (!gmm_ray(p, x, y, &o, &d, &tnear, &tfar)) continue; /* not produced by a slab */
        } else {
            x = (int)(i % (uint64_t)p->width);
            y = (int)(i / (uint64_t)p->width);
            s.pix = (uint32_t)i;
            if (!gmm_ray(p, x, y, &o, &d, &tnear, &tfar)) {
                if (out_n) out_n[i] = -1;  /* K:302-303: no write */
                continue;
            }
            s.t = tnear;
            s.pos[0] = o.x + d.x * tnear;
            s.pos[1] = o.y + d.y * tnear;
            s.pos[2] = o.z + d.z * tnear;
        }
        const uint32_t n0 = s.n;
        const int alive = gmm_march(v, NULL, p, z_lo, z_hi, slab, d, tfar, &s, mark);
        samples += (int64_t)(s.n - n0);
        if (alive) {
            gmm_pack(&s, rays_out + (uint64_t)(k_out++) * ORC_GMM_RAY_WORDS);
            continue;
        }
        const float rgba[4] = {s.sum[0] * p->brightness, s.sum[1] * p->brightness,
                               s.sum[2] * p->brightness, s.sum[3] * p->brightness};
        if (out_n) out_n[s.pix] = (int32_t)s.n;
        if (out) out[s.pix] = orc_pack(rgba);
        if (out_f) {
            out_f[(size_t)s.pix * 4 + 0] = sat(rgba[0]);
            out_f[(size_t)s.pix * 4 + 1] = sat(rgba[1]);
            out_f[(size_t)s.pix * 4 + 2] = sat(rgba[2]);
            out_f[(size_t)s.pix * 4 + 3] = sat(rgba[3]);
        }
    }
    if (n_out) *n_out = k_out;
    return samples;
}

int64_t orc_render_gmm_rows(const orc_gmm *v, const orc_render_params *p, int row_lo, int row_hi,
                            uint32_t *out, int nthreads) {
    int64_t acc = 0;
    if (row_lo < 0) row_lo = 0;
    if (row_hi > p->height) row_hi = p->height;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(+ : acc)
#endif
    for (int y = row_lo; y < row_hi; y++) {
        for (int x = 0; x < p->width; x++) {
            f3 o, d;
            float tnear, tfar;
            if (!gmm_ray(p, x, y, &o, &d, &tnear, &tfar)) continue;
            orc_gmm_ray s;
            memset(&s, 0, sizeof s);
            s.pix = (uint32_t)y * (uint32_t)p->width + (uint32_t)x;
            s.t = tnear;
            s.pos[0] = o.x + d.x * tnear;
            s.pos[1] = o.y + d.y * tnear;
            s.pos[2] = o.z + d.z * tnear;
            gmm_march(v, NULL, p, 0, v->nz, 0, d, tfar, &s, NULL);
            acc += s.n;
            const float rgba[4] = {s.sum[0] * p->brightness, s.sum[1] * p->brightness,
                                   s.sum[2] * p->brightness, s.sum[3] * p->brightness};
            if (out) out[s.pix] = orc_pack(rgba);
        }
    }
    (void)nthreads;
    return acc;
}

int64_t orc_render_gmm_rows_proc(const orc_gmm_proc *g, const orc_render_params *p,
                                 const int32_t *rows, int nrows, uint32_t *out, int32_t *out_n,
                                 int nthreads) {
    if (!g || g->K < 4 || g->K > 32) return -1;
    const orc_gmm v = {NULL, NULL, g->nx, g->ny, g->nz, g->K, 0, g->nz};
    const int W = p->width;
    int64_t acc = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads) reduction(+ : acc)
#endif
    for (int64_t i = 0; i < (int64_t)nrows * W; i++) {
        const int r = (int)(i / W), x = (int)(i % W), y = rows[r];
        out[i] = 0;
        out_n[i] = -1;
        f3 o, d;
        float tnear, tfar;
        if (!gmm_ray(p, x, y, &o, &d, &tnear, &tfar)) continue;
        orc_gmm_ray s;
        memset(&s, 0, sizeof s);
        s.t = tnear;
        s.pos[0] = o.x + d.x * tnear;
        s.pos[1] = o.y + d.y * tnear;
        s.pos[2] = o.z + d.z * tnear;
        gmm_march(&v, g, p, 0, g->nz, 0, d, tfar, &s, NULL);
        acc += s.n;
        const float rgba[4] = {s.sum[0] * p->brightness, s.sum[1] * p->brightness,
                               s.sum[2] * p->brightness, s.sum[3] * p->brightness};
        out[i] = orc_pack(rgba);
        out_n[i] = (int32_t)s.n;
    }
    (void)nthreads;
    return acc;
}
