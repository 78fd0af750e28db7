// vr_device.h -- device-side arithmetic of the d_render path for gfx950.
//
// Every function evaluates the reference expression it cites with the
// canonical arithmetic of DESIGN.md section 3: ISO C promotions as written in
// the reference source, no FMA contraction (the library is compiled with
// -ffp-contract=off), correctly rounded division/sqrt, CUDA texture-fetch
// rules with 8-bit fractional filter weights.  K = volumeRender_kernel.cu.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vr_logtab.h"

// log(2.0), correctly rounded (K:766)
#define VR_LN2_D 0x1.62e42fefa39efp-1

namespace vr {

constexpr int kMaxSteps = 500;             // K:276
constexpr float kTStep = 0.01f;            // K:277
constexpr float kOpacityThreshold = 0.95f; // K:278
constexpr int kTileW = 64;                 // tile = one 256-thread workgroup:
constexpr int kTileH = 4;                  //   64 x 4 pixels, one row per wave
constexpr uint32_t kPad = 0xFFFFFFFFu;     // tile-list padding

struct Params {
    float m[12];                 // c_invViewMatrix (K:116), row-major 3x4
    uint32_t W, H;
    uint32_t CW, CH;             // pixels rendered: x < CW, y < CH (render_kernel's grid
                                 // coverage, C:122 / K:2397; W, H otherwise)
    float density, brightness, toff, tscale;
    int nx, ny, nz;              // resident volume dims
    uint64_t sy, sz;             // record pitch of a voxel row / slice in HBM
    int m7x, m7y, m7z;           // render_kernel volumeSize (method 7)
    float enorm;                 // log((float)B)/log(2.0f), K:769
    int nb;                      // bins per record
    uint32_t tiles_x;            // ceil(W/16)
    const uint32_t *perm;        // full frame: tile of workgroup b (nullptr: xcd_slot order)
    uint32_t n_tiles;            // tiles in this launch
    const uint32_t *tile_list;   // nullptr: tile = launch slot
    uint32_t *out;
    float *out_f;
    int32_t *out_n;
    unsigned long long *mark;    // footprint bitset (count mode only)
    int box_max;                 // LDS-staged footprint box capacity (voxels per wave), 0 = off
    int wg_per_cu;               // occupancy cap through the LDS request (0 = none)
    int lds_cu, lds_wg;          // LDS bytes per CU / per workgroup (device attributes)
    int oblique;                 // view's screen x does not run along voxel rows
    int path;                    // kernel variant (vr_api.cpp fill_params)
    // 2x2 (x, y) micro-brick copy of the 8-bin records for the quad marches of
    // oblique views (nullptr: none), bsy / bsz its brick-row / slice pitches
    // in records (brick_index); the launch passes it as vol with sy / sz = bsy / bsz
    const float *bvol;
    uint64_t bsy, bsz;
    // axis-rows copy of the records (B <= 8) for views whose screen x runs along
    // the volume's y or z axis: record (x, y, z) at x * asx + y * asy + z * asz
    // (axis_copy_strides); the launch passes it as vol with sx / sy / sz = asx / asy / asz
    const float *avol;
    uint64_t asx, asy, asz;
    int axis_view;               // host dispatch: 1 / 2 = the view runs along y / z (fill_params)
    uint64_t sx;                 // record stride of x (gather MODE 3 only; 1 in x rows)
    // fractal/template codec (methods 4/5/6): codebook int4 per voxel, templates
    // [ntpl][nb], (bin, value) errors [voxel][err_slots]
    const int4 *cb;
    const float *tpl;
    const float2 *err;
    int ntpl, err_slots;
    int tpl_lds;                 // codec march: template table copied to LDS (bytes, 0 = no)
    int seg_lanes;               // ray-segmented march (path 7): lanes per ray
    // flexible blocks (methods 8/9/0): per-block (mean, variance, entropy, 0)
    const float4 *flex;
    int nflex;                   // blocks per axis
    // tooling (vr_debug_wave_clock): per wave {start, end, hw id} of the
    // per-ray pipelined, quad and ray-segmented marches, nullptr = off; slot
    // s's waves at [s * 4 + wave] (pipe, quad), [s * 8 + half * 4 + wave]
    // (quad2), [s * 16 + part * 4 + wave] (segmented)
    unsigned long long *wave_clock;
    // adaptive tile order: per-tile cost record of the pipelined march
    // (record_tile_cost), indexed by tile id, nullptr = off
    uint32_t *tile_cost;
    // GMM volumes (vr_gmm.hip): K components per voxel in
    // two planes, (w, mu) pairs [voxel][K][2] and sigma [voxel][K], voxel
    // order x + nx*(y + ny*(z - z_base)) for the resident slices
    // [z_base, z_base + nzs); nx/ny/nz above are the whole volume's dims.
    const float *gwm, *gsg;
    int gk;
    int z_base, nzs;
    int z_lo, z_hi;              // slab: samples whose footprint z0 lies in [z_lo, z_hi)
    const uint32_t *rays_in;     // slab chain: alive rays entering (GmmRay, 9 words), nullptr = camera
    uint32_t n_rays_in;
    uint32_t *rays_out;          // alive rays leaving the slab (nullptr: slab = whole volume)
    uint32_t *n_rays_out;
    int wq_map;                  // k_march_wq pixel map: 0 a 64-pixel row per wave, 1 16x4 blocks
    int quad2;                   // quad march with two lanes per ray (k_march_quad2)
    // ray-segmented march of a tile list: the first head_slots slots (a multiple
    // of 8: the longest tiles of every XCD sublist) take head_lanes lanes per ray
    // in the same launch (k_march_seg_head), the rest seg_lanes; 0 = off
    uint32_t head_slots;
    int head_lanes;
    int head_tail;               // the rest of such a list: 0 seg_lanes windows, 1 one lane per ray (k_march_pipe_head)
    int plane_axis;              // baked frame on a plane's copy: 1 y rows, 2 z rows (gather8 MODE 4 / 5), 3 8x2x2 bricks (MODE 6)
    int seg_map;                 // segmented / pipelined marches: 1 = a wave's rays as a compact pixel block (tuning)
    int duo;                     // LDS-box march (path 1, B <= 8, m1/m2/m3): samples per box (k_march_duo), 0/1 = k_march
    // tooling (vr_debug_box_check): 6 x u64, [0] violations, [1] worst overrun,
    // [2] out-of-volume box voxels, [3] decoded voxels, [4] lane slots, [5] spare
    unsigned long long *box_check;
};

// Record index of voxel (x, y, z) in the 2x2 (x, y) micro-brick layout (one
// 128-B line = the 4 records of an even (x, y) pair of rows, 8 bins): bsy
// records per brick row (2 * the even-padded width), bsz per slice.
__host__ __device__ __forceinline__ uint64_t brick_index(uint64_t x, uint64_t y, uint64_t z,
                                                         uint64_t bsy, uint64_t bsz) {
    return z * bsz + (y >> 1) * bsy + (x >> 1) * 4u + (y & 1u) * 2u + (x & 1u);
}

// Record strides of the axis-rows copy whose rows run along `axis` (1 = y,
// 2 = z): that axis is contiguous, then the other two in x, y, z order of
// increasing stride (y rows: y, x, z; z rows: z, y, x -- the z-slice order of
// the x-row layout for the slowest axis where it can be kept).
__host__ __device__ __forceinline__ void axis_copy_strides(int axis, uint64_t nx, uint64_t ny,
                                                           uint64_t nz, uint64_t &sx,
                                                           uint64_t &sy, uint64_t &sz) {
    if (axis == 1) {
        sy = 1; sx = ny; sz = nx * ny;
    } else {
        sz = 1; sy = nz; sx = nz * ny;
    }
}

// Baked statistics planes (basicDataProcessing, vr_stats.hip): 16 x 2 x 1
// bricks -- one 128-B line holds 16 x-neighbours of two y rows -- whose x
// runs overlap by one voxel (brick kx covers x = 15 kx .. 15 kx + 15), so the
// x-pair of every footprint is one 8-byte load inside one line.  Row pitch
// (floats per row of bricks, two y rows) and slice pitch: plane_pitches.  Fewer
// distinct lines per frame than x rows at both the row-aligned and the oblique
// bench views (simulated per 64x4 tile at 1024^3: C0 1.80 -> 1.57 GB, C1 4.47 ->
// 3.79; tools/footprint_sim.c LAYOUT=10).
constexpr uint32_t kPlaneStride = 15;  // x step between bricks (16 wide: one apron voxel)
__host__ __device__ __forceinline__ void plane_pitches(uint32_t nx, uint32_t ny, uint64_t &sy,
                                                       uint64_t &sz) {
    const uint64_t nbx = nx > 0 ? (uint64_t)(nx - 1) / kPlaneStride + 1 : 0;
    sy = nbx * 32u;
    sz = (uint64_t)((ny + 1) / 2) * sy;
}
// x / 15 for x < 2^16, and the offset of x's pair (x, x + 1) in its brick row
__host__ __device__ __forceinline__ uint32_t plane_bx(uint32_t x) {
    const uint32_t kx = (x * 0x8889u) >> 19;
    return kx * 32u + (x - kPlaneStride * kx);
}
// plane index of voxel (x, y, z) in the brick whose run starts at or below x
// by at most 14 (its home); x = 15 k (k > 0) is also stored at offset 15 of
// brick k - 1, where pairs starting at 15 k - 1 read it
// (a slice, (Y + 1) / 2 * sy floats, is < 2^32: the in-slice part is 32-bit and
// the index one 64-bit multiply-add)
__host__ __device__ __forceinline__ uint64_t plane_index(uint32_t x, uint32_t y, uint32_t z,
                                                         uint64_t sy, uint64_t sz) {
    return (uint64_t)z * sz + (uint32_t)((y >> 1) * (uint32_t)sy + (y & 1u) * 16u + plane_bx(x));
}

// Oblique-view copy of a baked plane (round 5): 8 x 2 x 2 bricks -- one 128-B
// line holds 8 x-neighbours of two y rows and two z slices -- whose x runs
// overlap by one voxel (brick kx covers x = 7 kx .. 7 kx + 7), so a footprint's
// x-pair is still one 8-byte load and its z pair often shares the line.  Row
// pitch sy (floats per row of bricks: a y pair), slice-pair pitch sz.
constexpr uint32_t kPlane8Stride = 7;
__host__ __device__ __forceinline__ void plane8_pitches(uint32_t nx, uint32_t ny, uint64_t &sy,
                                                        uint64_t &sz) {
    const uint64_t nbx = nx > 0 ? (uint64_t)(nx - 1) / kPlane8Stride + 1 : 0;
    sy = nbx * 32u;
    sz = (uint64_t)((ny + 1) / 2) * sy;
}
// x / 7 (exact for x < 2^30: 0x24924925 = (2^32 + 3) / 7) and the offset of
// x's pair (x, x + 1) in its brick row
__host__ __device__ __forceinline__ uint32_t plane8_bx(uint32_t x) {
    const uint32_t kx = (uint32_t)(((uint64_t)x * 0x24924925ull) >> 32);
    return kx * 32u + (x - kPlane8Stride * kx);
}
// index of voxel (x, y, z) in its home brick (x = 7 k, k > 0, is also stored at
// offset 7 of brick k - 1, where pairs starting at 7 k - 1 read it)
__host__ __device__ __forceinline__ uint64_t plane8_index(uint32_t x, uint32_t y, uint32_t z,
                                                          uint64_t sy, uint64_t sz) {
    return (uint64_t)(z >> 1) * sz +
           (uint32_t)((y >> 1) * (uint32_t)sy + (y & 1u) * 8u + (z & 1u) * 16u + plane8_bx(x));
}

constexpr int kBoxMax = 1024;    // default per-wave box capacity (4 KiB of f32 statistics)


__device__ __forceinline__ float clamp01(float u) { return fminf(fmaxf(u, 0.0f), 1.0f); }

// 9-bit fixed-point filter weight, 8 fractional bits
__device__ __forceinline__ float q8(float a) { return rintf(a * 256.0f) * (1.0f / 256.0f); }

__device__ __forceinline__ float lerpq(float a, float b, float t) {
    return (1.0f - t) * a + t * b;
}

// linear filter, normalised coordinate, clamp addressing (K:1865-1869)
__device__ __forceinline__ void lin_axis(float u, int n, int &i0, int &i1, float &a) {
    u = clamp01(u);
    float xb = u * (float)n - 0.5f;
    float fl = floorf(xb);
    float fr = xb - fl;
    int i = (int)fl;
    a = q8(fr);
    i0 = max(0, min(n - 1, i));
    i1 = max(0, min(n - 1, i + 1));
}

// point filter, normalised coordinate, clamp (index volume tex, K:2161-2165)
__device__ __forceinline__ int point_axis(float u, int n) {
    u = clamp01(u);
    int i = (int)floorf(u * (float)n);
    return min(i, n - 1);
}

// transfer function (K:2323-2326), linear / normalised / clamp (K:2337-2339)
// The 9 entries as bit masks (entry i = bit i; g in 2-bit fields of halves):
// r 0,1,1,1,0,0,0,1,0  g 0,0,.5,1,1,1,0,0,0  b 0,0,0,0,0,1,1,1,0  a 0,1,1,1,1,1,1,1,0
// -- one bit-field extract + convert per channel instead of compare chains.
__device__ __forceinline__ float4 tf_entry(int i) {
    const uint32_t u = (uint32_t)i;  // 0 <= i <= 8 (lin_axis clamps)
    const float r = (float)((0x08Eu >> u) & 1u);
    const float g = (float)((0xA90u >> (2u * u)) & 3u) * 0.5f;
    const float b = (float)((0x0E0u >> u) & 1u);
    const float a = (float)((0x0FEu >> u) & 1u);
    return make_float4(r, g, b, a);
}

__device__ __forceinline__ float4 transfer(float x) {
    int i0, i1;
    float a;
    lin_axis(x, 9, i0, i1, a);
    const float4 t0 = tf_entry(i0), t1 = tf_entry(i1);
    return make_float4(lerpq(t0.x, t1.x, a), lerpq(t0.y, t1.y, a), lerpq(t0.z, t1.z, a),
                       lerpq(t0.w, t1.w, a));
}

__device__ __forceinline__ float sat(float x) {  // __saturatef, NaN -> 0
    return (x > 0.0f) ? (x > 1.0f ? 1.0f : x) : 0.0f;
}

// rgbaFloatToInt, K:186-193
__device__ __forceinline__ uint32_t pack_rgba(float r, float g, float b, float a) {
    r = sat(r); g = sat(g); b = sat(b); a = sat(a);
    return ((uint32_t)(a * 255.0f) << 24) | ((uint32_t)(b * 255.0f) << 16) |
           ((uint32_t)(g * 255.0f) << 8) | (uint32_t)(r * 255.0f);
}

// Division by a constant with the reference's double rounding: q0 = m*R,
// corrected once with an exact FMA residual (Markstein), R = RN(1/D).
// tests/c/divcheck.c proves it bit-identical to `m / D` for every float m
// and each of the three divisors below (~16 cycles instead of ~58 for the
// full IEEE double-division sequence on gfx950).
__device__ __forceinline__ double div_const(double m, double D, double R) {
#ifdef VR_ABLATE_DIV  // timing ablation builds only (tools/build_variants.sh): NOT exact
    return m * R;
#endif
    const double q0 = m * R;
    const double e = __builtin_fma(-q0, D, m);
    const double q = __builtin_fma(e, R, q0);
    return (q0 == 0.0 || __builtin_isinf(q0)) ? q0 : q;
}
constexpr double kMeanD = 0.0217, kMeanR = 1.0 / 0.0217;          // K:758
constexpr double kVarD = 0.000021, kVarR = 1.0 / 0.000021;        // K:759

// (float)((double)m / D) for a float m when only the float rounding is kept:
// the reciprocal multiply (float)((double)m * (1/D)) is bit-identical for
// every one of the 2^32 float inputs for D = 0.0217 and 0.000021
// (tests/c/divcheck.c) -- no Markstein correction, no 0 / inf selects.
__device__ __forceinline__ float div_to_float(float m, double R) {
    return (float)((double)m * R);
}

// (float)((double)v / 0.000021) (K:759) without f64 in the common case: one
// FMA against the reciprocal split in two floats for |v| in [2^-100, FLT_MAX];
// zeros and infinities give v * Ch, NaN propagates, and the tiny inputs with
// subnormal quotients take div_to_float.  Bit-identical for every one of the 2^32
// float inputs (tests/c/divcheck.c, div_var_f32).
__device__ __forceinline__ float div_var_f32(float v) {
    constexpr float Ch = (float)kVarR;
    constexpr float Cl = (float)(kVarR - (double)Ch);
    const float av = __builtin_fabsf(v);
    if (av >= 0x1p-100f && av <= 0x1.fffffep127f) return __builtin_fmaf(v, Ch, v * Cl);
    if (v == 0.0f || !(av <= 0x1.fffffep127f)) return v * Ch;
    return div_to_float(v, kVarR);
}

// binWidth, K:736-738
__device__ __forceinline__ float bin_width(int nb) {
    const float maxh = (float)0.0217;
    return (maxh - 0.0f) / (float)nb;
}

// K:742-747: mean += p * (binWidth * i + binWidth / 2.0), float accumulator.
// The bin centre c_i = (double)(bw * i) + bw / 2.0 is a sum of two floats a
// few binades apart, so it has at most 29 significant bits for B <= 16
// (tests/test_oracle.py::test_bin_centres_fit_29_bits); the double product
// (double)p * c_i of a 24-bit float is then exact, and
// (double)mean + p * c_i rounded once is exactly fma(p, c_i, mean): one f64
// op per bin fewer, bit-identical.  B = 32: 23 of the 32 centres fit 29 bits
// and take the fused form, bins 23-31 (30 bits) keep mul + add; the choice is
// made per bin at compile time (centre_bits evaluates the same float / double
// expressions as the loop below).
constexpr int centre_bits(int nb, int i) {
    const float maxh = (float)0.0217;
    const float bw = (maxh - 0.0f) / (float)nb;          // bin_width
    double c = (double)(bw * (float)i) + (double)bw / 2.0;
    while (c < 4503599627370496.0) c *= 2.0;            // scale into [2^52, 2^53): exact
    while (c >= 9007199254740992.0) c *= 0.5;
    unsigned long long m = (unsigned long long)c;
    int b = 53;
    while ((m & 1ull) == 0ull) {
        m >>= 1;
        b--;
    }
    return b;
}

template <int B, int I>
__device__ __forceinline__ void mean_bins(const float (&p)[B], float bw, double half, float &mean) {
    if constexpr (I < B) {
        const double c = (double)(bw * (float)I) + half;
#ifndef VR_NO_FMA_MEAN  // A/B builds only
        constexpr bool fused = centre_bits(B, I) <= 29;
#else
        constexpr bool fused = false;
#endif
        if constexpr (fused) mean = (float)__builtin_fma((double)p[I], c, (double)mean);
        else mean = (float)((double)mean + (double)p[I] * c);
        mean_bins<B, I + 1>(p, bw, half, mean);
    }
}

template <int B>
__device__ __forceinline__ float raw_mean(const float (&p)[B]) {
    const float bw = bin_width(B);
    const double half = (double)bw / 2.0;
    float mean = 0.0f;
    mean_bins<B, 0>(p, bw, half, mean);
    return mean;
}
static_assert(centre_bits(16, 15) == 29 && centre_bits(32, 22) == 29 && centre_bits(32, 23) == 30,
              "bin-centre widths (tests/test_oracle.py::test_bin_centres_fit_29_bits)");

// K:749-755 (float arithmetic)
template <int B>
__device__ __forceinline__ float raw_variance(const float (&p)[B], float mean) {
    const float maxh = (float)0.0217;
    float var = 0.0f;
#pragma unroll
    for (int i = 0; i < B; i++) {
        const float d = ((float)i / (float)B) * maxh - mean;
        var = var + p[i] * d * d;
    }
    return var;
}

// log of a float as the reference evaluates it, (float)log((double)x)
// (DESIGN.md section 3), for finite x > 0.  y = log x is evaluated in double
// to ~2^-52 relative; unless y lies within 2^-44 |y| of a float rounding
// midpoint, rounding y to float already gives the rounding of the exact
// logarithm -- and so of the double log -- and only the remaining ~2^-20 of
// inputs evaluate the double log.  Exhaustively equal to (float)log((double)x)
// over all positive floats (vr_selftest_logf, tests/test_gpu_parity.py).
//
// Reduction (vr_logtab.h, tools/gen_logtab.py): x = m 2^e with m in [0.75,
// 1.5) (exact frexpf, one doubling), c = 0.75 + i/256 the nearest of 193
// centres -- m + 1.5 * 2^15 rounds m to a multiple of 2^-8 (the ulp there), so
// c = (m + K) - K exactly and i is read off the sum's bits, no conversions --
// d = m - c exact (Sterbenz), r = d / c as d * RN(1/c) in double (|r| <=
// 2^-8.58), log x = e ln2 + log c + log1p r with log1p r = r + r^2 (-1/2 +
// r/3 - r^2/4 + r^3/5) (truncation < r^6/6: <= 2^-45.5 relative to the
// result, whose smallest values |log x| >= 2^-9 away from c = 1 have |r| <=
// 2^-9).  x near 1 has e = 0 and c = 1, so e ln2 + log c never cancels: plain
// double arithmetic, one fma and one add for the sum (round 6: the 65-centre
// form on m in [1, 2) needed degree 7 and a double-double sum -- 1024^3 x 8
// C0 entropy 3.52 ms, of which the exact logarithm took 1.53 ms by ablation,
// profiles/r06/logtab/).  The midpoint test reads y's low 29 mantissa bits (a
// float's half-ulp pattern is 1 << 28 there whatever y's binade): more than
// 512 double ulps (~2^-43 |y|) from a midpoint, the float rounding of y is
// that of the exact logarithm.  Infinities and NaN leave the fast form.
__device__ __forceinline__ bool logf_fast_tabp(float x, float &r, const LogEnt *tab) {
    constexpr float kRound = 49152.0f;         // 1.5 * 2^15: ulp 2^-8
    int e;
    float m = frexpf(x, &e);                   // x = m 2^e, m in [0.5, 1), also subnormal x
    if (m < 0.75f) {
        m = m * 2.0f;                          // [1, 1.5), exact
        e -= 1;
    }
    const float s = m + kRound;                // m rounded to 2^-8 (+ kRound)
    const float c = s - kRound;                // exact: 0.75 + i/256
    const float d = m - c;                     // exact, |d| <= 1/512
    // i = 256 c - 192 = bits(s) - bits(kRound) - 192 (one ulp of s per 2^-8)
    // (clamped: an infinite or NaN x, which leaves the fast form, must not
    // index past the table)
    const uint32_t i = min(__float_as_uint(s) - (__float_as_uint(kRound) + 192u), 192u);
    const LogEnt t = tab[i];
    const double rr = (double)d * t.inv;
    double q = 1.0 / 5.0;
    q = fma(q, rr, -1.0 / 4.0);
    q = fma(q, rr, 1.0 / 3.0);
    q = fma(q, rr, -0.5);
    const double p = fma(rr * rr, q, rr);      // log1p(rr)
    const double y = fma((double)e, kLn2, t.hi) + p;
    r = (float)y;
    // |lo29 - 2^28| > 512 in 32-bit unsigned arithmetic: one sub, one compare
    const uint32_t lo29 = __double2loint(y) & 0x1FFFFFFFu;
    return __float_as_uint(x) < 0x7F800000u &&                  // finite (x > 0 here)
           lo29 - (0x10000000u - 512u) > 1024u;                 // > ~2^-43 |y| from a midpoint
}

// the table in constant memory / a copy in the kernel's LDS (copy_logtab)
__device__ __forceinline__ bool logf_fast_tab(float x, float &r) {
    return logf_fast_tabp(x, r, kLogTab);
}

// Copies the log table into LDS (kLogTabN x 16 bytes); the workgroup must
// then __syncthreads() before the first use.
__device__ __forceinline__ void copy_logtab(LogEnt *dst) {
    for (uint32_t i = threadIdx.x; i < (uint32_t)kLogTabN; i += blockDim.x) dst[i] = kLogTab[i];
}

// The round-1 form: atanh series of (m - 1)/(m + 1), one f64 division, no
// table.  Kept for the kernels where the table's memory loads sit on the
// critical path: the wave-staged and quad entropy marches (methods 3) measured
// slower with the table (1024^3 x 8: C0 4.96 -> 5.33 ms, C1 11.4 -> 12.1), the
// codec entropy (method 6, 8 decodes per sample) faster (C0 23.6 -> 12.5).
__device__ __forceinline__ bool logf_fast_series(float x, float &r) {
    int e;
    double m = frexp((double)x, &e);  // x = m 2^e, m in [0.5, 1)
    if (m < 0.70710678118654752440) {
        m = m * 2.0;
        e -= 1;
    }
    const double s = (m - 1.0) / (m + 1.0);  // |s| <= 0.1716
    const double z = s * s;
    // log m = 2 atanh s = 2s (1 + z/3 + z^2/5 + ... + z^8/17), remainder < 2^-50
    double q = 1.0 / 17.0;
    q = fma(q, z, 1.0 / 15.0);
    q = fma(q, z, 1.0 / 13.0);
    q = fma(q, z, 1.0 / 11.0);
    q = fma(q, z, 1.0 / 9.0);
    q = fma(q, z, 1.0 / 7.0);
    q = fma(q, z, 1.0 / 5.0);
    q = fma(q, z, 1.0 / 3.0);
    const double s2 = s + s;
    const double y = fma((double)e, VR_LN2_D, fma(s2 * z, q, s2));
    r = (float)y;
    if (r == 0.0f) return false;                  // x near 1: let the double log decide
    const double d = y - (double)r;               // exact
    int er;
    const float mr = frexpf(fabsf(r), &er);       // |r| = mr 2^er
    double half = ldexp(1.0, er - 25);            // half an ulp of r
    if (mr == 0.5f && d * (double)r < 0.0) half *= 0.5;  // below a power of two
    return fabs(fabs(d) - half) > 0x1p-44 * fabs(y);
}

template <bool TAB = false>
__device__ __forceinline__ float logf_canon(float x) {
    float r;
    if (x == 1.0f) return 0.0f;
    if (TAB ? logf_fast_tab(x, r) : logf_fast_series(x, r)) return r;
    return (float)log((double)x);
}

__device__ __forceinline__ float logf_canon_p(float x, const LogEnt *tab) {
#ifdef VR_ABLATE_LOG  // timing ablation builds only (tools/build_variants.sh): NOT exact
    return __logf(x);
#endif
    float r;  // x = 1 takes the fast form: i = 64, c = 1, d = 0, y = +0
    if (logf_fast_tabp(x, r, tab)) return r;
    return (float)log((double)x);
}

// The entropy's (double)logf(p) / log(2.0) (K:766) for a float's log m:
// 1 / RN(ln 2) split as Rh (29 significant bits: m * Rh exact for a float m)
// + Rl, and fma(m, Rl, m * Rh) -- one rounding of m (Rh + Rl) -- equals the
// correctly rounded quotient for every float m, zeros, infinities and NaN
// included (tests/c/divcheck.c): two f64 ops, no selects (the Markstein form
// took a multiply, two fmas and an infinity select)
constexpr double kLn2RecHi = 0x1.7154765p+0, kLn2RecLo = 0x1.5c17f278eff00p-31;
__device__ __forceinline__ double div_ln2(float m) {
    const double md = (double)m;
    return __builtin_fma(md, kLn2RecLo, md * kLn2RecHi);
}

// The entropy terms t = (double)logf(p) / log(2.0) of N bins (K:766; 0 for
// p <= 0, whose bins the reference skips).  The N fast logarithms run without
// a branch -- independent f64 chains the scheduler interleaves -- and the rare
// double-log fallbacks share one branch (a branch per bin around each log
// serialised the chains).  N = 4 (1024^3 x 8 entropy, one process, against
// the branch per bin: C0 2.78 -> 2.63 ms, C1 6.35 -> 5.88; N = 2 2.74 / 5.96,
// N = 8 3.00 / 5.87: registers; profiles/r06/logtab/r6w_*.log).
// A zero or negative p gives a bounded table index and its value is
// discarded by the select; NaN takes the fallback.
#ifndef VR_ENT_CHUNK
#define VR_ENT_CHUNK 4
#endif
constexpr int kEntChunk = VR_ENT_CHUNK;
template <int N>
__device__ __forceinline__ void ent_terms(const float (&p)[N], const LogEnt *tab, double (&t)[N]) {
    float l[N];
#ifdef VR_ABLATE_LOG  // timing ablation builds only (tools/build_variants.sh): NOT exact
#pragma unroll
    for (int k = 0; k < N; k++) l[k] = __logf(p[k]);
#else
    bool all = true, f[N];
#pragma unroll
    for (int k = 0; k < N; k++) {
        f[k] = logf_fast_tabp(p[k], l[k], tab);
        all = all && f[k];
    }
    if (!all) {
#pragma unroll
        for (int k = 0; k < N; k++)
            if (!f[k] && !(p[k] <= 0)) l[k] = (float)log((double)p[k]);
    }
#endif
#pragma unroll
    for (int k = 0; k < N; k++) t[k] = p[k] <= 0 ? 0.0 : div_ln2(l[k]);
}

// K:761-769 with the log table at `tab` (an LDS copy)
template <int B>
__device__ __forceinline__ float entropy_p(const float (&p)[B], float enorm, const LogEnt *tab) {
    constexpr int N = B < kEntChunk ? B : kEntChunk;
    float ent = 0.0f;
#pragma unroll
    for (int i = 0; i < B; i += N) {
        float q[N];
        double t[N];
#pragma unroll
        for (int k = 0; k < N; k++) q[k] = p[i + k];
        ent_terms<N>(q, tab, t);
#pragma unroll
        for (int k = 0; k < N; k++) ent = (float)((double)ent + (double)q[k] * t[k]);
    }
    ent = -ent;
    return ent / enorm;
}

// K:761-769
template <int B, bool TAB = false>
__device__ __forceinline__ float entropy(const float (&p)[B], float enorm) {
    float ent = 0.0f;
#pragma unroll
    for (int i = 0; i < B; i++) {
        const float pr = p[i];
        const double t = pr <= 0 ? 0.0 : div_ln2(logf_canon<TAB>(pr));
        ent = (float)((double)ent + (double)pr * t);
    }
    ent = -ent;
    return ent / enorm;
}

// the statistic a method samples, K:758-769 (M: 1 mean, 2 variance, 3 entropy;
// 0 / -1: the record is a statistic already baked by basicDataProcessing, B = 1,
// gathered with 32-bit / 64-bit addressing, vr_march.h gather8)
template <int B, int M>
__device__ __forceinline__ float record_stat(const float (&p)[B], float enorm) {
    if constexpr (M <= 0) {
        static_assert(B == 1, "baked statistics are one float per voxel");
        return p[0];
    } else if constexpr (M == 1) {
        return div_to_float(raw_mean<B>(p), kMeanR);
    } else if constexpr (M == 2) {
        const float mean = raw_mean<B>(p);
        return div_var_f32(raw_variance<B>(p, mean));
    } else {
        return entropy<B>(p, enorm);
    }
}

// record_stat with the entropy's log table in LDS (tab: copy_logtab)
template <int B, int M>
__device__ __forceinline__ float record_stat_p(const float (&p)[B], float enorm, const LogEnt *tab) {
    if constexpr (M == 3) return entropy_p<B>(p, enorm, tab);
    else return record_stat<B, M>(p, enorm);
}

// ---- fractal/template codec, methods 4/5/6 (K:195-222, 775-871) ----
// Decode of one codec voxel: template row, flipped and circularly shifted
// (fractalDecoding, K:195-222), NE sparse errors added with a clamp at 0
// (K:805-823; bin ids outside [0, B) skipped), renormalised (K:826-835).
constexpr int kCodecPre = 4;  // error pairs per voxel gathered with the codebook entry

// tpl: the template table (global or an LDS copy); pre: the voxel's first
// kCodecPre error pairs (gathered unconditionally when err_slots allows);
// further pairs are read from e.
template <int B>
__device__ __forceinline__ void codec_decode_pre(const float *tpl, const int4 c,
                                                 const float2 (&pre)[kCodecPre],
                                                 const float2 *e, float (&dec)[B]) {
    const float *row = tpl + (uint32_t)c.x * B;
#pragma unroll
    for (int m = 0; m < B; m++) {
        int i = m - c.y;                    // dec[(i + shift) mod B] = src[i]
        if (i < 0) i += B;
        dec[m] = row[c.z ? B - 1 - i : i];
    }
    for (int j = 0; j < c.w; j++) {
        float2 ev;
        if (j < kCodecPre) {
            ev = pre[0];
#pragma unroll
            for (int k = 1; k < kCodecPre; k++)
                if (j == k) ev = pre[k];
        } else {
            ev = e[j];
        }
        const int idx = (int)ev.x;
#pragma unroll
        for (int m = 0; m < B; m++) {
            if (m == idx) {
                float v = dec[m] + ev.y;
                if (v < 0) v = 0;
                dec[m] = v;
            }
        }
    }
    float total = 0.0f;
#pragma unroll
    for (int i = 0; i < B; i++) total = total + dec[i];
    if (total > 0) {
#pragma unroll
        for (int i = 0; i < B; i++) dec[i] = dec[i] / total;
    }
}

template <int B>
__device__ __forceinline__ void codec_decode(const Params &P, uint64_t vidx, float (&dec)[B]) {
    const float2 *e = P.err + vidx * (uint64_t)P.err_slots;
    float2 pre[kCodecPre];
#pragma unroll
    for (int k = 0; k < kCodecPre; k++) pre[k] = k < P.err_slots ? e[k] : make_float2(0.f, 0.f);
    codec_decode_pre<B>(P.tpl, P.cb[vidx], pre, e, dec);
}

// statistic C (0 mean, 1 variance, 2 entropy) of a codec voxel, K:837-868: the
// bin centre is used in both mean and variance
template <int B, int C>
__device__ __forceinline__ float codec_stat_of(const float (&dec)[B], float enorm) {
    if constexpr (C == 0) {  // K:857, the same (float)((double)mean / 0.0217) as K:758
        return div_to_float(raw_mean<B>(dec), kMeanR);
    } else if constexpr (C == 1) {
        const float mean = raw_mean<B>(dec);
        const float bw = bin_width(B);
        const double half = (double)bw / 2.0;
        float var = 0.0f;
#pragma unroll
        for (int i = 0; i < B; i++) {
            const double d = ((double)(bw * (float)i) + half) - (double)mean;
            var = (float)((double)var + (double)dec[i] * d * d);
        }
        return div_var_f32(var);
    } else {
        return entropy<B, true>(dec, enorm);  // table log: faster for the codec march
    }
}

template <int B, int C>
__device__ __forceinline__ float codec_stat(const Params &P, uint64_t vidx) {
    float dec[B];
    codec_decode<B>(P, vidx, dec);
    return codec_stat_of<B, C>(dec, P.enorm);
}

// ---- runtime-B variants (bin counts without a compiled specialisation) ----
__device__ __forceinline__ float raw_mean_rt(const float *__restrict__ p, int nb) {
    const float bw = bin_width(nb);
    const double half = (double)bw / 2.0;
    float mean = 0.0f;
    for (int i = 0; i < nb; i++) {
        const double c = (double)(bw * (float)i) + half;
        mean = (float)((double)mean + (double)p[i] * c);
    }
    return mean;
}

template <int M>
__device__ __forceinline__ float record_stat_rt(const float *__restrict__ p, int nb,
                                                float enorm) {
    if constexpr (M == 1) {
        return (float)div_const((double)raw_mean_rt(p, nb), kMeanD, kMeanR);
    } else if constexpr (M == 2) {
        const float mean = raw_mean_rt(p, nb);
        const float maxh = (float)0.0217;
        float var = 0.0f;
        for (int i = 0; i < nb; i++) {
            const float d = ((float)i / (float)nb) * maxh - mean;
            var = var + p[i] * d * d;
        }
        return div_var_f32(var);
    } else {
        float ent = 0.0f;
        for (int i = 0; i < nb; i++) {
            const float pr = p[i];
            const double t =
                pr <= 0 ? 0.0 : div_ln2(logf_canon(pr));
            ent = (float)((double)ent + (double)pr * t);
        }
        ent = -ent;
        return ent / enorm;
    }
}

// load one B-float record (vectorised)
template <int B>
__device__ __forceinline__ void load_rec(const float *__restrict__ vol, uint64_t vidx,
                                         float (&r)[B]) {
    const float *src = vol + vidx * (uint64_t)B;
    if constexpr (B % 4 == 0) {
#pragma unroll
        for (int i = 0; i < B / 4; i++) {
#ifdef VR_NT_LOADS  // A/B builds only: non-temporal record loads
            typedef float f4v __attribute__((ext_vector_type(4)));
            const f4v qv = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(src + 4 * i));
            const float4 q = make_float4(qv.x, qv.y, qv.z, qv.w);
#else
            const float4 q = *reinterpret_cast<const float4 *>(src + 4 * i);
#endif
            r[4 * i + 0] = q.x; r[4 * i + 1] = q.y; r[4 * i + 2] = q.z; r[4 * i + 3] = q.w;
        }
    } else if constexpr (B == 2) {
        const float2 q = *reinterpret_cast<const float2 *>(src);
        r[0] = q.x; r[1] = q.y;
    } else {
#pragma unroll
        for (int i = 0; i < B; i++) r[i] = src[i];
    }
}

}  // namespace vr
