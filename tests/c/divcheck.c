/*
 * divcheck.c -- exhaustive proof that the march's fast division by a constant
 * is bit-identical to the reference's double division.
 *
 * The reference divides float statistics by double constants and rounds the
 * quotient to float:  (float)((double)m / 0.0217)      (K:758)
 *                     (float)((double)v / 0.000021)    (K:759)
 *                     (double)logf(p) / log(2.0)       (K:766, kept in double)
 * The kernel computes q0 = m*R, e = fma(-q0, D, m), q = fma(e, R, q0) with
 * R = 1/D rounded to nearest (Markstein's correction step), returning q0 itself
 * when it is +-0 or +-inf.  This program
 * checks every one of the 2^32 float inputs for each divisor and prints the
 * number of mismatches (0 expected) -- and the same for the float-only
 * variance division div_var_f32 and the multiply-only div_to_float below -- comparing the float result for the first
 * two and the full double result for the third.
 *
 *   gcc -O2 -fopenmp -ffp-contract=off divcheck.c -lm && ./a.out
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static inline float bits_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline uint64_t d_bits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

static inline double fast_div(double m, double D, double R) {
    const double q0 = m * R;
    if (q0 == 0.0 || isinf(q0)) return q0;  /* +-0, +-inf: keep the sign / infinity */
    const double e = fma(-q0, D, m);
    return fma(e, R, q0);
}

/* float-only division by 0.000021 (vr_device.h div_var_f32): one FMA against
 * the reciprocal split in two floats, for |m| in [2^-100, FLT_MAX]; zeros and
 * infinities return m * Ch; NaN propagates; the remaining tiny inputs (whose
 * quotients are subnormal) take the double path */
static inline float div_var_f32(float m) {
    const double R = 1.0 / 0.000021;
    const float Ch = (float)R, Cl = (float)(R - (double)Ch);
    const float am = fabsf(m);
    if (am >= 0x1p-100f && am <= 0x1.fffffep127f) return fmaf(m, Ch, m * Cl);
    if (m == 0.0f || !(am <= 0x1.fffffep127f)) return m * Ch;
    return (float)fast_div((double)m, 0.000021, R);
}

int main(void) {
    const double Ds[3] = {0.0217, 0.000021, 0x1.62e42fefa39efp-1};
    const char *names[3] = {"0.0217 (mean, K:758)", "0.000021 (variance, K:759)",
                            "log(2.0) (entropy, K:766)"};
    long long total_bad = 0;
    for (int k = 0; k < 3; k++) {
        const double D = Ds[k], R = 1.0 / D;
        long long bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
        for (int64_t i = 0; i <= 0xFFFFFFFFll; i++) {
            const float m = bits_f((uint32_t)i);
            const double ref = (double)m / D, got = fast_div((double)m, D, R);
            if (k < 2) {
                const float a = (float)ref, b = (float)got;
                if (f_bits(a) != f_bits(b) && !(isnan(a) && isnan(b))) bad++;
            } else {
                if (d_bits(ref) != d_bits(got) && !(isnan(ref) && isnan(got))) bad++;
            }
        }
        printf("%-28s mismatches: %lld\n", names[k], bad);
        total_bad += bad;
    }
    {
        long long bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
        for (int64_t i = 0; i <= 0xFFFFFFFFll; i++) {
            const float m = bits_f((uint32_t)i);
            const float a = (float)((double)m / 0.000021), b = div_var_f32(m);
            if (f_bits(a) != f_bits(b) && !(isnan(a) && isnan(b))) bad++;
        }
        printf("%-28s mismatches: %lld\n", "0.000021 float-only (var)", bad);
        total_bad += bad;
    }
    /* rounded to float, the reciprocal multiply alone suffices (vr_device.h
     * div_to_float): (float)((double)m * (1/D)) == (float)((double)m / D) */
    for (int k = 0; k < 2; k++) {
        const double D = Ds[k], R = 1.0 / D;
        long long bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
        for (int64_t i = 0; i <= 0xFFFFFFFFll; i++) {
            const float m = bits_f((uint32_t)i);
            const float a = (float)((double)m / D), b = (float)((double)m * R);
            if (f_bits(a) != f_bits(b) && !(isnan(a) && isnan(b))) bad++;
        }
        printf("%-28s mismatches: %lld\n", k ? "0.000021 multiply-only" : "0.0217 multiply-only", bad);
        total_bad += bad;
    }
    /* the entropy's division by ln 2 (vr_device.h div_ln2): the reciprocal of
     * RN(ln 2) split as Rh (29 significant bits, so m * Rh is exact for a
     * float m) + Rl; fma(m, Rl, m * Rh) rounds m (Rh + Rl) once, and equals
     * the correctly rounded m / RN(ln 2) -- double result compared -- for every
     * float, zeros, infinities and NaN included (no selects) */
    {
        const double D = Ds[2], Rh = 0x1.7154765p+0, Rl = 0x1.5c17f278eff00p-31;
        long long bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
        for (int64_t i = 0; i <= 0xFFFFFFFFll; i++) {
            const double m = (double)bits_f((uint32_t)i);
            const double ref = m / D, got = fma(m, Rl, m * Rh);
            if (d_bits(ref) != d_bits(got) && !(isnan(ref) && isnan(got))) bad++;
        }
        printf("%-28s mismatches: %lld\n", "log(2.0) split reciprocal", bad);
        total_bad += bad;
    }
    return total_bad != 0;
}
