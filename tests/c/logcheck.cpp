// logcheck.cpp -- host restatement of the device's exact float logarithm
// (vr_device.h logf_fast_tabp, table vr_logtab.h from tools/gen_logtab.py),
// checked against (float)log((double)x) for every positive finite float.
// Prints the mismatches of the fast form where it claims exactness (0
// expected) and the inputs it leaves to the double log.  The device function
// itself is checked the same way on the GPU (vr_selftest_logf,
// tests/test_gpu_parity.py); this pins the algorithm and the generated table
// on the CPU.
//
//   g++ -O2 -fopenmp -ffp-contract=off -I<csrc> logcheck.cpp && ./a.out
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

#define __constant__
#include "vr_logtab.h"

static inline uint32_t f_bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
static inline float bits_f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
static inline uint64_t d_bits(double d) { uint64_t u; std::memcpy(&u, &d, 8); return u; }

static bool fast_log(float x, float &r) {
    const float kRound = 49152.0f;
    int e;
    float m = std::frexp(x, &e);
    if (m < 0.75f) {
        m = m * 2.0f;
        e -= 1;
    }
    const float s = m + kRound;
    const float c = s - kRound;
    const float d = m - c;
    uint32_t i = f_bits(s) - (f_bits(kRound) + 192u);
    if (i > 192u) i = 192u;
    const vr::LogEnt t = vr::kLogTab[i];
    const double rr = (double)d * t.inv;
    double q = 1.0 / 5.0;
    q = std::fma(q, rr, -1.0 / 4.0);
    q = std::fma(q, rr, 1.0 / 3.0);
    q = std::fma(q, rr, -0.5);
    const double p = std::fma(rr * rr, q, rr);
    const double y = std::fma((double)e, vr::kLn2, t.hi) + p;
    r = (float)y;
    const uint32_t lo29 = (uint32_t)d_bits(y) & 0x1FFFFFFFu;
    return f_bits(x) < 0x7F800000u && lo29 - (0x10000000u - 512u) > 1024u;
}

int main() {
    long long bad = 0, slow = 0;
#pragma omp parallel for reduction(+ : bad, slow) schedule(static)
    for (int64_t b = 1; b < 0x7F800000ll; b++) {
        const float x = bits_f((uint32_t)b);
        float r;
        if (!fast_log(x, r)) {
            slow++;
            continue;
        }
        if (f_bits(r) != f_bits((float)std::log((double)x))) bad++;
    }
    std::printf("fast-form mismatches: %lld\nfallbacks: %lld\n", bad, slow);
    return bad != 0 || slow >= (1ll << 16);
}
