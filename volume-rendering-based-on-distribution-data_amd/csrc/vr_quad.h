// vr_quad.h -- quad (4-lane) and DPP helpers shared by the march families
// (vr_kernels.hip: per-ray / box / quad marches; vr_m7.hip: method 7;
// vr_codec.hip: methods 4/5/6), and their register-budget knobs.
#pragma once

#include "vr_device.h"
#include "vr_march.h"

namespace vr {

// quad_perm DPP: lane g of each quad reads lane sel[g] of its quad
template <int CTRL>
__device__ __forceinline__ float qperm(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int qpermi(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
constexpr int kQ0 = 0x00, kQ1 = 0x55, kQ2 = 0xAA, kQ3 = 0xFF;  // broadcast lane 0/1/2/3
constexpr int kQx1 = 0xB1;   // [1,0,3,2]
constexpr int kQ0101 = 0x44; // [0,1,0,1]
constexpr int kQ2323 = 0xEE; // [2,3,2,3]

template <int G>
__device__ __forceinline__ int bcast_g(int v) {
    if constexpr (G == 0) return qpermi<kQ0>(v);
    else if constexpr (G == 1) return qpermi<kQ1>(v);
    else if constexpr (G == 2) return qpermi<kQ2>(v);
    else return qpermi<kQ3>(v);
}

template <int D>
__device__ __forceinline__ void quad_xchg(float4 &a, float4 &b, bool up) {
    // butterfly over bit D of (register, lane): the lower lane keeps a and
    // receives its partner's a into b; the upper lane keeps b, receives into a
    // (selects on values, never on references: a select of two array
    // addresses keeps the arrays out of registers)
    constexpr int X = D == 1 ? 0xB1 : 0x4E;  // quad_perm [1,0,3,2] / [2,3,0,1]
    const float a0 = a.x, a1 = a.y, a2 = a.z, a3 = a.w;
    const float b0 = b.x, b1 = b.y, b2 = b.z, b3 = b.w;
    const float u0 = qperm<X>(up ? a0 : b0), u1 = qperm<X>(up ? a1 : b1);
    const float u2 = qperm<X>(up ? a2 : b2), u3 = qperm<X>(up ? a3 : b3);
    a = make_float4(up ? u0 : a0, up ? u1 : a1, up ? u2 : a2, up ? u3 : a3);
    b = make_float4(up ? b0 : u0, up ? b1 : u1, up ? b2 : u2, up ? b3 : u3);
}
// M[R] in lane g = chunk g of ray R's record  ->  M[c] in lane g = chunk c of ray g's record
__device__ __forceinline__ void quad_transpose(float4 (&M)[4], uint32_t g) {
    quad_xchg<2>(M[0], M[2], (g & 2u) != 0);
    quad_xchg<2>(M[1], M[3], (g & 2u) != 0);
    quad_xchg<1>(M[0], M[1], (g & 1u) != 0);
    quad_xchg<1>(M[2], M[3], (g & 1u) != 0);
}

__device__ __forceinline__ void mark_foot(const Params &P, const Foot &f) {
    const uint64_t nx = (uint64_t)P.nx, ny = (uint64_t)P.ny;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint64_t z = (j & 4) ? f.z1 : f.z0, y = (j & 2) ? f.y1 : f.y0;
        const uint64_t x = (j & 1) ? f.x1 : f.x0;
        mark_voxel(P.mark, (z * ny + y) * nx + x);
    }
}

// footprint packed for the quad broadcast:
//   w0 = x0 | y0 << 16,  w1 = z0 | dx << 16 | dy << 17 | dz << 18 | live << 19,
//   w2 = filter weights in 9-bit fixed point (exact: q8 gives k/256, k <= 256)
struct FootPacked {
    int w0, w1, w2;
};

__device__ __forceinline__ FootPacked pack_foot(const Foot &f, bool live) {
    FootPacked p;
    p.w0 = f.x0 | (f.y0 << 16);
    p.w1 = f.z0 | ((f.x1 - f.x0) << 16) | ((f.y1 - f.y0) << 17) | ((f.z1 - f.z0) << 18) |
           ((live ? 1 : 0) << 19);
    p.w2 = (int)(f.ax * 256.0f) | ((int)(f.ay * 256.0f) << 9) | ((int)(f.az * 256.0f) << 18);
    return p;
}

// pair swap: from the chunks of combos (c, c') build lane g's full record of
// corner (x = g >> 1, combo = g & 1 ? c' : c)
__device__ __forceinline__ float swp(float i1, float i2, bool odd, bool hi) {
    const float recv = qperm<kQx1>(odd ? i1 : i2);
    return hi ? (odd ? i2 : recv) : (odd ? recv : i1);
}
__device__ __forceinline__ void pair_swap(const float4 &i1, const float4 &i2, bool odd,
                                          float (&rec)[8]) {
    rec[0] = swp(i1.x, i2.x, odd, false); rec[1] = swp(i1.y, i2.y, odd, false);
    rec[2] = swp(i1.z, i2.z, odd, false); rec[3] = swp(i1.w, i2.w, odd, false);
    rec[4] = swp(i1.x, i2.x, odd, true);  rec[5] = swp(i1.y, i2.y, odd, true);
    rec[6] = swp(i1.z, i2.z, odd, true);  rec[7] = swp(i1.w, i2.w, odd, true);
}

// in-quad trilinear blend of ray (G, q): lane g holds corner (x = g>>1, y = g&1)
// at z0 (s0) and z1 (s1).  Same lerp order as blend8 (x, then y, then z).
template <int G>
__device__ __forceinline__ float qc_blend(const FootPacked &fp, float s0, float s1) {
    const int w2 = bcast_g<G>(fp.w2);
    const float ax = (float)(w2 & 0x1FF) * (1.0f / 256.0f);
    const float ay = (float)((w2 >> 9) & 0x1FF) * (1.0f / 256.0f);
    const float az = (float)((w2 >> 18) & 0x1FF) * (1.0f / 256.0f);
    // x: lane g gets c(y = g&1, z) = lerp(s(x0,y), s(x1,y), ax)
    const float cz0 = lerpq(qperm<kQ0101>(s0), qperm<kQ2323>(s0), ax);
    const float cz1 = lerpq(qperm<kQ0101>(s1), qperm<kQ2323>(s1), ax);
    // y: c(z) = lerp(c(y0,z), c(y1,z), ay), identical in all four lanes
    const float c0 = lerpq(qperm<kQ0>(cz0), qperm<kQ1>(cz0), ay);
    const float c1 = lerpq(qperm<kQ0>(cz1), qperm<kQ1>(cz1), ay);
    return lerpq(c0, c1, az);
}

#ifndef VR_WIDE_WAVES
#define VR_WIDE_WAVES 2
#endif
#ifndef VR_WIDE_MINW
#define VR_WIDE_MINW 1      // waves per SIMD the register allocation must allow
#endif
constexpr bool WQ3 = true;  // entropy through the quad-cooperative wide march
#ifndef M7_WQ_MAP
#define M7_WQ_MAP 1         // k_march_m7wq pixel map default (P.wq_map)
#endif
#ifndef VR_QUAD_WAVES
#define VR_QUAD_WAVES 1  // minimum waves per SIMD the register allocation must allow
#endif
}  // namespace vr
