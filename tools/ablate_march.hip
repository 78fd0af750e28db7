// ablate_march.hip -- timing-only ablations of the march (not product code).
//
// Variants of the B=8 / method-1 march, all WITHOUT early termination (every
// hit ray marches to tfar, so every variant does the same number of samples):
//   0  production decode (f64 terms), real gathers
//   1  f32-only decode, real gathers
//   2  production decode, gathers from a 64 KiB L1-resident window
//   3  real gathers, trivial decode (sum of the record floats)
//   4  no gathers (synthetic record values), production decode
// Output values are written so nothing is dead-code eliminated.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I<csrc> ablate_march.hip -L... -lvr
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/vr.h"
#include "vr_device.h"

using namespace vr;

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

template <int V>
__device__ __forceinline__ float decode(const float (&p)[8], float enorm) {
    if constexpr (V == 1) {
        const float bw = bin_width(8);
        float m = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; i++) m = m + p[i] * (bw * (float)i + bw * 0.5f);
        return m * (1.0f / 0.0217f);
    } else if constexpr (V == 3) {
        return ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
    } else {
        return record_stat<8, 1>(p, enorm);
    }
}

template <int V>
__global__ __launch_bounds__(256) void k_abl(const float *__restrict__ vol, Params P) {
    const uint32_t tile = blockIdx.x;
    const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const uint32_t lx = ((wave & 1u) << 3) | (lane & 7u), ly = ((wave >> 1) << 3) | (lane >> 3);
    const uint32_t x = (tile % P.tiles_x) * 16 + lx, y = (tile / P.tiles_x) * 16 + ly;
    if (x >= P.W || y >= P.H) return;
    const float *M = P.m;
    const float u = ((float)x / (float)P.W) * 2.0f - 1.0f;
    const float v = ((float)y / (float)P.H) * 2.0f - 1.0f;
    const float ox = M[3], oy = M[7], oz = M[11];
    const float inv = 1.0f / sqrtf(u * u + v * v + 4.0f);
    const float ax = u * inv, ay = v * inv, az = -2.0f * inv;
    const float dx = ax * M[0] + ay * M[1] + az * M[2];
    const float dy = ax * M[4] + ay * M[5] + az * M[6];
    const float dz = ax * M[8] + ay * M[9] + az * M[10];
    const float ix = 1.0f / dx, iy = 1.0f / dy, iz = 1.0f / dz;
    const float bx = ix * (-1.0f - ox), by = iy * (-1.0f - oy), bz = iz * (-1.0f - oz);
    const float tx = ix * (1.0f - ox), ty = iy * (1.0f - oy), tz = iz * (1.0f - oz);
    float tn = fmaxf(fmaxf(fminf(tx, bx), fminf(ty, by)), fmaxf(fminf(tx, bx), fminf(tz, bz)));
    const float tf = fminf(fminf(fmaxf(tx, bx), fmaxf(ty, by)), fminf(fmaxf(tx, bx), fmaxf(tz, bz)));
    if (!(tf > tn)) return;
    if (tn < 0.0f) tn = 0.0f;
    float px = ox + dx * tn, py = oy + dy * tn, pz = oz + dz * tn, tt = tn;
    float acc = 0.0f;
    for (int i = 0; i < kMaxSteps; i++) {
        int x0, x1, y0, y1, z0, z1;
        float wx, wy, wz;
        lin_axis(px * 0.5f + 0.5f, P.nx, x0, x1, wx);
        lin_axis(py * 0.5f + 0.5f, P.ny, y0, y1, wy);
        lin_axis(pz * 0.5f + 0.5f, P.nz, z0, z1, wz);
        const uint64_t nx = P.nx, ny = P.ny;
        uint64_t r00 = ((uint64_t)z0 * ny + y0) * nx, r10 = ((uint64_t)z0 * ny + y1) * nx;
        uint64_t r01 = ((uint64_t)z1 * ny + y0) * nx, r11 = ((uint64_t)z1 * ny + y1) * nx;
        uint64_t vi[8] = {r00 + x0, r00 + x1, r10 + x0, r10 + x1, r01 + x0, r01 + x1, r11 + x0, r11 + x1};
        if (V == 2) {
#pragma unroll
            for (int j = 0; j < 8; j++) vi[j] &= 2047;  // 2048 records = 64 KiB
        }
        float s[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            float rec[8];
            if constexpr (V == 4) {
#pragma unroll
                for (int k = 0; k < 8; k++) rec[k] = (float)((vi[j] >> (k * 3)) & 7) * 0.125f;
            } else {
                load_rec<8>(vol, vi[j], rec);
            }
            s[j] = decode<V>(rec, P.enorm);
        }
        const float c0 = lerpq(lerpq(s[0], s[1], wx), lerpq(s[2], s[3], wx), wy);
        const float c1 = lerpq(lerpq(s[4], s[5], wx), lerpq(s[6], s[7], wx), wy);
        const float smp = lerpq(c0, c1, wz);
        const float4 col = transfer(smp);
        acc = acc + col.w * 0.05f + smp * 1e-9f;
        tt = tt + kTStep;
        if (tt > tf) break;
        px = px + dx * kTStep;
        py = py + dy * kTStep;
        pz = pz + dz * kTStep;
    }
    P.out[(uint64_t)y * P.W + x] = __float_as_uint(acc);
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 1024;
    const int W = 1920, H = 1080, reps = 5;
    vr_extent dims = {(size_t)n, (size_t)n, (size_t)n};
    if (vr_synthesize(dims, 8, 20261015ull) != 0) {
        fprintf(stderr, "synth: %s\n", vr_last_error());
        return 1;
    }
    const float *vol;
    int nb;
    vr_volume_info(&dims, &nb, &vol);
    uint32_t *out;
    CK(hipMalloc(&out, (size_t)W * H * 4));
    Params P;
    memset(&P, 0, sizeof P);
    const float m[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 4};
    memcpy(P.m, m, sizeof m);
    P.W = W; P.H = H; P.nx = P.ny = P.nz = n; P.nb = 8; P.enorm = 3.0f;
    P.tiles_x = (W + 15) / 16;
    P.out = out;
    const uint32_t ntiles = P.tiles_x * ((H + 15) / 16);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](int v) {
        switch (v) {
        case 0: hipLaunchKernelGGL(k_abl<0>, dim3(ntiles), dim3(256), 0, 0, vol, P); break;
        case 1: hipLaunchKernelGGL(k_abl<1>, dim3(ntiles), dim3(256), 0, 0, vol, P); break;
        case 2: hipLaunchKernelGGL(k_abl<2>, dim3(ntiles), dim3(256), 0, 0, vol, P); break;
        case 3: hipLaunchKernelGGL(k_abl<3>, dim3(ntiles), dim3(256), 0, 0, vol, P); break;
        case 4: hipLaunchKernelGGL(k_abl<4>, dim3(ntiles), dim3(256), 0, 0, vol, P); break;
        }
    };
    const char *names[] = {"f64 decode + gathers", "f32 decode + gathers",
                           "f64 decode, L1-resident gathers", "trivial decode + gathers",
                           "f64 decode, no gathers"};
    std::vector<float> best(5, 1e30f);
    for (int round = 0; round < reps; round++) {
        for (int v = 0; v < 5; v++) {
            run(v);
            CK(hipEventRecord(e0, 0));
            run(v);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best[v]) best[v] = ms;
        }
    }
    for (int v = 0; v < 5; v++) printf("variant %d  %-36s %8.3f ms\n", v, names[v], best[v]);
    return 0;
}
