// replay_loads.hip -- memory-only replay of the march's gather patterns (tooling).
// Rays march like the production kernels (1024^3 x 8 bins, no early
// termination, trivial "decode") for cameras C0 (runSingleTest) and C1
// (display() at rotation 30,45).  Gather patterns:
//   0 per-ray   : lane = ray, 16 dwordx4 per step (8 corners x 2 halves)
//   1 quad      : quad lanes load 2 full records of one ray (k_march_quad)
//   2 quad-contig: each 4-lane group reads one ray's x0/x1 pair (64 contiguous
//                  bytes) per (y,z) combo; records complete after a 4x4 DPP
//                  transpose (not performed here: memory side only)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "../include/vr.h"
#include "vr_device.h"

using namespace vr;

__device__ __forceinline__ bool ray_of(const Params &P, uint32_t x, uint32_t y, float &px,
                                       float &py, float &pz, float &dx, float &dy, float &dz,
                                       int &nsteps) {
    const float *M = P.m;
    const float u = ((float)x / (float)P.W) * 2.0f - 1.0f;
    const float v = ((float)y / (float)P.H) * 2.0f - 1.0f;
    const float inv = 1.0f / sqrtf(u * u + v * v + 4.0f);
    const float ax = u * inv, ay = v * inv, az = -2.0f * inv;
    dx = ax * M[0] + ay * M[1] + az * M[2];
    dy = ax * M[4] + ay * M[5] + az * M[6];
    dz = ax * M[8] + ay * M[9] + az * M[10];
    const float ox = M[3], oy = M[7], oz = M[11];
    const float ix = 1.0f / dx, iy = 1.0f / dy, iz = 1.0f / dz;
    const float bx = ix * (-1.0f - ox), by = iy * (-1.0f - oy), bz = iz * (-1.0f - oz);
    const float tx = ix * (1.0f - ox), ty = iy * (1.0f - oy), tz = iz * (1.0f - oz);
    float tn = fmaxf(fmaxf(fminf(tx, bx), fminf(ty, by)), fmaxf(fminf(tx, bx), fminf(tz, bz)));
    const float tf = fminf(fminf(fmaxf(tx, bx), fmaxf(ty, by)), fminf(fmaxf(tx, bx), fmaxf(tz, bz)));
    if (!(tf > tn)) return false;
    if (tn < 0.0f) tn = 0.0f;
    px = ox + dx * tn; py = oy + dy * tn; pz = oz + dz * tn;
    nsteps = min(kMaxSteps, (int)((tf - tn) / kTStep));
    return true;
}

template <int PAT>
__global__ __launch_bounds__(256) void k_replay(const float *__restrict__ vol, Params P) {
    const uint32_t tile = blockIdx.x;
    const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63;
    uint32_t lx, ly, TW = 16, TH = 16;
    if (PAT == 0) { lx = ((wave & 1u) << 3) | (lane & 7u); ly = ((wave >> 1) << 3) | (lane >> 3); }
    else if (PAT == 3) { lx = lane; ly = wave; TW = 64; TH = 4; }
    else if (PAT == 4) { lx = lane & 31u; ly = wave * 2 + (lane >> 5); TW = 32; TH = 8; }
    else if (PAT == 5) { lx = lane & 15u; ly = wave * 4 + (lane >> 4); }
    else if (PAT == 7) { lx = lane; ly = wave; TW = 64; TH = 4; }
    else if (PAT == 6) { lx = lane & 31u; ly = wave * 2 + (lane >> 5); TW = 32; TH = 8; }
    else { lx = lane >> 2; ly = wave * 4 + (lane & 3); }
    const uint32_t ntx = (P.W + TW - 1) / TW;
    const uint32_t x = (tile % ntx) * TW + lx, y = (tile / ntx) * TH + ly;
    float px = 0, py = 0, pz = 0, dx = 0, dy = 0, dz = 0;
    int nsteps = 0;
    const bool hit = x < P.W && y < P.H && ray_of(P, x, y, px, py, pz, dx, dy, dz, nsteps);
    if ((PAT == 0 || (PAT >= 3 && PAT != 7)) && !hit) return;
    float acc = 0.0f;
    int i = 0;
    while (true) {
        const bool alive = hit && i < nsteps;
        if (PAT == 0 || (PAT >= 3 && PAT != 7)) { if (!alive) break; }
        else if (PAT == 7) { if (__ballot(alive) == 0) break; }
        else if (__ballot(alive) == 0) break;
        int x0, x1, y0, y1, z0, z1;
        float a;
        const float qx = px + dx * kTStep * i, qy = py + dy * kTStep * i, qz = pz + dz * kTStep * i;
        lin_axis(qx * 0.5f + 0.5f, P.nx, x0, x1, a);
        lin_axis(qy * 0.5f + 0.5f, P.ny, y0, y1, a);
        lin_axis(qz * 0.5f + 0.5f, P.nz, z0, z1, a);
        float4 r[16];
        if constexpr (PAT == 7) {
            // x0 record per combo for every lane; x1 only where the right neighbour's
            // x0 is not this lane's x1 (here: lane 63 and every 14th lane)
            const bool fix = lane == 63 || (lane % 14) == 13;
            const uint64_t rows[4] = {z0 * P.sz + y0 * P.sy, z0 * P.sz + y1 * P.sy,
                                      z1 * P.sz + y0 * P.sy, z1 * P.sz + y1 * P.sy};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float4 *p0 = reinterpret_cast<const float4 *>(vol + (rows[j] + x0) * 8);
                r[4 * j + 0] = p0[0]; r[4 * j + 1] = p0[1];
                r[4 * j + 2] = make_float4(0, 0, 0, 0); r[4 * j + 3] = r[4 * j + 2];
                if (fix && alive) {
                    const float4 *p1 = reinterpret_cast<const float4 *>(vol + (rows[j] + x1) * 8);
                    r[4 * j + 2] = p1[0]; r[4 * j + 3] = p1[1];
                }
            }
        } else if constexpr (PAT == 0 || PAT >= 3) {
            const uint64_t rows[4] = {z0 * P.sz + y0 * P.sy, z0 * P.sz + y1 * P.sy,
                                      z1 * P.sz + y0 * P.sy, z1 * P.sz + y1 * P.sy};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float4 *p0 = reinterpret_cast<const float4 *>(vol + (rows[j] + x0) * 8);
                const float4 *p1 = reinterpret_cast<const float4 *>(vol + (rows[j] + x1) * 8);
                r[4 * j + 0] = p0[0]; r[4 * j + 1] = p0[1];
                r[4 * j + 2] = p1[0]; r[4 * j + 3] = p1[1];
            }
        } else {
            const int g = lane & 3;
            const int pk0 = x0 | (y0 << 16), pk1 = z0 | ((x1 - x0) << 16) | ((y1 - y0) << 17) | ((z1 - z0) << 18) | ((alive ? 1 : 0) << 19);
#pragma unroll
            for (int G = 0; G < 4; G++) {
                int w0, w1;
                switch (G) {
                case 0: w0 = __builtin_amdgcn_mov_dpp(pk0, 0x00, 0xF, 0xF, false); w1 = __builtin_amdgcn_mov_dpp(pk1, 0x00, 0xF, 0xF, false); break;
                case 1: w0 = __builtin_amdgcn_mov_dpp(pk0, 0x55, 0xF, 0xF, false); w1 = __builtin_amdgcn_mov_dpp(pk1, 0x55, 0xF, 0xF, false); break;
                case 2: w0 = __builtin_amdgcn_mov_dpp(pk0, 0xAA, 0xF, 0xF, false); w1 = __builtin_amdgcn_mov_dpp(pk1, 0xAA, 0xF, 0xF, false); break;
                default: w0 = __builtin_amdgcn_mov_dpp(pk0, 0xFF, 0xF, 0xF, false); w1 = __builtin_amdgcn_mov_dpp(pk1, 0xFF, 0xF, 0xF, false); break;
                }
                if (!((w1 >> 19) & 1)) { r[4 * G] = r[4 * G + 1] = r[4 * G + 2] = r[4 * G + 3] = make_float4(0, 0, 0, 0); continue; }
                const uint32_t gx0 = w0 & 0xFFFF, gy0 = (uint32_t)w0 >> 16, gz0 = w1 & 0xFFFF;
                const uint32_t ddx = (w1 >> 16) & 1, ddy = (w1 >> 17) & 1, ddz = (w1 >> 18) & 1;
                if constexpr (PAT == 1) {
                    const uint32_t xx = gx0 + ((g & 1) ? ddx : 0), yy = gy0 + ((g >> 1) ? ddy : 0);
                    const uint64_t row = (uint64_t)yy * P.sy + xx;
                    const float4 *p0 = reinterpret_cast<const float4 *>(vol + ((uint64_t)gz0 * P.sz + row) * 8);
                    const float4 *p1 = reinterpret_cast<const float4 *>(vol + ((uint64_t)(gz0 + ddz) * P.sz + row) * 8);
                    r[4 * G + 0] = p0[0]; r[4 * G + 1] = p0[1]; r[4 * G + 2] = p1[0]; r[4 * G + 3] = p1[1];
                } else {
                    // 4 combos (y,z); lane g reads chunk g of the 64-B x-pair (x1 = x0+1 assumed)
#pragma unroll
                    for (int c = 0; c < 4; c++) {
                        const uint64_t rec = (uint64_t)(gz0 + ((c >> 1) ? ddz : 0)) * P.sz +
                                             (uint64_t)(gy0 + ((c & 1) ? ddy : 0)) * P.sy + gx0;
                        r[4 * G + c] = reinterpret_cast<const float4 *>(vol + rec * 8)[g];
                    }
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 16; k++) acc += r[k].x + r[k].w;
        i++;
    }
    if (x < P.W && y < P.H) P.out[(uint64_t)y * P.W + x] = __float_as_uint(acc);
}

int main() {
    const int n = 1024, W = 1920, H = 1080;
    vr_extent dims = {(size_t)n, (size_t)n, (size_t)n};
    if (vr_synthesize(dims, 8, 20261015ull) != 0) return 1;
    const float *vol;
    int nb;
    vr_volume_info(&dims, &nb, &vol);
    size_t sy, sz;
    vr_volume_layout(&sy, &sz);
    uint32_t *out;
    hipMalloc(&out, (size_t)W * H * 4);
    Params P;
    memset(&P, 0, sizeof P);
    P.W = W; P.H = H; P.nx = P.ny = P.nz = n; P.sy = sy; P.sz = sz;
    P.tiles_x = (W + 15) / 16;
    P.out = out;
    const uint32_t ntiles = P.tiles_x * ((H + 15) / 16);
    // C0 and C1 (display(): glRotatef(-30,x) glRotatef(-45,y) glTranslatef(0,0,4))
    const float c0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 4};
    const float c1[12] = {0.70710677f, 0.0f, -0.70710677f, -2.828427f, 0.35355338f, 0.8660254f,
                          0.35355338f, 1.4142135f, 0.61237246f, -0.5f, 0.61237246f, 2.4494898f};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"per-ray", "quad", "quad-contig", "per-ray 64x1", "per-ray 32x2", "per-ray 16x4", "32x2 pipelined", "x0 + neighbour x1"};
    for (int cam = 0; cam < 2; cam++) {
        memcpy(P.m, cam ? c1 : c0, sizeof c0);
        for (int pat = 0; pat < 8; pat++) {
            if (pat == 6) continue;
            float best = 1e30f;
            for (int rep = 0; rep < 3; rep++) {
                auto go = [&]() {
                    if (pat == 0) hipLaunchKernelGGL(k_replay<0>, dim3(ntiles), dim3(256), 0, 0, vol, P);
                    if (pat == 1) hipLaunchKernelGGL(k_replay<1>, dim3(ntiles), dim3(256), 0, 0, vol, P);
                    if (pat == 2) hipLaunchKernelGGL(k_replay<2>, dim3(ntiles), dim3(256), 0, 0, vol, P);
                    if (pat == 3) hipLaunchKernelGGL(k_replay<3>, dim3(30 * 270), dim3(256), 0, 0, vol, P);
                    if (pat == 4) hipLaunchKernelGGL(k_replay<4>, dim3(60 * 135), dim3(256), 0, 0, vol, P);
                    if (pat == 5) hipLaunchKernelGGL(k_replay<5>, dim3(ntiles), dim3(256), 0, 0, vol, P);
                    if (pat == 7) hipLaunchKernelGGL(k_replay<7>, dim3(30 * 270), dim3(256), 0, 0, vol, P);
                };
                go();
                hipEventRecord(e0);
                go();
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            printf("C%d %-12s %.3f ms (no ET, loads only)\n", cam, names[pat], best);
        }
    }
    return 0;
}
