// vr_kernels.hip -- gfx950 kernels of the distribution-volume ray caster.
//
//  k_march<B, M, COUNT>  the d_render per-ray march (K:272-717) for methods
//                        1/2/3: one lane per ray, one 8x8 ray block per wave,
//                        one 16x16-pixel tile per 256-thread workgroup,
//                        XCD-aware tile order.  Per step the statistic is
//                        decoded from the 8 corner distribution records and
//                        blended with 8-bit filter weights.
//  k_march_m7<B>         method 7, software-interpolated corner means
//                        (K:320-367, 395-480), stateful along the ray.
//  k_synth               the synthetic distribution volume, written in HBM.
//  k_unscatter           rank-0 frame assembly of gathered tiles.
//  k_popcount            footprint bitset -> U.
//
// K = volumeRender_kernel.cu of the reference.
#include "vr_device.h"
#include "vr_internal.h"

namespace vr {

// Blocks are dealt round-robin over the 8 XCDs (blockIdx % 8 = XCD group).
// Give each group a contiguous run of tiles so neighbouring tiles, which share
// their apron of voxel records, meet in the same L2.  Bijective for any n.
__device__ __forceinline__ uint32_t xcd_slot(uint32_t bid, uint32_t n) {
    const uint32_t q = n >> 3, r = n & 7;
    const uint32_t g = bid & 7, i = bid >> 3;
    const uint32_t base = g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q;
    return base + i;
}

struct Ray {
    float ox, oy, oz, dx, dy, dz, tnear, tfar;
};

// eye ray + intersectBox, K:288-306
__device__ __forceinline__ bool make_ray(const Params &P, uint32_t x, uint32_t y, Ray &r) {
    const float *M = P.m;
    const float u = ((float)x / (float)P.W) * 2.0f - 1.0f;
    const float v = ((float)y / (float)P.H) * 2.0f - 1.0f;
    r.ox = 0.0f * M[0] + 0.0f * M[1] + 0.0f * M[2] + 1.0f * M[3];
    r.oy = 0.0f * M[4] + 0.0f * M[5] + 0.0f * M[6] + 1.0f * M[7];
    r.oz = 0.0f * M[8] + 0.0f * M[9] + 0.0f * M[10] + 1.0f * M[11];
    const float inv = 1.0f / sqrtf(u * u + v * v + (-2.0f) * (-2.0f));
    const float ax = u * inv, ay = v * inv, az = -2.0f * inv;
    r.dx = ax * M[0] + ay * M[1] + az * M[2];
    r.dy = ax * M[4] + ay * M[5] + az * M[6];
    r.dz = ax * M[8] + ay * M[9] + az * M[10];
    const float ix = 1.0f / r.dx, iy = 1.0f / r.dy, iz = 1.0f / r.dz;
    const float bx = ix * (-1.0f - r.ox), by = iy * (-1.0f - r.oy), bz = iz * (-1.0f - r.oz);
    const float tx = ix * (1.0f - r.ox), ty = iy * (1.0f - r.oy), tz = iz * (1.0f - r.oz);
    const float mnx = fminf(tx, bx), mny = fminf(ty, by), mnz = fminf(tz, bz);
    const float mxx = fmaxf(tx, bx), mxy = fmaxf(ty, by), mxz = fmaxf(tz, bz);
    r.tnear = fmaxf(fmaxf(mnx, mny), fmaxf(mnx, mnz));
    r.tfar = fminf(fminf(mxx, mxy), fminf(mxx, mxz));
    if (!(r.tfar > r.tnear)) return false;
    if (r.tnear < 0.0f) r.tnear = 0.0f;
    return true;
}

__device__ __forceinline__ void mark_voxel(unsigned long long *mark, uint64_t idx) {
    atomicOr(mark + (idx >> 6), 1ull << (idx & 63));
}

// tex3D(originalQueryTex, p) of the method's statistic, K:601/619/635
template <int B, int M, bool COUNT>
__device__ __forceinline__ float sample_tri(const float *__restrict__ vol, const Params &P,
                                            float px, float py, float pz) {
    int x0, x1, y0, y1, z0, z1;
    float ax, ay, az;
    lin_axis(px * 0.5f + 0.5f, P.nx, x0, x1, ax);
    lin_axis(py * 0.5f + 0.5f, P.ny, y0, y1, ay);
    lin_axis(pz * 0.5f + 0.5f, P.nz, z0, z1, az);
    const uint64_t nx = (uint64_t)P.nx, ny = (uint64_t)P.ny;
    const uint64_t r00 = ((uint64_t)z0 * ny + (uint64_t)y0) * nx;
    const uint64_t r10 = ((uint64_t)z0 * ny + (uint64_t)y1) * nx;
    const uint64_t r01 = ((uint64_t)z1 * ny + (uint64_t)y0) * nx;
    const uint64_t r11 = ((uint64_t)z1 * ny + (uint64_t)y1) * nx;
    const uint64_t vidx[8] = {r00 + x0, r00 + x1, r10 + x0, r10 + x1,
                              r01 + x0, r01 + x1, r11 + x0, r11 + x1};
    if constexpr (COUNT) {
#pragma unroll
        for (int j = 0; j < 8; j++) mark_voxel(P.mark, vidx[j]);
    }
    float s[8];
    if constexpr (B > 0) {
        // corners per load group: keep <= 64 record floats live
        constexpr int CG = (B >= 64) ? 1 : ((64 / B) > 8 ? 8 : (64 / B));
#pragma unroll
        for (int g = 0; g < 8; g += CG) {
            float rec[CG][B];
#pragma unroll
            for (int j = 0; j < CG; j++) load_rec<B>(vol, vidx[g + j], rec[j]);
#pragma unroll
            for (int j = 0; j < CG; j++) s[g + j] = record_stat<B, M>(rec[j], P.enorm);
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++)
            s[j] = record_stat_rt<M>(vol + vidx[j] * (uint64_t)P.nb, P.nb, P.enorm);
    }
    const float c00 = lerpq(s[0], s[1], ax);
    const float c10 = lerpq(s[2], s[3], ax);
    const float c01 = lerpq(s[4], s[5], ax);
    const float c11 = lerpq(s[6], s[7], ax);
    const float c0 = lerpq(c00, c10, ay);
    const float c1 = lerpq(c01, c11, ay);
    return lerpq(c0, c1, az);
}

// pixel of this thread inside its tile: wave w covers the 8x8 quadrant w
__device__ __forceinline__ void tile_pixel(uint32_t t, uint32_t &lx, uint32_t &ly) {
    const uint32_t wave = t >> 6, lane = t & 63;
    lx = ((wave & 1u) << 3) | (lane & 7u);
    ly = ((wave >> 1) << 3) | (lane >> 3);
}

__device__ __forceinline__ void write_pixel(const Params &P, uint64_t o, int n, float r,
                                            float g, float b, float a) {
    if (P.out_n) P.out_n[o] = n;
    if (n < 0) return;
    P.out[o] = pack_rgba(r, g, b, a);
    if (P.out_f) {
        reinterpret_cast<float4 *>(P.out_f)[o] = make_float4(sat(r), sat(g), sat(b), sat(a));
    }
}

// composite one classified sample, K:683-699; returns true on early exit
__device__ __forceinline__ bool composite(const Params &P, float sample, float &sx, float &sy,
                                          float &sz, float &sw) {
    float4 col = transfer((sample - P.toff) * P.tscale);
    col.w = col.w * P.density;
    col.x = col.x * col.w;
    col.y = col.y * col.w;
    col.z = col.z * col.w;
    const float om = 1.0f - sw;
    sx = sx + col.x * om;
    sy = sy + col.y * om;
    sz = sz + col.z * om;
    sw = sw + col.w * om;
    return sw > kOpacityThreshold;
}

template <int B, int M, bool COUNT>
__global__ __launch_bounds__(256) void k_march(const float *__restrict__ vol, Params P) {
    const uint32_t slot = xcd_slot(blockIdx.x, gridDim.x);
    const uint32_t tile = P.tile_list ? P.tile_list[slot] : slot;
    if (tile == kPad) return;
    uint32_t lx, ly;
    tile_pixel(threadIdx.x, lx, ly);
    const uint32_t x = (tile % P.tiles_x) * kTile + lx;
    const uint32_t y = (tile / P.tiles_x) * kTile + ly;
    if (x >= P.W || y >= P.H) return;
    const uint64_t o = P.tile_list ? (uint64_t)slot * 256u + ly * 16u + lx
                                   : (uint64_t)y * P.W + x;
    Ray r;
    if (!make_ray(P, x, y, r)) {
        if (P.out_n) P.out_n[o] = -1;
        return;
    }
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = r.tnear;
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
    int n = 0;
    for (int i = 0; i < kMaxSteps; i++) {
        const float sample = sample_tri<B, M, COUNT>(vol, P, px, py, pz);
        n = i + 1;
        if (composite(P, sample, sx, sy, sz, sw)) break;
        t = t + kTStep;
        if (t > r.tfar) break;
        px = px + stx;
        py = py + sty;
        pz = pz + stz;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
}

// ---- method 7: software trilinear of corner means, K:320-367, 395-480 ----
struct M7 {
    float fx, fy, fz, cx, cy, cz;  // interPos[0] and interPos[7]
    float mean[8];
};

template <int B>
__device__ __forceinline__ float corner_mean(const float *__restrict__ vol, const Params &P,
                                             float ux, float uy, float uz) {
    const int ix = point_axis(ux, P.nx), iy = point_axis(uy, P.ny), iz = point_axis(uz, P.nz);
    const uint64_t vidx = ((uint64_t)iz * (uint64_t)P.ny + (uint64_t)iy) * (uint64_t)P.nx + ix;
    if constexpr (B > 0) {
        float rec[B];
        load_rec<B>(vol, vidx, rec);
        return raw_mean<B>(rec);
    } else {
        return raw_mean_rt(vol + vidx * (uint64_t)P.nb, P.nb);
    }
}

template <int B>
__device__ void m7_refresh(const float *__restrict__ vol, const Params &P, float px, float py,
                           float pz, M7 &m) {
    const float qx = px * 0.5f + 0.5f, qy = py * 0.5f + 0.5f, qz = pz * 0.5f + 0.5f;
    m.fx = floorf(qx * (float)P.m7x) / (float)P.m7x;
    m.cx = ceilf(qx * (float)P.m7x) / (float)P.m7x;
    m.fy = floorf(qy * (float)P.m7y) / (float)P.m7y;
    m.cy = ceilf(qy * (float)P.m7y) / (float)P.m7y;
    m.fz = floorf(qz * (float)P.m7z) / (float)P.m7z;
    m.cz = ceilf(qz * (float)P.m7z) / (float)P.m7z;
#pragma unroll
    for (int j = 0; j < 8; j++)
        m.mean[j] = corner_mean<B>(vol, P, (j & 1) ? m.cx : m.fx, (j & 2) ? m.cy : m.fy,
                                   (j & 4) ? m.cz : m.fz);
}

template <int B>
__global__ __launch_bounds__(256) void k_march_m7(const float *__restrict__ vol, Params P) {
    const uint32_t slot = xcd_slot(blockIdx.x, gridDim.x);
    const uint32_t tile = P.tile_list ? P.tile_list[slot] : slot;
    if (tile == kPad) return;
    uint32_t lx, ly;
    tile_pixel(threadIdx.x, lx, ly);
    const uint32_t x = (tile % P.tiles_x) * kTile + lx;
    const uint32_t y = (tile / P.tiles_x) * kTile + ly;
    if (x >= P.W || y >= P.H) return;
    const uint64_t o = P.tile_list ? (uint64_t)slot * 256u + ly * 16u + lx
                                   : (uint64_t)y * P.W + x;
    Ray r;
    if (!make_ray(P, x, y, r)) {
        if (P.out_n) P.out_n[o] = -1;
        return;
    }
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = r.tnear;
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
    M7 m;
    m7_refresh<B>(vol, P, px, py, pz, m);
    int n = 0;
    for (int i = 0; i < kMaxSteps; i++) {
        const float qx = px * 0.5f + 0.5f, qy = py * 0.5f + 0.5f, qz = pz * 0.5f + 0.5f;
        if (qx < m.fx || qy < m.fy || qz < m.fz || qx > m.cx || qy > m.cy || qz > m.cz)
            m7_refresh<B>(vol, P, px, py, pz, m);  // inInterpolation, K:253-270, 396
        const float xd = (px * 0.5f + 0.5f - m.fx) / (m.cx - m.fx);
        const float yd = (py * 0.5f + 0.5f - m.fy) / (m.cy - m.fy);
        const float zd = (pz * 0.5f + 0.5f - m.fz) / (m.cz - m.fz);
        const float *mn = m.mean;
        const float m00 = (float)((double)mn[0] * (1.0 - (double)xd) + (double)(mn[1] * xd));
        const float m10 = (float)((double)mn[2] * (1.0 - (double)xd) + (double)(mn[3] * xd));
        const float m01 = (float)((double)mn[4] * (1.0 - (double)xd) + (double)(mn[5] * xd));
        const float m11 = (float)((double)mn[6] * (1.0 - (double)xd) + (double)(mn[7] * xd));
        const float m0 = (float)((double)m00 * (1.0 - (double)yd) + (double)(m10 * yd));
        const float m1 = (float)((double)m01 * (1.0 - (double)yd) + (double)(m11 * yd));
        const float im = (float)((double)m0 * (1.0 - (double)zd) + (double)(m1 * zd));
        const float sample = im * 50.0f;  // K:479
        n = i + 1;
        if (composite(P, sample, sx, sy, sz, sw)) break;
        t = t + kTStep;
        if (t > r.tfar) break;
        px = px + stx;
        py = py + sty;
        pz = pz + stz;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
}

// ---- synthetic volume ----
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <int B>
__global__ __launch_bounds__(256) void k_synth(float *__restrict__ vol, SynthArgs a) {
    const uint64_t nvox = (uint64_t)a.nx * a.ny * a.nz;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvox; v += stride) {
        const uint32_t x = (uint32_t)(v % (uint64_t)a.nx);
        const uint64_t yz = v / (uint64_t)a.nx;
        const uint32_t y = (uint32_t)(yz % (uint64_t)a.ny);
        const uint32_t z = (uint32_t)(yz / (uint64_t)a.ny);
        float f = 0.0f;
#pragma unroll
        for (int k = 0; k < kSynthBlobs; k++)
            f = f + ((a.amp[k] * a.gx[k * a.nx + x]) * a.gy[k * a.ny + y]) * a.gz[k * a.nz + z];
        if (f > 1.0f) f = 1.0f;
        const int nb = B > 0 ? B : a.nb;
        float *dst = vol + v * (uint64_t)nb;
        if (nb == 1) {
            dst[0] = f;
            continue;
        }
        int q = (int)(f * 4096.0f);
        if (q > kSynthQ - 1) q = kSynthQ - 1;
        const int g = (int)(splitmix64(a.seed ^ v) & (kSynthG - 1));
        const float *src = a.table + ((uint64_t)g * kSynthQ + (uint64_t)q) * (uint64_t)nb;
        if constexpr (B > 0 && B % 4 == 0) {
#pragma unroll
            for (int i = 0; i < B / 4; i++)
                reinterpret_cast<float4 *>(dst)[i] = reinterpret_cast<const float4 *>(src)[i];
        } else {
            for (int i = 0; i < nb; i++) dst[i] = src[i];
        }
    }
}

__global__ __launch_bounds__(256) void k_unscatter(const uint32_t *__restrict__ packed,
                                                   const uint32_t *__restrict__ lists,
                                                   uint32_t tiles_x, uint32_t *__restrict__ frame,
                                                   uint32_t W, uint32_t H) {
    const uint32_t tile = lists[blockIdx.x];
    if (tile == kPad) return;
    const uint32_t px = (tile % tiles_x) * kTile + (threadIdx.x & 15u);
    const uint32_t py = (tile / tiles_x) * kTile + (threadIdx.x >> 4);
    if (px >= W || py >= H) return;
    frame[(uint64_t)py * W + px] = packed[(uint64_t)blockIdx.x * 256u + threadIdx.x];
}

__global__ __launch_bounds__(256) void k_popcount(const unsigned long long *__restrict__ bits,
                                                  uint64_t nwords,
                                                  unsigned long long *__restrict__ total) {
    unsigned long long acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += stride)
        acc += __popcll(bits[i]);
    // wave reduction then one atomic per wave
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(total, acc);
}

// ------------------------------ launchers ---------------------------------

template <int B, bool COUNT>
static hipError_t march_b(int method, const float *vol, const Params &P, uint32_t nslots,
                          hipStream_t s) {
    const dim3 grid(nslots), block(256);
    switch (method) {
    case 1: hipLaunchKernelGGL((k_march<B, 1, COUNT>), grid, block, 0, s, vol, P); break;
    case 2: hipLaunchKernelGGL((k_march<B, 2, COUNT>), grid, block, 0, s, vol, P); break;
    case 3: hipLaunchKernelGGL((k_march<B, 3, COUNT>), grid, block, 0, s, vol, P); break;
    case 7:
        if (COUNT) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_march_m7<B>), grid, block, 0, s, vol, P);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <bool COUNT>
static hipError_t march_dispatch(int nb, int method, const float *vol, const Params &P,
                                 uint32_t nslots, hipStream_t s) {
    switch (nb) {
    case 1: return march_b<1, COUNT>(method, vol, P, nslots, s);
    case 2: return march_b<2, COUNT>(method, vol, P, nslots, s);
    case 4: return march_b<4, COUNT>(method, vol, P, nslots, s);
    case 8: return march_b<8, COUNT>(method, vol, P, nslots, s);
    case 16: return march_b<16, COUNT>(method, vol, P, nslots, s);
    case 32: return march_b<32, COUNT>(method, vol, P, nslots, s);
    default: return march_b<0, COUNT>(method, vol, P, nslots, s);
    }
}

hipError_t launch_march(int nb, int method, const float *vol, const Params &P,
                        uint32_t nslots, bool count, hipStream_t s) {
    if (nslots == 0) return hipSuccess;
    return count ? march_dispatch<true>(nb, method, vol, P, nslots, s)
                 : march_dispatch<false>(nb, method, vol, P, nslots, s);
}

hipError_t launch_synth(float *vol, const SynthArgs &a, hipStream_t s) {
    const uint64_t nvox = (uint64_t)a.nx * a.ny * a.nz;
    uint64_t blocks = (nvox + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    const dim3 grid((uint32_t)blocks), block(256);
    switch (a.nb) {
    case 1: hipLaunchKernelGGL((k_synth<1>), grid, block, 0, s, vol, a); break;
    case 4: hipLaunchKernelGGL((k_synth<4>), grid, block, 0, s, vol, a); break;
    case 8: hipLaunchKernelGGL((k_synth<8>), grid, block, 0, s, vol, a); break;
    case 16: hipLaunchKernelGGL((k_synth<16>), grid, block, 0, s, vol, a); break;
    case 32: hipLaunchKernelGGL((k_synth<32>), grid, block, 0, s, vol, a); break;
    default: hipLaunchKernelGGL((k_synth<0>), grid, block, 0, s, vol, a); break;
    }
    return hipGetLastError();
}

hipError_t launch_unscatter(const uint32_t *packed, const uint32_t *lists, uint32_t ntiles,
                            uint32_t tiles_x, uint32_t *frame, uint32_t W, uint32_t H,
                            hipStream_t s) {
    if (ntiles == 0) return hipSuccess;
    hipLaunchKernelGGL(k_unscatter, dim3(ntiles), dim3(256), 0, s, packed, lists, tiles_x,
                       frame, W, H);
    return hipGetLastError();
}

hipError_t launch_popcount(const unsigned long long *bits, uint64_t nwords,
                           unsigned long long *total, hipStream_t s) {
    uint64_t blocks = (nwords + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_popcount, dim3((uint32_t)blocks), dim3(256), 0, s, bits, nwords,
                       total);
    return hipGetLastError();
}

}  // namespace vr
