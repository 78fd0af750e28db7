// vr_stats.hip -- basicDataProcessing (K:1798-1887): per-voxel statistics baked
// once into float planes, the build's counterpart of the reference's
// originalQueryTex / fractalQueryTex (d_basicDataProcessing, K:722-871).
//
// The march decodes a statistic from the 8 corner records of every sample
// (methods 1-6); that statistic is a pure function of one
// record, so decoding it once per voxel into a plane and blending the plane's
// 8 corners with the same filter gives the same float for every sample, bit
// for bit.  A baked frame reads 4 bytes per corner voxel instead of B * 4
// (raw records) or a codebook entry + errors (codec), so the march is no
// longer bound by the distribution bytes.  Planes are laid out in 16 x 2 x 1
// bricks with a one-voxel x apron (plane_index, vr_device.h): plane k < 3 of
// the raw volume holds statistic k+1 of voxel (x, y, z), plane 3 method 7's
// corner mean (the codec volume: 3 planes).

#include "vr_internal.h"

namespace vr {

// a voxel's statistic at its home position and, for x = 15 k (k > 0), in the
// apron (offset 15) of brick k - 1
__device__ __forceinline__ void put_plane(float *__restrict__ out, uint32_t x, uint32_t y,
                                          uint32_t z, uint64_t psy, uint64_t psz, float v) {
    const uint64_t h = plane_index(x, y, z, psy, psz);
    out[h] = v;
    if (x > 0 && plane_bx(x) % 32u == 0) out[h - 32u + kPlaneStride] = v;
}

// One thread per voxel of an x-row (grid: x blocks of 256, y rows, z slices);
// each record is read once, coalesced, and its statistics written to the four
// planes (mean, variance, entropy; plane 3: method 7's undivided corner mean).  The same functions as the march (record_stat), so the
// planes hold exactly the per-corner values the march would decode; the
// entropy's exact logarithm uses the LDS table (both logarithm forms are
// exact, vr_selftest_logf).
template <int B>
__global__ __launch_bounds__(256) void k_bake_raw(const float *__restrict__ vol, Params P,
                                                  float *__restrict__ out, uint64_t plane,
                                                  uint64_t psy, uint64_t psz) {
    __shared__ LogEnt tab[65];
    copy_logtab(tab);
    __syncthreads();
    const uint32_t x = blockIdx.x * 256u + threadIdx.x;
    if (x >= (uint32_t)P.nx) return;
    const uint64_t off = (uint64_t)blockIdx.z * P.sz + (uint64_t)blockIdx.y * P.sy + x;
    float m, v, e, c;
    if constexpr (B > 0) {
        float p[B];
        load_rec<B>(vol, off, p);
        m = record_stat<B, 1>(p, P.enorm);
        v = record_stat<B, 2>(p, P.enorm);
        e = entropy_p<B>(p, P.enorm, tab);
        c = raw_mean<B>(p);
    } else {
        const float *p = vol + off * (uint64_t)P.nb;
        m = record_stat_rt<1>(p, P.nb, P.enorm);
        v = record_stat_rt<2>(p, P.nb, P.enorm);
        e = record_stat_rt<3>(p, P.nb, P.enorm);
        c = raw_mean_rt(p, P.nb);
    }
    const uint32_t y = blockIdx.y, z = blockIdx.z;
    put_plane(out, x, y, z, psy, psz, m);
    put_plane(out + plane, x, y, z, psy, psz, v);
    put_plane(out + 2 * plane, x, y, z, psy, psz, e);
    put_plane(out + 3 * plane, x, y, z, psy, psz, c);  // method 7's corner mean (K:347-367), before the / 0.0217
}

// codec voxels (methods 4/5/6, K:775-871): decode once, statistics C = 0, 1, 2
template <int B>
__global__ __launch_bounds__(256) void k_bake_codec(Params P, float *__restrict__ out,
                                                    uint64_t plane, uint64_t psy, uint64_t psz) {
    const uint32_t x = blockIdx.x * 256u + threadIdx.x;
    if (x >= (uint32_t)P.nx) return;
    const uint64_t off = (uint64_t)blockIdx.z * P.sz + (uint64_t)blockIdx.y * P.sy + x;
    float dec[B];
    codec_decode<B>(P, off, dec);
    const uint32_t y = blockIdx.y, z = blockIdx.z;
    put_plane(out, x, y, z, psy, psz, codec_stat_of<B, 0>(dec, P.enorm));
    put_plane(out + plane, x, y, z, psy, psz, codec_stat_of<B, 1>(dec, P.enorm));
    put_plane(out + 2 * plane, x, y, z, psy, psz, codec_stat_of<B, 2>(dec, P.enorm));
}

static bool bake_grid(const Params &P, dim3 &grid) {
    if (P.nx <= 0 || P.ny <= 0 || P.nz <= 0 || P.ny > 65535 || P.nz > 65535) return false;
    grid = dim3((uint32_t)(P.nx + 255) / 256u, (uint32_t)P.ny, (uint32_t)P.nz);
    return true;
}

hipError_t launch_bake_raw(const float *vol, const Params &P, float *out, uint64_t plane,
                           uint64_t psy, uint64_t psz, hipStream_t s) {
    dim3 grid;
    if (!bake_grid(P, grid)) return hipErrorInvalidValue;
    const dim3 block(256);
    switch (P.nb) {
    case 1: hipLaunchKernelGGL((k_bake_raw<1>), grid, block, 0, s, vol, P, out, plane, psy, psz); break;
    case 2: hipLaunchKernelGGL((k_bake_raw<2>), grid, block, 0, s, vol, P, out, plane, psy, psz); break;
    case 4: hipLaunchKernelGGL((k_bake_raw<4>), grid, block, 0, s, vol, P, out, plane, psy, psz); break;
    case 8: hipLaunchKernelGGL((k_bake_raw<8>), grid, block, 0, s, vol, P, out, plane, psy, psz); break;
    case 16: hipLaunchKernelGGL((k_bake_raw<16>), grid, block, 0, s, vol, P, out, plane, psy, psz); break;
    case 32: hipLaunchKernelGGL((k_bake_raw<32>), grid, block, 0, s, vol, P, out, plane, psy, psz); break;
    default: hipLaunchKernelGGL((k_bake_raw<0>), grid, block, 0, s, vol, P, out, plane, psy, psz); break;
    }
    return hipGetLastError();
}

hipError_t launch_bake_codec(const Params &P, float *out, uint64_t plane, uint64_t psy,
                             uint64_t psz, hipStream_t s) {
    dim3 grid;
    if (!bake_grid(P, grid)) return hipErrorInvalidValue;
    const dim3 block(256);
    switch (P.nb) {
    case 1: hipLaunchKernelGGL((k_bake_codec<1>), grid, block, 0, s, P, out, plane, psy, psz); break;
    case 2: hipLaunchKernelGGL((k_bake_codec<2>), grid, block, 0, s, P, out, plane, psy, psz); break;
    case 4: hipLaunchKernelGGL((k_bake_codec<4>), grid, block, 0, s, P, out, plane, psy, psz); break;
    case 8: hipLaunchKernelGGL((k_bake_codec<8>), grid, block, 0, s, P, out, plane, psy, psz); break;
    case 16: hipLaunchKernelGGL((k_bake_codec<16>), grid, block, 0, s, P, out, plane, psy, psz); break;
    case 32: hipLaunchKernelGGL((k_bake_codec<32>), grid, block, 0, s, P, out, plane, psy, psz); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---- 2x2 (x, y) micro-brick copy of an 8-bin volume (oblique views) ----
// One 128-B line holds the records (x, y), (x+1, y), (x, y+1), (x+1, y+1) of
// an even (x, y): record (x, y, z) sits at z*bsz + (y>>1)*bsy + (x>>1)*4 +
// (y&1)*2 + (x&1) (brick_index).  Like a cudaArray, the copy is the
// library's own layout of the uploaded records (K:1913-1918); the quad march
// of oblique views reads it.  One thread per record.
__global__ __launch_bounds__(256) void k_brick8(const float *__restrict__ vol, Params P,
                                                float *__restrict__ out, uint64_t bsy,
                                                uint64_t bsz) {
    const uint32_t x = blockIdx.x * 256u + threadIdx.x;
    if (x >= (uint32_t)P.nx) return;
    const uint32_t y = blockIdx.y, z = blockIdx.z;
    const uint64_t src = (uint64_t)z * P.sz + (uint64_t)y * P.sy + x;
    const uint64_t dst = brick_index(x, y, z, bsy, bsz);
    const float4 *s4 = reinterpret_cast<const float4 *>(vol + src * 8);
    float4 *d4 = reinterpret_cast<float4 *>(out + dst * 8);
    const float4 a = s4[0], b = s4[1];
    d4[0] = a;
    d4[1] = b;
}

// axis-rows copy (views along y / z): one thread per record, x-row reads coalesced
template <int B>
__global__ __launch_bounds__(256) void k_axis_copy(const float *__restrict__ vol, Params P,
                                                   float *__restrict__ out, uint64_t asx,
                                                   uint64_t asy, uint64_t asz) {
    const uint32_t x = blockIdx.x * 256u + threadIdx.x;
    if (x >= (uint32_t)P.nx) return;
    const uint32_t y = blockIdx.y, z = blockIdx.z;
    float r[B];
    load_rec<B>(vol, (uint64_t)z * P.sz + (uint64_t)y * P.sy + x, r);
    float *d = out + (x * asx + y * asy + z * asz) * B;
#pragma unroll
    for (int i = 0; i < B; i++) d[i] = r[i];
}

hipError_t launch_axis_copy(const float *vol, const Params &P, float *out, uint64_t asx,
                            uint64_t asy, uint64_t asz, hipStream_t s) {
    dim3 grid;
    if (!bake_grid(P, grid)) return hipErrorInvalidValue;
    switch (P.nb) {
    case 1: hipLaunchKernelGGL(k_axis_copy<1>, grid, dim3(256), 0, s, vol, P, out, asx, asy, asz); break;
    case 2: hipLaunchKernelGGL(k_axis_copy<2>, grid, dim3(256), 0, s, vol, P, out, asx, asy, asz); break;
    case 4: hipLaunchKernelGGL(k_axis_copy<4>, grid, dim3(256), 0, s, vol, P, out, asx, asy, asz); break;
    case 8: hipLaunchKernelGGL(k_axis_copy<8>, grid, dim3(256), 0, s, vol, P, out, asx, asy, asz); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Axis copy of one baked plane (views whose screen x runs along the volume's y
// or z): the plane's 16 x 2 x 1 bricks with that axis in the
// brick rows -- axis 1: y rows (y fast, x pairs, z slices), axis 2: z rows (z
// fast, y pairs, x slices); gather8 MODE 4 / 5 reads it.  One thread per
// voxel, grid over (fast, pair, slow) of the copy so its writes are coalesced.
__global__ __launch_bounds__(256) void k_plane_axis(const float *__restrict__ src, uint64_t ssy,
                                                    uint64_t ssz, float *__restrict__ out,
                                                    uint64_t dsy, uint64_t dsz, uint32_t nfast,
                                                    int axis) {
    const uint32_t f = blockIdx.x * 256u + threadIdx.x;
    if (f >= nfast) return;
    const uint32_t p = blockIdx.y, s = blockIdx.z;
    const uint32_t x = axis == 2 ? s : p, y = axis == 2 ? p : f, z = axis == 2 ? f : s;
    put_plane(out, f, p, s, dsy, dsz, src[plane_index(x, y, z, ssy, ssz)]);
}

hipError_t launch_plane_axis(const float *src, uint64_t ssy, uint64_t ssz, float *out,
                             uint64_t dsy, uint64_t dsz, int nx, int ny, int nz, int axis,
                             hipStream_t s) {
    const uint32_t nf = axis == 2 ? nz : ny, np = axis == 2 ? ny : nx, ns = axis == 2 ? nx : nz;
    if (nf == 0 || np == 0 || ns == 0 || np > 65535 || ns > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_plane_axis, dim3((nf + 255) / 256, np, ns), dim3(256), 0, s, src, ssy,
                       ssz, out, dsy, dsz, nf, axis);
    return hipGetLastError();
}

hipError_t launch_brick8(const float *vol, const Params &P, float *out, uint64_t bsy,
                         uint64_t bsz, hipStream_t s) {
    dim3 grid;
    if (!bake_grid(P, grid)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_brick8, grid, dim3(256), 0, s, vol, P, out, bsy, bsz);
    return hipGetLastError();
}

// Streaming read of a resident buffer (bench.py's measured read ceiling,
// SURVEY.md 8(d)): every 16-B chunk read once, coalesced (16 B per lane, 4
// loads in flight per lane), grid-strided over a fixed grid; the chunks are
// folded into one xor per thread and one word per workgroup so no load is dead.
__global__ __launch_bounds__(256) void k_stream_read(const uint4 *__restrict__ p, uint64_t n,
                                                     uint32_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    uint32_t acc = 0;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
        acc ^= c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
    }
    for (; i < n; i += stride) {
        const uint4 a = p[i];
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    __shared__ uint32_t red[256];
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t v = red[threadIdx.x] ^ red[threadIdx.x + 64] ^ red[threadIdx.x + 128] ^
                           red[threadIdx.x + 192];
        red[threadIdx.x] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t v = 0;
        for (int k = 0; k < 64; k++) v ^= red[k];
        out[blockIdx.x] = v;
    }
}

hipError_t launch_stream_read(const void *buf, uint64_t bytes, uint32_t *out, uint32_t nblocks,
                              hipStream_t s) {
    if (!buf || !out || nblocks == 0 || (reinterpret_cast<uintptr_t>(buf) & 15u))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_stream_read, dim3(nblocks), dim3(256), 0, s,
                       reinterpret_cast<const uint4 *>(buf), bytes / 16u, out);
    return hipGetLastError();
}

}  // namespace vr
