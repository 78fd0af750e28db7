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

#include <algorithm>
#include <type_traits>

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
    __shared__ LogEnt tab[kLogTabN];
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
// of oblique views reads it.  One thread per record, a
// workgroup per 128 x 2 records (y pair 2 by): lanes 4q .. 4q+3 write the
// whole line of x pair q, and each row's 128 records are read as 4 KB runs.
// (One row per workgroup wrote every line in two halves from two workgroups:
// 1024^3 x 8, 17.4 ms; profiles/r04/final/kernel_stats_1024x8_C1.csv.)
__global__ __launch_bounds__(256) void k_brick8(const float *__restrict__ vol, Params P,
                                                float *__restrict__ out, uint64_t bsy,
                                                uint64_t bsz) {
    const uint32_t t = threadIdx.x;
    const uint32_t x = blockIdx.x * 128u + (t >> 2) * 2u + (t & 1u);
    const uint32_t y = blockIdx.y * 2u + ((t >> 1) & 1u), z = blockIdx.z;
    if (x >= (uint32_t)P.nx || y >= (uint32_t)P.ny) return;
    const uint64_t src = (uint64_t)z * P.sz + (uint64_t)y * P.sy + x;
    const uint64_t dst = brick_index(x, y, z, bsy, bsz);
    const float4 *s4 = reinterpret_cast<const float4 *>(vol + src * 8);
    float4 *d4 = reinterpret_cast<float4 *>(out + dst * 8);
    const float4 a = s4[0], b = s4[1];
    d4[0] = a;
    d4[1] = b;
}

// Axis-rows copy (views along y / z, axis_copy_strides): a transpose of x with
// the copy's fast axis f (y or z) in every slice s of the third axis.  One
// workgroup moves a 32 (x) x 32 (f) tile through LDS: it reads 32 x rows of 32
// records (32*B floats contiguous each) and writes 32 f runs of 32 records, so
// both sides are whole lines.  A record-per-thread copy wrote each record to
// its own line (1024^3 x 8 z rows: 60.3 ms, ~1.1 TB/s of the 64 GiB moved;
// profiles/r04/final/kernel_stats_1024x8_S.csv).  Element granularity is a
// float4 for B >= 4, a float below; LDS rows are padded by one float4.
constexpr int AXT = 32;
template <int B>
__global__ __launch_bounds__(256) void k_axis_copy(const float *__restrict__ vol,
                                                   float *__restrict__ out, uint32_t nx,
                                                   uint32_t nf, uint64_t ssf, uint64_t sss,
                                                   uint64_t dsx, uint64_t dss, uint32_t tiles_x) {
    using V = typename std::conditional<(B >= 4), float4, float>::type;
    constexpr int RS = B >= 4 ? B / 4 : B;             // V slots per record
    constexpr int PER_ROW = AXT * RS;                  // V slots of one 32-record row
    constexpr int ROW = PER_ROW + 1;
    __shared__ V tile[AXT * ROW];
    const uint32_t tx = blockIdx.x % tiles_x, tf = blockIdx.x / tiles_x, s = blockIdx.y;
    const uint32_t x0 = tx * AXT, f0 = tf * AXT;
    const uint32_t wx = min((uint32_t)AXT, nx - x0), wf = min((uint32_t)AXT, nf - f0);
    const V *src = reinterpret_cast<const V *>(vol);
    V *dst = reinterpret_cast<V *>(out);
    // read: row f of the tile = records (x0 .. x0+31, f0 + f, s), contiguous in x
    for (int e = threadIdx.x; e < AXT * PER_ROW; e += 256) {
        const int f = e / PER_ROW, c = e % PER_ROW;    // c = x * RS + slot
        const uint32_t x = c / RS;
        if ((uint32_t)f < wf && x < wx) {
            const uint64_t rec = (uint64_t)s * sss + (uint64_t)(f0 + f) * ssf + x0;
            tile[f * ROW + c] = src[rec * RS + c];
        }
    }
    __syncthreads();
    // write: run x of the copy = records (x0 + x, f0 .. f0+31, s), contiguous in f
    for (int e = threadIdx.x; e < AXT * PER_ROW; e += 256) {
        const int x = e / PER_ROW, c = e % PER_ROW;    // c = f * RS + slot
        const uint32_t f = c / RS, k = c % RS;
        if ((uint32_t)x < wx && f < wf) {
            const uint64_t rec = (uint64_t)s * dss + (uint64_t)(x0 + x) * dsx + f0;
            dst[rec * RS + c] = tile[f * ROW + x * RS + k];
        }
    }
}

hipError_t launch_axis_copy(const float *vol, const Params &P, float *out, uint64_t asx,
                            uint64_t asy, uint64_t asz, hipStream_t s) {
    if (P.nx <= 0 || P.ny <= 0 || P.nz <= 0) return hipErrorInvalidValue;
    // fast axis of the copy: stride 1 (axis_copy_strides); s = the remaining one
    const bool zrows = asz == 1;
    if (!(zrows || asy == 1)) return hipErrorInvalidValue;
    const uint32_t nf = zrows ? P.nz : P.ny, ns = zrows ? P.ny : P.nz;
    const uint64_t ssf = zrows ? P.sz : P.sy, sss = zrows ? P.sy : P.sz;
    const uint64_t dss = zrows ? asy : asz;
    const uint32_t tiles_x = (P.nx + AXT - 1) / AXT, tiles_f = (nf + AXT - 1) / AXT;
    if (ns > 65535 || (uint64_t)tiles_x * tiles_f > 0x7fffffffull) return hipErrorInvalidValue;
    const dim3 grid(tiles_x * tiles_f, ns);
#define VR_AXC(BB)                                                                                 \
    hipLaunchKernelGGL(k_axis_copy<BB>, grid, dim3(256), 0, s, vol, out, (uint32_t)P.nx, nf, ssf, \
                       sss, asx, dss, tiles_x)
    switch (P.nb) {
    case 1: VR_AXC(1); break;
    case 2: VR_AXC(2); break;
    case 4: VR_AXC(4); break;
    case 8: VR_AXC(8); break;
    default: return hipErrorInvalidValue;
    }
#undef VR_AXC
    return hipGetLastError();
}

// Axis copy of one baked plane (views whose screen x runs along the volume's y
// or z): the plane's 16 x 2 x 1 bricks with that axis in the
// brick rows -- axis 1: y rows (y fast, x pairs, z slices), axis 2: z rows (z
// fast, y pairs, x slices); gather8 MODE 4 / 5 reads it.  A workgroup moves a
// tile of 30 x by 30 f (the copy's fast axis; 30 = two bricks' home runs) --
// for axis 2 by a y pair, for axis 1 in one z slice -- through LDS: it reads
// whole source bricks (x runs) and writes whole copy bricks (f runs), the
// apron voxel of each copy brick included (put_plane).  One voxel per thread
// with the grid over the copy's order read the source across its lines
// (1024^3 z rows: 20.6 ms for 8 GiB moved; profiles/r04/final/bench_1024x8_S_baked.json).
constexpr int PLT = 30;
__global__ __launch_bounds__(256) void k_plane_axis(const float *__restrict__ src, uint64_t ssy,
                                                    uint64_t ssz, float *__restrict__ out,
                                                    uint64_t dsy, uint64_t dsz, uint32_t nx,
                                                    uint32_t ny, uint32_t nz, int axis,
                                                    uint32_t tiles_x) {
    constexpr int XP = PLT + 1;                           // padded x extent in LDS
    __shared__ float tile[2 * PLT * XP];                  // [o][f][x], o: the y pair (axis 2)
    const uint32_t nf = axis == 2 ? nz : ny;
    const uint32_t x0 = (blockIdx.x % tiles_x) * PLT, f0 = (blockIdx.x / tiles_x) * PLT;
    const uint32_t no = axis == 2 ? 2u : 1u;              // y rows (axis 2) / z slices (axis 1)
    const uint32_t o0 = blockIdx.y * no;                  // first y (axis 2) / the z (axis 1)
    const uint32_t wx = min((uint32_t)PLT, nx - x0), wf = min((uint32_t)PLT, nf - f0);
    const uint32_t wo = min(no, (axis == 2 ? ny : nz) - o0);
    for (uint32_t e = threadIdx.x; e < no * PLT * PLT; e += 256) {
        const uint32_t xi = e % PLT, fi = (e / PLT) % PLT, oi = e / (PLT * PLT);
        if (xi < wx && fi < wf && oi < wo) {
            const uint32_t x = x0 + xi, f = f0 + fi, o = o0 + oi;
            const uint32_t y = axis == 2 ? o : f, z = axis == 2 ? f : o;
            tile[(oi * PLT + fi) * XP + xi] = src[plane_index(x, y, z, ssy, ssz)];
        }
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < no * PLT * PLT; e += 256) {
        const uint32_t fi = e % PLT, xi = (e / PLT) % PLT, oi = e / (PLT * PLT);
        if (xi < wx && fi < wf && oi < wo) {
            const uint32_t x = x0 + xi, f = f0 + fi, o = o0 + oi;
            // copy coordinates (fast, pair, slow): axis 2 (z, y, x), axis 1 (y, x, z)
            const uint32_t pp = axis == 2 ? o : x, ss = axis == 2 ? x : o;
            put_plane(out, f, pp, ss, dsy, dsz, tile[(oi * PLT + fi) * XP + xi]);
        }
    }
}

hipError_t launch_plane_axis(const float *src, uint64_t ssy, uint64_t ssz, float *out,
                             uint64_t dsy, uint64_t dsz, int nx, int ny, int nz, int axis,
                             hipStream_t s) {
    if (nx <= 0 || ny <= 0 || nz <= 0 || (axis != 1 && axis != 2) || nx >= 65536 ||
        ny >= 65536 || nz >= 65536)
        return hipErrorInvalidValue;
    const uint32_t nf = axis == 2 ? nz : ny;
    const uint32_t tiles_x = (nx + PLT - 1) / PLT, tiles_f = (nf + PLT - 1) / PLT;
    const uint32_t gy = axis == 2 ? (uint32_t)(ny + 1) / 2u : (uint32_t)nz;
    hipLaunchKernelGGL(k_plane_axis, dim3(tiles_x * tiles_f, gy), dim3(256), 0, s, src, ssy, ssz,
                       out, dsy, dsz, (uint32_t)nx, (uint32_t)ny, (uint32_t)nz, axis, tiles_x);
    return hipGetLastError();
}

// the 8 x 2 x 2 brick copy of a 16 x 2 x 1 plane (oblique views, gather8 MODE
// 6): one thread per copy float, in the copy's order (brick, then y, z, x in
// the brick), so the writes are whole lines; the reads walk 8-voxel x runs of
// the source bricks
__global__ __launch_bounds__(256) void k_plane8(const float *__restrict__ src, uint64_t ssy,
                                                uint64_t ssz, float *__restrict__ out,
                                                uint64_t total, uint32_t nbx, uint32_t nyp,
                                                uint32_t nx, uint32_t ny, uint32_t nz) {
    for (uint64_t e = (uint64_t)blockIdx.x * 256u + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * 256u) {
        const uint32_t o = (uint32_t)(e & 31u);
        const uint64_t brick = e >> 5;
        const uint32_t kx = (uint32_t)(brick % nbx);
        const uint64_t rest = brick / nbx;
        const uint32_t yp = (uint32_t)(rest % nyp), zp = (uint32_t)(rest / nyp);
        const uint32_t x = kPlane8Stride * kx + (o & 7u), y = 2u * yp + ((o >> 3) & 1u);
        const uint32_t z = 2u * zp + (o >> 4);
        out[e] = (x < nx && y < ny && z < nz) ? src[plane_index(x, y, z, ssy, ssz)] : 0.0f;
    }
}

hipError_t launch_plane8(const float *src, uint64_t ssy, uint64_t ssz, float *out, uint64_t dsy,
                         uint64_t dsz, int nx, int ny, int nz, hipStream_t s) {
    if (nx <= 0 || ny <= 0 || nz <= 0 || nx >= 65536 || ny >= 65536 || nz >= 65536)
        return hipErrorInvalidValue;
    const uint32_t nbx = (uint32_t)(dsy / 32u), nyp = (uint32_t)(ny + 1) / 2u;
    const uint64_t total = dsz * (uint64_t)((nz + 1) / 2);
    if (dsz != (uint64_t)nyp * dsy) return hipErrorInvalidValue;
    const uint64_t blocks = std::min<uint64_t>((total + 255) / 256, 1u << 20);
    hipLaunchKernelGGL(k_plane8, dim3((uint32_t)blocks), dim3(256), 0, s, src, ssy, ssz, out,
                       total, nbx, nyp, (uint32_t)nx, (uint32_t)ny, (uint32_t)nz);
    return hipGetLastError();
}

hipError_t launch_brick8(const float *vol, const Params &P, float *out, uint64_t bsy,
                         uint64_t bsz, hipStream_t s) {
    if (P.nx <= 0 || P.ny <= 0 || P.nz <= 0 || P.nz > 65535) return hipErrorInvalidValue;
    const dim3 grid((uint32_t)(P.nx + 127) / 128u, (uint32_t)(P.ny + 1) / 2u, (uint32_t)P.nz);
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
