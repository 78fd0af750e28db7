// vr_flex.hip -- flexible blocks (queryMethod 8/9/0): the dataProcessing
// pre-pass (K:1735-1796) and the march that samples its block statistics.
//
// The reference builds per-block statistics from an integral histogram stored
// as dyadic "spans" (loaders C:709-997): every block corner's prefix box
// [1, x] x [1, y] x [1, z] is split into dyadic sub-spans (K:1248-1282), each
// sub-span's histogram is looked up -- fractal-coded (template, flip, shift,
// sparse errors, renormalised) when it holds >= 8 voxels, else a sparse
// "simple" histogram -- and summed weighted by its voxel count (K:1318-1544);
// the block histogram is +c0+c3+c4+c7-c1-c2-c5-c6 of its 8 corner sums
// (K:1041-1051, the reference's sign pattern and corner choice kept), clamped,
// normalised, and reduced to mean / variance / entropy (K:1053-1119).  The
// march samples those with an unnormalised linear texture of 500^3 float4
// (zeros past the blocks, K:1691-1714) at (p*0.5+0.5)*nFlexBlock (K:654-680).
//
// MI355X form: the reference scans all 131072 table entries per sub-span (a
// 194 s pre-pass, ver1.9.6.txt:9); here the host sorts the span keys once and
// every sub-span is a binary search.  One workgroup per corner decodes its
// sub-spans in parallel into LDS and one lane per bin sums them in sub-span
// order (the reference's shared-memory float atomics have no fixed order;
// DESIGN.md 4.7 lists this and the other choices for undefined behaviour).
#include "vr_internal.h"
#include "vr_march.h"

namespace vr {

constexpr int kFlexSubMax = 216;             // 6 x 6 x 6 dyadic sub-spans (K:881)
constexpr int kFlexRow = kFlexMaxBins + 1;   // LDS row stride (bank spread)

__device__ __forceinline__ int flex_split(int x, int (&lo)[6], int (&hi)[6]) {
    int n = 0;
    for (int i = 0; i <= 6; i++) {  // K:1248-1258
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

__device__ __forceinline__ int flex_lookup(const uint64_t *keys, const int32_t *idx, int n,
                                           uint64_t key) {
    int a = 0, b = n;  // first key >= key
    while (a < b) {
        const int m = (a + b) >> 1;
        if (keys[m] < key) a = m + 1; else b = m;
    }
    return (a < n && keys[a] == key) ? idx[a] : -1;
}

// one workgroup per corner (block n = blockIdx / 8, corner blockIdx % 8)
__global__ __launch_bounds__(256) void k_flex_corners(FlexTables T, int bs, int nblk,
                                                      float *__restrict__ corner_hist,
                                                      unsigned int *missing) {
    __shared__ float sh[kFlexSubMax * kFlexRow];
    const int cid = blockIdx.x, n = cid >> 3, c = cid & 7;
    const int D = T.dim, nb = T.nb;
    const int bx = n % nblk, by = (n / nblk) % nblk, bz = n / (nblk * nblk);
    // block span, K:935-1024 (1-based, last block cut at D); corners K:1151-1228
    const int x = (c & 1) ? (bx == nblk - 1 ? D : (bx + 1) * bs) : 1 + bx * bs;
    const int y = (c & 2) ? (by == nblk - 1 ? D : (by + 1) * bs) : 1 + by * bs;
    const int z = (c & 4) ? (bz == nblk - 1 ? D : (bz + 1) * bs) : 1 + bz * bs;
    int xl[6], xh[6], yl[6], yh[6], zl[6], zh[6];
    const int nx = flex_split(x, xl, xh), ny = flex_split(y, yl, yh), nz = flex_split(z, zl, zh);
    const int nsub = nx * ny * nz;
    const int t = threadIdx.x;
    if (t < nsub) {
        const int i = t / (ny * nz), j = (t / nz) % ny, k = t % nz;
        int l[3] = {0, 0, 0}, h[3] = {0, 0, 0};
        // fixed-index selects keep the split arrays in registers
#pragma unroll
        for (int q = 0; q < 6; q++) {
            if (q == i) { l[0] = xl[q]; h[0] = xh[q]; }
            if (q == j) { l[1] = yl[q]; h[1] = yh[q]; }
            if (q == k) { l[2] = zl[q]; h[2] = zh[q]; }
        }
        const int w = (h[0] - l[0] + 1) * (h[1] - l[1] + 1) * (h[2] - l[2] + 1);
        float *row = sh + t * kFlexRow;
        bool found = false;
        if (w >= 8) {  // fractal-coded span, K:1349-1437
            const int e = flex_lookup(T.fkeys, T.fidx, T.nfk,
                                      span_key(l[0], l[1], l[2], h[0], h[1], h[2]));
            if (e >= 0) {
                found = true;
                const int4 cb = T.fcode[e];
                const float *orig = T.tpl + (size_t)cb.x * nb;
                for (int q = 0; q < nb; q++) {  // flexibleFractalDecoding, K:225-250
                    int m = q + cb.y;
                    if (m >= nb) m -= nb;
                    row[m] = cb.z ? orig[nb - 1 - q] : orig[q];
                }
                const float2 *er = T.ferr + (size_t)e * nb;
                for (int q = 0; q < cb.w; q++) {  // K:1400-1418
                    const float2 ev = er[q];
                    const int b = (int)ev.x;
                    if (b < 0 || b >= nb) continue;
                    float v = row[b] + ev.y;
                    row[b] = v < 0 ? 0.0f : v;
                }
                float total = 0.0f;  // K:1420-1431
                for (int q = 0; q < nb; q++) total = total + row[q];
                for (int q = 0; q < nb; q++) row[q] = row[q] / total;
            }
        } else {  // simple histogram, 0-based span, K:1438-1531
            const int e = flex_lookup(T.skeys, T.sidx, T.nsk,
                                      span_key(l[0] - 1, l[1] - 1, l[2] - 1, h[0] - 1, h[1] - 1,
                                               h[2] - 1));
            for (int q = 0; q < nb; q++) row[q] = 0.0f;
            if (e >= 0) {
                found = true;
                const float2 *pr = T.shist + (size_t)e * nb;
                for (int q = 0; q < T.scount[e]; q++) {
                    const float2 pv = pr[q];
                    const int b = (int)pv.x;
                    if (b < 0 || b >= nb) continue;
                    row[b] = pv.y;
                }
            }
        }
        if (!found) {
            atomicOr(missing, 1u);
            for (int q = 0; q < nb; q++) row[q] = 0.0f;
        }
        const float fw = (float)w;
        for (int q = 0; q < nb; q++) row[q] = row[q] * fw;  // K:1402, 1520
    }
    __syncthreads();
    if (t < nb) {
        float acc = 0.0f;
        for (int s = 0; s < nsub; s++) acc = acc + sh[s * kFlexRow + t];
        corner_hist[(size_t)cid * nb + t] = acc;
    }
}

// d_computeBlock, K:1033-1126: one 64-lane workgroup per block
__global__ __launch_bounds__(64) void k_flex_blocks(int nb, const float *__restrict__ ch,
                                                    float4 *__restrict__ out) {
    __shared__ float h[kFlexMaxBins];
    __shared__ float tot;
    const int n = blockIdx.x, s = threadIdx.x;
    const float *c = ch + (size_t)n * 8 * nb;
    if (s < nb) {
        float v = c[0 * nb + s] + c[3 * nb + s] + c[4 * nb + s] + c[7 * nb + s] -
                  c[1 * nb + s] - c[2 * nb + s] - c[5 * nb + s] - c[6 * nb + s];
        h[s] = v < 0 ? 0.0f : v;
    }
    __syncthreads();
    if (s == 0) {
        float total = 0.0f;
        for (int q = 0; q < nb; q++) total += h[q];
        tot = total;
    }
    __syncthreads();
    const float total = tot;
    if (s < nb && !(total <= 0)) {
        float v = h[s] / total;
        if (v < 0) v = 0;
        if (v > 1) v = 1;
        h[s] = v;
    }
    __syncthreads();
    if (s == 0) {
        const float bw = (255.0f - 0.0f) / (float)nb;
        const double half = (double)bw / 2.0;
        float mean = 0.0f;
        for (int i = 0; i < nb; i++)
            mean = (float)((double)mean + (double)h[i] * ((double)(bw * (float)i) + half));
        float var = 0.0f;
        for (int i = 0; i < nb; i++) {
            const double d = ((double)(bw * (float)i) + half) - (double)mean;
            var = (float)((double)var + (double)h[i] * d * d);
        }
        float ent = 0.0f;
        for (int i = 0; i < nb; i++) {
            const float pr = h[i];
            const double t = pr <= 0 ? 0.0 : div_ln2(logf_canon(pr));
            ent = (float)((double)ent + (double)pr * t);
        }
        ent = -ent;
        // log((float)flexNBin) / log(2.0f), float overloads (K:1115)
        const float enorm = (float)log((double)(float)nb) / (float)log((double)2.0f);
        out[n] = make_float4(mean, var, ent / enorm, 0.0f);
    }
}

// flexBlockTex: unnormalised coordinate, linear filter, clamp on 500^3 texels
// holding the blocks at [0, nflex) per axis and zeros elsewhere (K:1691-1714)
constexpr int kFlexTex = 500;  // nMaxBlockDim, K:93
__device__ __forceinline__ void lin_axis_unnorm(float u, int &i0, int &i1, float &a) {
    const float xb = u - 0.5f;
    const float fl = floorf(xb);
    const int i = (int)fl;
    a = q8(xb - fl);
    i0 = max(0, min(kFlexTex - 1, i));
    i1 = max(0, min(kFlexTex - 1, i + 1));
}

template <int C>
__device__ __forceinline__ float flex_texel(const Params &P, int x, int y, int z) {
    const int n = P.nflex;
    if (x >= n || y >= n || z >= n) return 0.0f;
    const float4 v = P.flex[((size_t)z * n + y) * n + x];
    return C == 0 ? v.x : (C == 1 ? v.y : v.z);
}

template <int C>
__device__ __forceinline__ float flex_sample(const Params &P, float px, float py, float pz) {
    const float nf = (float)P.nflex;
    int x0, x1, y0, y1, z0, z1;
    float ax, ay, az;
    lin_axis_unnorm((px * 0.5f + 0.5f) * nf, x0, x1, ax);
    lin_axis_unnorm((py * 0.5f + 0.5f) * nf, y0, y1, ay);
    lin_axis_unnorm((pz * 0.5f + 0.5f) * nf, z0, z1, az);
    const float c00 = lerpq(flex_texel<C>(P, x0, y0, z0), flex_texel<C>(P, x1, y0, z0), ax);
    const float c10 = lerpq(flex_texel<C>(P, x0, y1, z0), flex_texel<C>(P, x1, y1, z0), ax);
    const float c01 = lerpq(flex_texel<C>(P, x0, y0, z1), flex_texel<C>(P, x1, y0, z1), ax);
    const float c11 = lerpq(flex_texel<C>(P, x0, y1, z1), flex_texel<C>(P, x1, y1, z1), ax);
    const float c0 = lerpq(c00, c10, ay);
    const float c1 = lerpq(c01, c11, ay);
    return lerpq(c0, c1, az);
}

// the d_render march (K:282-716) with the flexible-block sample source; the
// block table is a few KiB and stays in L2, so one lane per ray marches plainly
template <int C>
__global__ __launch_bounds__(256) void k_march_flex(Params P) {
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;
    uint32_t lx, ly;
    tile_pixel(threadIdx.x, lx, ly);
    const uint32_t x = (tile % P.tiles_x) * kTileW + lx;
    const uint32_t y = (tile / P.tiles_x) * kTileH + ly;
    if (x >= P.CW || y >= P.CH) return;
    const uint64_t o = P.tile_list ? (uint64_t)slot * 256u + ly * kTileW + lx
                                   : (uint64_t)y * P.W + x;
    Ray r;
    if (!make_ray(P, x, y, r)) {
        write_miss(P, o);
        return;
    }
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = r.tnear;
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
    int n = 0;
    for (int i = 0; i < kMaxSteps; i++) {
        n = i + 1;
        if (composite(P, flex_sample<C>(P, px, py, pz), sx, sy, sz, sw)) break;  // K:698
        t = t + kTStep;            // K:701
        if (t > r.tfar) break;     // K:703
        px = px + stx;             // K:706
        py = py + sty;
        pz = pz + stz;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
}

hipError_t launch_flex_corners(const FlexTables &t, int block, int nblk, float *corner_hist,
                               unsigned int *missing, hipStream_t s) {
    const uint32_t ncorner = (uint32_t)nblk * nblk * nblk * 8u;
    hipLaunchKernelGGL(k_flex_corners, dim3(ncorner), dim3(256), 0, s, t, block, nblk,
                       corner_hist, missing);
    return hipGetLastError();
}

hipError_t launch_flex_blocks(int nb, int nblk, const float *corner_hist, float4 *blocks,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_flex_blocks, dim3((uint32_t)nblk * nblk * nblk), dim3(64), 0, s, nb,
                       corner_hist, blocks);
    return hipGetLastError();
}

hipError_t launch_march_flex(int method, const Params &P, uint32_t nslots, hipStream_t s) {
    const dim3 grid(nslots), block(256);
    switch (method) {  // K:654-680: 9 -> .x mean, 0 -> .y variance, 8 -> .z entropy
    case 9: hipLaunchKernelGGL((k_march_flex<0>), grid, block, 0, s, P); break;
    case 0: hipLaunchKernelGGL((k_march_flex<1>), grid, block, 0, s, P); break;
    case 8: hipLaunchKernelGGL((k_march_flex<2>), grid, block, 0, s, P); break;
    default: return hipErrorInvalidValue;
    }
    note_kernel("k_march_flex", P.nb, method);
    return hipGetLastError();
}

}  // namespace vr
