// vr_m7.hip -- method 7 (K:320-367, 395-480): the software-trilinear blend of
// corner means, stateful along the ray (a cell's 8 corner means are refreshed
// only when the sample leaves the cell, inInterpolation K:253-270).
//
//  k_march_m7_quad   B = 8 oblique views, method-7 grid = volume: quad lanes
//                    gather a cell's corners as contiguous 64-B x-pairs
//  k_march_m7_pipe   B <= 8: the next position's cell gathered ahead
//  k_march_m7        any B (runtime B = 0), and baked corner means (BK)
//  k_march_m7wq      B = 16, 32: quad-cooperative refreshes + DPP transpose
//
// K = volumeRender_kernel.cu of the reference.
#include "vr_device.h"
#include "vr_internal.h"
#include "vr_march.h"
#include "vr_quad.h"

#include <cstdlib>

namespace vr {

struct M7Cell {
    float fx, fy, fz, cx, cy, cz;
};

__device__ __forceinline__ M7Cell m7_cell(const Params &P, float px, float py, float pz) {
    const float qx = px * 0.5f + 0.5f, qy = py * 0.5f + 0.5f, qz = pz * 0.5f + 0.5f;
    M7Cell c;
    c.fx = floorf(qx * (float)P.m7x) / (float)P.m7x;
    c.cx = ceilf(qx * (float)P.m7x) / (float)P.m7x;
    c.fy = floorf(qy * (float)P.m7y) / (float)P.m7y;
    c.cy = ceilf(qy * (float)P.m7y) / (float)P.m7y;
    c.fz = floorf(qz * (float)P.m7z) / (float)P.m7z;
    c.cz = ceilf(qz * (float)P.m7z) / (float)P.m7z;
    return c;
}

// ---- method 7, quad-cooperative (B == 8, oblique views) ----
// k_march_m7_pipe's corner cache with the quad march's gathers: the 4 lanes of
// a quad read each of their 4 rays' cell corners as contiguous 64-byte x-pairs
// (qc_gather), a pair swap gives lane g the records of corner (x = g>>1,
// y = g&1) at z0 and z1, and lane g keeps the corner means of those two
// corners for every ray of its quad (refreshed only when the ray leaves its
// cell, K:253-270, 396).  The blend gathers a ray's 8 means inside the quad
// (quad_perm broadcasts) and evaluates K:395-480's double lerps exactly as the
// one-lane march.  The next position's cell is gathered group by group while
// the current one blends (rolling prefetch); when no refresh follows, those
// records are the current cell's (cache hits) and are discarded.  Used when the
// method-7 grid equals the volume (cell corners then lie within 2 voxels).
// A cell's corner voxels are point-sampled from its float bounds (K:359-364):
// floor(floor(q N)/N * N) can come out one below floor(q N), so x1 - x0 (and
// y, z) is 0, 1 or 2 -- the pair is not always adjacent.  The cell is packed
// with both corners of every axis (w0 = x0 | x1 << 16, w1 = y0 | y1 << 16,
// w2 = z0 | z1 << 16, w3 = live), and lane g reads 16-byte chunk g & 1 of
// record x0 (g < 2) or x1 (g >= 2): one contiguous 64-byte run per combo when
// the records are adjacent, the two halves otherwise.
struct CellPacked {
    int w0, w1, w2, w3;
};

__device__ __forceinline__ CellPacked pack_cell(const Params &P, const M7Cell &c, bool live) {
    CellPacked p;
    p.w0 = point_axis(c.fx, P.nx) | (point_axis(c.cx, P.nx) << 16);
    p.w1 = point_axis(c.fy, P.ny) | (point_axis(c.cy, P.ny) << 16);
    p.w2 = point_axis(c.fz, P.nz) | (point_axis(c.cz, P.nz) << 16);
    p.w3 = live ? 1 : 0;
    return p;
}

// BR: vol is the 2x2 (x, y) micro-brick copy (brick_index; P.sy / P.sz are its pitches)
template <int G, bool BR = false>
__device__ __forceinline__ bool qc_gather_cell(const float *__restrict__ vol, const Params &P,
                                               const CellPacked &cp, uint32_t g, float4 (&L)[4]) {
    const bool live = bcast_g<G>(cp.w3) != 0;
    if (live) {
        const uint32_t w0 = (uint32_t)bcast_g<G>(cp.w0), w1 = (uint32_t)bcast_g<G>(cp.w1),
                       w2 = (uint32_t)bcast_g<G>(cp.w2);
        const uint64_t xr = g < 2 ? (w0 & 0xFFFFu) : (w0 >> 16);
        const uint64_t y0 = w1 & 0xFFFFu, y1 = w1 >> 16, z0 = w2 & 0xFFFFu, z1 = w2 >> 16;
        const uint32_t chunk = g & 1u;
        uint64_t r00, r10, r01, r11;
        if constexpr (BR) {
            const uint64_t bx = (xr >> 1) * 4u + (xr & 1u);
            const uint64_t ry0 = (y0 >> 1) * P.sy + (y0 & 1u) * 2u + bx;
            const uint64_t ry1 = (y1 >> 1) * P.sy + (y1 & 1u) * 2u + bx;
            r00 = z0 * P.sz + ry0; r10 = z0 * P.sz + ry1;
            r01 = z1 * P.sz + ry0; r11 = z1 * P.sz + ry1;
        } else {
            r00 = z0 * P.sz + y0 * P.sy + xr; r10 = z0 * P.sz + y1 * P.sy + xr;
            r01 = z1 * P.sz + y0 * P.sy + xr; r11 = z1 * P.sz + y1 * P.sy + xr;
        }
        L[0] = reinterpret_cast<const float4 *>(vol + r00 * 8)[chunk];
        L[1] = reinterpret_cast<const float4 *>(vol + r10 * 8)[chunk];
        L[2] = reinterpret_cast<const float4 *>(vol + r01 * 8)[chunk];
        L[3] = reinterpret_cast<const float4 *>(vol + r11 * 8)[chunk];
    }
    return live;
}

template <int K>
__device__ __forceinline__ float qbcast(float v) {
    return qperm<K == 0 ? kQ0 : K == 1 ? kQ1 : K == 2 ? kQ2 : kQ3>(v);
}

template <int G, bool BR>
__device__ __forceinline__ float m7q_group(const float *__restrict__ vol, const Params &P,
                                           bool refresh_any, int refresh_bits, float xd, float yd,
                                           float zd, const CellPacked &fn, bool &ln, uint32_t g,
                                           float4 (&L)[4], float (&mz)[2]) {
    const bool odd = g & 1u;
    float r0[8], r1[8];
    pair_swap(L[0], L[1], odd, r0);  // corner (x = g>>1, y = g&1) at z0
    pair_swap(L[2], L[3], odd, r1);  //                              at z1
    ln = qc_gather_cell<G, BR>(vol, P, fn, g, L);
    if (refresh_any && ((refresh_bits >> G) & 1)) {  // ray G left its cell: its new means
        mz[0] = raw_mean<8>(r0);
        mz[1] = raw_mean<8>(r1);
    }
    // ray G's 8 corner means on every lane: lane 0 (x0,y0), 1 (x0,y1), 2 (x1,y0), 3 (x1,y1)
    const float fxd = __int_as_float(bcast_g<G>(__float_as_int(xd)));
    const float fyd = __int_as_float(bcast_g<G>(__float_as_int(yd)));
    const float fzd = __int_as_float(bcast_g<G>(__float_as_int(zd)));
    float mn[8];
    mn[0] = qbcast<0>(mz[0]); mn[2] = qbcast<1>(mz[0]); mn[1] = qbcast<2>(mz[0]); mn[3] = qbcast<3>(mz[0]);
    mn[4] = qbcast<0>(mz[1]); mn[6] = qbcast<1>(mz[1]); mn[5] = qbcast<2>(mz[1]); mn[7] = qbcast<3>(mz[1]);
    const float m00 = (float)((double)mn[0] * (1.0 - (double)fxd) + (double)(mn[1] * fxd));
    const float m10 = (float)((double)mn[2] * (1.0 - (double)fxd) + (double)(mn[3] * fxd));
    const float m01 = (float)((double)mn[4] * (1.0 - (double)fxd) + (double)(mn[5] * fxd));
    const float m11 = (float)((double)mn[6] * (1.0 - (double)fxd) + (double)(mn[7] * fxd));
    const float m0 = (float)((double)m00 * (1.0 - (double)fyd) + (double)(m10 * fyd));
    const float m1 = (float)((double)m01 * (1.0 - (double)fyd) + (double)(m11 * fyd));
    return (float)((double)m0 * (1.0 - (double)fzd) + (double)(m1 * fzd));
}

template <bool BR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_QUAD_WAVES, 8))) void k_march_m7_quad(const float *__restrict__ vol, Params P) {
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;  // uniform per workgroup
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t q = lane >> 2, g = lane & 3u;
    const uint32_t lx = wave * 16u + q, ly = g;  // 16x4 block per wave, quad = a column
    const uint32_t x = (tile % P.tiles_x) * kTileW + lx;
    const uint32_t y = (tile / P.tiles_x) * kTileH + ly;
    const bool valid = x < P.CW && y < P.CH;
    const uint64_t o = P.tile_list ? (uint64_t)slot * 256u + ly * kTileW + lx
                                   : (uint64_t)y * P.W + x;
    Ray r;
    bool alive = valid && make_ray(P, x, y, r);
    const bool hit = alive;
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = r.tnear;
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
    int n = 0;
    // the home ray's cell (K:320-352): the first sample always takes its means
    // from the records gathered here (the one-lane march's initial refresh)
    M7Cell cur = m7_cell(P, px, py, pz);
    bool first = true;
    float4 L0[4], L1[4], L2[4], L3[4];
    float mz0[2] = {0.f, 0.f}, mz1[2] = {0.f, 0.f}, mz2[2] = {0.f, 0.f}, mz3[2] = {0.f, 0.f};
    const CellPacked fc = pack_cell(P, cur, alive);
    bool lc[4];
    lc[0] = qc_gather_cell<0, BR>(vol, P, fc, g, L0);
    lc[1] = qc_gather_cell<1, BR>(vol, P, fc, g, L1);
    lc[2] = qc_gather_cell<2, BR>(vol, P, fc, g, L2);
    lc[3] = qc_gather_cell<3, BR>(vol, P, fc, g, L3);
    for (int i = 0; i < kMaxSteps; i++) {
        if (!wave_any(alive)) break;
        // the home ray at its current sample: refresh due? (its new cell's
        // records are the ones gathered for this position)
        const float qx = px * 0.5f + 0.5f, qy = py * 0.5f + 0.5f, qz = pz * 0.5f + 0.5f;
        bool refresh = false;
        if (alive) {
            refresh = first || qx < cur.fx || qy < cur.fy || qz < cur.fz || qx > cur.cx ||
                      qy > cur.cy || qz > cur.cz;
            if (refresh) cur = m7_cell(P, px, py, pz);
        }
        first = false;
        const float xd = (qx - cur.fx) / (cur.cx - cur.fx);
        const float yd = (qy - cur.fy) / (cur.cy - cur.fy);
        const float zd = (qz - cur.fz) / (cur.cz - cur.fz);
        const float tn = t + kTStep;                                        // K:701
        const bool cont = alive && !(tn > r.tfar) && (i + 1 < kMaxSteps);  // K:703, 381
        const float nx = px + stx, ny = py + sty, nz = pz + stz;            // K:706
        const CellPacked fn = pack_cell(P, m7_cell(P, nx, ny, nz), cont);
        // refresh flags of the quad's 4 rays, bit G = ray (G, q)
        const int rb = refresh ? 1 << g : 0;
        const int rbits = qpermi<kQ0>(rb) | qpermi<kQ1>(rb) | qpermi<kQ2>(rb) | qpermi<kQ3>(rb);
        const bool rany = rbits != 0;
        bool ln[4];
        const float b0 = m7q_group<0, BR>(vol, P, rany, rbits, xd, yd, zd, fn, ln[0], g, L0, mz0);
        const float b1 = m7q_group<1, BR>(vol, P, rany, rbits, xd, yd, zd, fn, ln[1], g, L1, mz1);
        const float b2 = m7q_group<2, BR>(vol, P, rany, rbits, xd, yd, zd, fn, ln[2], g, L2, mz2);
        const float b3 = m7q_group<3, BR>(vol, P, rany, rbits, xd, yd, zd, fn, ln[3], g, L3, mz3);
        const float im = g == 0 ? b0 : (g == 1 ? b1 : (g == 2 ? b2 : b3));
        if (alive) {
            n = i + 1;
            if (composite(P, im * 50.0f, sx, sy, sz, sw) || !cont) {  // K:479, K:698
                alive = false;
            } else {
                t = tn;
                px = nx;
                py = ny;
                pz = nz;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) lc[k] = ln[k];
    }
    (void)lc;
    if (!valid) return;
    if (!hit) {
        write_miss(P, o);
        return;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
}

// ---- method 7: software trilinear of corner means, K:320-367, 395-480 ----
struct M7 {
    float fx, fy, fz, cx, cy, cz;  // interPos[0] and interPos[7]
    float mean[8];
};

// the corner mean of one record (K:347-367); BK: the record is the corner mean
// itself, baked by basicDataProcessing (plane 3, vr_stats.hip; B = 1)
template <int B, bool BK>
__device__ __forceinline__ float m7_rec_mean(const float (&rec)[B]) {
    if constexpr (BK) {
        static_assert(B == 1, "baked corner means are one float per voxel");
        return rec[0];
    } else {
        return raw_mean<B>(rec);
    }
}

template <int B, bool BK = false>
__device__ __forceinline__ float corner_mean(const float *__restrict__ vol, const Params &P,
                                             float ux, float uy, float uz) {
    const int ix = point_axis(ux, P.nx), iy = point_axis(uy, P.ny), iz = point_axis(uz, P.nz);
    // BK: the baked plane's 16 x 2 x 1 bricks (plane_index, P.sy / P.sz its pitches)
    const uint64_t vidx = BK ? plane_index((uint32_t)ix, (uint32_t)iy, (uint32_t)iz, P.sy, P.sz)
                             : (uint64_t)iz * P.sz + (uint64_t)iy * P.sy + (uint64_t)ix;
    if constexpr (B > 0) {
        float rec[B];
        load_rec<B>(vol, vidx, rec);
        return m7_rec_mean<B, BK>(rec);
    } else {
        return raw_mean_rt(vol + vidx * (uint64_t)P.nb, P.nb);
    }
}

template <int B, bool BK = false>
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
        m.mean[j] = corner_mean<B, BK>(vol, P, (j & 1) ? m.cx : m.fx, (j & 2) ? m.cy : m.fy,
                                       (j & 4) ? m.cz : m.fz);
}

// ---- method 7, software-pipelined (B <= 8) ----
// The corner cache of K:320-367 / 395-480 refreshes when a sample leaves the
// cell [interPos[0], interPos[7]] (inInterpolation, K:253-270).  At 1024^3 a
// step of 0.01 crosses ~5 voxels, so nearly every step refreshes and the march
// is a chain of dependent 8-record gathers, like methods 1/2.  Here the 8
// corner records of the NEXT position's cell are gathered before the current
// sample is blended (two register sets, unrolled by two, as march_pipe_tile).
// If the next sample stays inside the current cell, no refresh happens and
// the gathered records -- the same cell's, cache hits -- are discarded; if it
// leaves, the refresh at that position computes exactly that cell
// (floor/ceil of the same float position), so it decodes the gathered
// records.  Bit-identical to k_march_m7.
template <int B, bool BK = false>
__device__ __forceinline__ void m7_gather(const float *__restrict__ vol, const Params &P,
                                          const M7Cell &c, float (&rec)[8][B]) {
    const int x0 = point_axis(c.fx, P.nx), x1 = point_axis(c.cx, P.nx);
    const int y0 = point_axis(c.fy, P.ny), y1 = point_axis(c.cy, P.ny);
    const int z0 = point_axis(c.fz, P.nz), z1 = point_axis(c.cz, P.nz);
    const int xs[2] = {x0, x1}, ys[2] = {y0, y1}, zs[2] = {z0, z1};
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint32_t x = (uint32_t)xs[j & 1], y = (uint32_t)ys[(j >> 1) & 1],
                       z = (uint32_t)zs[j >> 2];
        load_rec<B>(vol, BK ? plane_index(x, y, z, P.sy, P.sz)
                            : (uint64_t)z * P.sz + (uint64_t)y * P.sy + x, rec[j]);
    }
}

#ifndef VR_M7_PIPE_MAXWAVES
#define VR_M7_PIPE_MAXWAVES 8
#endif
template <int B, bool BK = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, VR_M7_PIPE_MAXWAVES))) void k_march_m7_pipe(const float *__restrict__ vol, Params P) {
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;
    uint32_t lx, ly;
    lane_pixel(P, threadIdx.x, lx, ly);
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
    M7Cell cur = m7_cell(P, px, py, pz), ca, cb;  // K:320-352 at the first sample
    float mean[8];
    float ra[8][B], rb[8][B];
    m7_gather<B, BK>(vol, P, cur, ra);
#pragma unroll
    for (int j = 0; j < 8; j++) mean[j] = m7_rec_mean<B, BK>(ra[j]);
    ca = cur;
    int n = 0;
    bool alive = true;
    // one step: sample at (px, py, pz) with the cell whose records are (cc, rc)
    // if a refresh is due; gather the next position's cell into (cn, rn)
    auto step = [&](int i, const M7Cell &cc, const float (&rc)[8][B], M7Cell &cn,
                    float (&rn)[8][B]) {
        const float qx = px * 0.5f + 0.5f, qy = py * 0.5f + 0.5f, qz = pz * 0.5f + 0.5f;
        if (qx < cur.fx || qy < cur.fy || qz < cur.fz || qx > cur.cx || qy > cur.cy ||
            qz > cur.cz) {  // inInterpolation, K:253-270, 396: refresh from (cc, rc)
            cur = cc;
#pragma unroll
            for (int j = 0; j < 8; j++) mean[j] = m7_rec_mean<B, BK>(rc[j]);
        }
        const float tn = t + kTStep;                                 // K:701
        const bool cont = !(tn > r.tfar) && (i + 1 < kMaxSteps);    // K:703, K:381
        const float nx = px + stx, ny = py + sty, nz = pz + stz;    // K:706
        cn = m7_cell(P, nx, ny, nz);
        m7_gather<B, BK>(vol, P, cn, rn);
        const float xd = (px * 0.5f + 0.5f - cur.fx) / (cur.cx - cur.fx);
        const float yd = (py * 0.5f + 0.5f - cur.fy) / (cur.cy - cur.fy);
        const float zd = (pz * 0.5f + 0.5f - cur.fz) / (cur.cz - cur.fz);
        const float m00 = (float)((double)mean[0] * (1.0 - (double)xd) + (double)(mean[1] * xd));
        const float m10 = (float)((double)mean[2] * (1.0 - (double)xd) + (double)(mean[3] * xd));
        const float m01 = (float)((double)mean[4] * (1.0 - (double)xd) + (double)(mean[5] * xd));
        const float m11 = (float)((double)mean[6] * (1.0 - (double)xd) + (double)(mean[7] * xd));
        const float m0 = (float)((double)m00 * (1.0 - (double)yd) + (double)(m10 * yd));
        const float m1 = (float)((double)m01 * (1.0 - (double)yd) + (double)(m11 * yd));
        const float im = (float)((double)m0 * (1.0 - (double)zd) + (double)(m1 * zd));
        n = i + 1;
        if (composite(P, im * 50.0f, sx, sy, sz, sw) || !cont) {    // K:479, K:698
            alive = false;
        } else {
            t = tn;
            px = nx;
            py = ny;
            pz = nz;
        }
    };
    for (int i = 0; i < kMaxSteps; i += 2) {
        step(i, ca, ra, cb, rb);
        if (!alive) break;
        step(i + 1, cb, rb, ca, ra);
        if (!alive) break;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
}

template <int B, bool BK = false>
__global__ __launch_bounds__(256) void k_march_m7(const float *__restrict__ vol, Params P) {
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;
    uint32_t lx, ly;
    lane_pixel(P, threadIdx.x, lx, ly);
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
    M7 m;
    m7_refresh<B, BK>(vol, P, px, py, pz, m);
    int n = 0;
    for (int i = 0; i < kMaxSteps; i++) {
        const float qx = px * 0.5f + 0.5f, qy = py * 0.5f + 0.5f, qz = pz * 0.5f + 0.5f;
        if (qx < m.fx || qy < m.fy || qz < m.fz || qx > m.cx || qy > m.cy || qz > m.cz)
            m7_refresh<B, BK>(vol, P, px, py, pz, m);  // inInterpolation, K:253-270, 396
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

// ---- method 7 for wide records (B = 16, 32), quad-cooperative refreshes ----
// k_march_m7's refresh gathers 8 lane-owned records (texture-address-bound at
// B = 32, as k_march_wide).  Here a refresh loads the 8 corner records of the
// quad rays that need one with the quad gathers and DPP transpose of
// k_march_wq (corner batches of 64 / B records double-buffered), then each
// lane decodes its own corners' means (K:347-367).  The loop is wave-uniform;
// cell test, lerps and composite are k_march_m7's.
struct QuadCell {
    int x[4], y[4], z[4], nd[4];  // per quad ray: floor | ceil << 16 per axis; refresh flag
};

template <int B>
__device__ __forceinline__ void m7q_gather(const float *__restrict__ vol, const Params &P,
                                           const QuadCell &q, int j, uint32_t g,
                                           float4 (&M)[B / 16][4]) {
#pragma unroll
    for (int R = 0; R < 4; R++) {
        if (q.nd[R]) {
            const uint32_t ax = (uint32_t)q.x[R], ay = (uint32_t)q.y[R], az = (uint32_t)q.z[R];
            const uint64_t x = (j & 1) ? (ax >> 16) : (ax & 0xFFFFu);
            const uint64_t y = (j & 2) ? (ay >> 16) : (ay & 0xFFFFu);
            const uint64_t z = (j & 4) ? (az >> 16) : (az & 0xFFFFu);
            const float4 *rec =
                reinterpret_cast<const float4 *>(vol + (z * P.sz + y * P.sy + x) * (uint64_t)B);
#pragma unroll
            for (int s = 0; s < B / 16; s++) M[s][R] = rec[4 * s + g];
        }
    }
}

// transpose a gathered corner and return this lane's record's undivided mean
template <int B>
__device__ __forceinline__ float m7q_decode(float4 (&Mc)[B / 16][4], uint32_t g, bool need) {
#pragma unroll
    for (int s = 0; s < B / 16; s++) quad_transpose(Mc[s], g);
    float mean = 0.0f;
    if (need) {
        float p[B];
#pragma unroll
        for (int s = 0; s < B / 16; s++)
#pragma unroll
            for (int c = 0; c < 4; c++) {
                p[16 * s + 4 * c + 0] = Mc[s][c].x;
                p[16 * s + 4 * c + 1] = Mc[s][c].y;
                p[16 * s + 4 * c + 2] = Mc[s][c].z;
                p[16 * s + 4 * c + 3] = Mc[s][c].w;
            }
        mean = raw_mean<B>(p);
    }
    return mean;
}

// corner batches K (in A) and K + 1 (in Bf) of one refresh; the batch after
// K + 1 (if any) is gathered into A while K + 1 decodes
template <int B, int K>
__device__ __forceinline__ void m7q_pair(const float *__restrict__ vol, const Params &P,
                                         const QuadCell &q, uint32_t g, bool need,
                                         float4 (&A)[64 / B][B / 16][4],
                                         float4 (&Bf)[64 / B][B / 16][4], float (&mn)[8]) {
    constexpr int CG = 64 / B, NB = 8 / CG;
#pragma unroll
    for (int c = 0; c < CG; c++) m7q_gather<B>(vol, P, q, (K + 1) * CG + c, g, Bf[c]);
#pragma unroll
    for (int c = 0; c < CG; c++) {
        const float v = m7q_decode<B>(A[c], g, need);
        if (need) mn[K * CG + c] = v;
    }
    if constexpr (K + 2 < NB) {
#pragma unroll
        for (int c = 0; c < CG; c++) m7q_gather<B>(vol, P, q, (K + 2) * CG + c, g, A[c]);
    }
#pragma unroll
    for (int c = 0; c < CG; c++) {
        const float v = m7q_decode<B>(Bf[c], g, need);
        if (need) mn[(K + 1) * CG + c] = v;
    }
}

template <int B>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_WIDE_MINW, VR_WIDE_WAVES))) void k_march_m7wq(const float *__restrict__ vol, Params P) {
    constexpr int CG = 64 / B, NB = 8 / CG;
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;
    uint32_t lx, ly;
    if (P.wq_map) {  // a wave takes a 16x4 block, a quad one pixel column (k_march_wq)
        lx = (threadIdx.x >> 6) * 16u + ((threadIdx.x & 63u) >> 2);
        ly = threadIdx.x & 3u;
    } else {
        tile_pixel(threadIdx.x, lx, ly);
    }
    const uint32_t x = (tile % P.tiles_x) * kTileW + lx;
    const uint32_t y = (tile / P.tiles_x) * kTileH + ly;
    const bool valid = x < P.CW && y < P.CH;
    const uint64_t o = P.tile_list ? (uint64_t)slot * 256u + ly * kTileW + lx
                                   : (uint64_t)y * P.W + x;
    const uint32_t g = threadIdx.x & 3u;
    // every lane stays to the end: the quads exchange records at every refresh
    Ray r = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    bool alive = valid && make_ray(P, x, y, r);
    const bool hit = alive;
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = r.tnear;
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
    M7 m = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f}};
    int n = 0;
    for (int i = 0; i < kMaxSteps; i++) {
        if (!wave_any(alive)) break;
        const float qx = px * 0.5f + 0.5f, qy = py * 0.5f + 0.5f, qz = pz * 0.5f + 0.5f;
        // the first sample fills the cache (K:320-367), later ones refresh on
        // leaving the cell (inInterpolation, K:253-270, 396)
        const bool need = alive && (i == 0 || qx < m.fx || qy < m.fy || qz < m.fz ||
                                    qx > m.cx || qy > m.cy || qz > m.cz);
        if (wave_any(need)) {
            if (need) {  // m7_refresh's cell bounds
                m.fx = floorf(qx * (float)P.m7x) / (float)P.m7x;
                m.cx = ceilf(qx * (float)P.m7x) / (float)P.m7x;
                m.fy = floorf(qy * (float)P.m7y) / (float)P.m7y;
                m.cy = ceilf(qy * (float)P.m7y) / (float)P.m7y;
                m.fz = floorf(qz * (float)P.m7z) / (float)P.m7z;
                m.cz = ceilf(qz * (float)P.m7z) / (float)P.m7z;
            }
            // corner voxels (corner_mean's point_axis), broadcast over the quad
            const int cx = point_axis(m.fx, P.nx) | (point_axis(m.cx, P.nx) << 16);
            const int cy = point_axis(m.fy, P.ny) | (point_axis(m.cy, P.ny) << 16);
            const int cz = point_axis(m.fz, P.nz) | (point_axis(m.cz, P.nz) << 16);
            const int nd = need ? 1 : 0;
            QuadCell q;
            q.x[0] = bcast_g<0>(cx); q.y[0] = bcast_g<0>(cy); q.z[0] = bcast_g<0>(cz); q.nd[0] = bcast_g<0>(nd);
            q.x[1] = bcast_g<1>(cx); q.y[1] = bcast_g<1>(cy); q.z[1] = bcast_g<1>(cz); q.nd[1] = bcast_g<1>(nd);
            q.x[2] = bcast_g<2>(cx); q.y[2] = bcast_g<2>(cy); q.z[2] = bcast_g<2>(cz); q.nd[2] = bcast_g<2>(nd);
            q.x[3] = bcast_g<3>(cx); q.y[3] = bcast_g<3>(cy); q.z[3] = bcast_g<3>(cz); q.nd[3] = bcast_g<3>(nd);
            float4 A[CG][B / 16][4], Bf[CG][B / 16][4];
#pragma unroll
            for (int c = 0; c < CG; c++) m7q_gather<B>(vol, P, q, c, g, A[c]);
            m7q_pair<B, 0>(vol, P, q, g, need, A, Bf, m.mean);
            if constexpr (NB == 4) m7q_pair<B, 2>(vol, P, q, g, need, A, Bf, m.mean);
        }
        if (alive) {
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
            n = i + 1;
            if (composite(P, im * 50.0f, sx, sy, sz, sw)) {  // K:479
                alive = false;
            } else {
                t = t + kTStep;
                if (t > r.tfar) {
                    alive = false;
                } else {
                    px = px + stx;
                    py = py + sty;
                    pz = pz + stz;
                }
            }
        }
    }
    if (!valid) return;
    if (!hit) {
        write_miss(P, o);
        return;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
}

// ------------------------------ launcher ----------------------------------

template <int B>
static hipError_t march_m7_b(int method, const float *vol, const Params &P, uint32_t nslots,
                             hipStream_t s) {
    const dim3 grid(nslots), block(256);
    if (method == -7) {  // method 7 over the baked corner means (plane 3, vr_stats.hip)
        if constexpr (B == 1) {
            // 4-byte corners: the plain march (the look-ahead gather of
            // k_march_m7_pipe only adds loads), 4 workgroups per CU on row-aligned
            // views, 2 on oblique ones (1024^3 C0 0.68 -> 0.64 ms, C1 2.03 -> 1.67;
            // profiles/r02/baked_m7.log)
            note_kernel("k_march_m7", B, method);
            hipLaunchKernelGGL((k_march_m7<1, true>), grid, block,
                               cap_lds(P, P.wg_per_cu > 0 ? P.wg_per_cu : (P.oblique ? 2 : 4)), s,
                               vol, P);
            return hipGetLastError();
        }
        return hipErrorInvalidValue;
    }
    if (method != 7) return hipErrorInvalidValue;
    if constexpr (B == 8) {
        // oblique views with the method-7 grid equal to the volume: the
        // quad-cooperative march (VR_M7_QUAD=0 disables), 2 workgroups per CU
        const char *eq = tuning("VR_M7_QUAD");
        const bool quad = !(eq && std::atoi(eq) == 0);
        if (quad && P.oblique && P.m7x == P.nx && P.m7y == P.ny && P.m7z == P.nz) {
            const size_t qlds = cap_lds(P, P.wg_per_cu > 0 ? P.wg_per_cu : 2);
            if (P.bvol) {
                note_kernel("k_march_m7_quad_brick", B, method);
                Params Q = P;
                Q.sy = P.bsy;
                Q.sz = P.bsz;
                hipLaunchKernelGGL(k_march_m7_quad<true>, grid, block, qlds, s, P.bvol, Q);
            } else {
                note_kernel("k_march_m7_quad", B, method);
                hipLaunchKernelGGL(k_march_m7_quad<false>, grid, block, qlds, s, vol, P);
            }
            return hipGetLastError();
        }
    }
    if constexpr (B == 16 || B == 32) {
        // wide records: quad-cooperative refreshes (VR_M7_WQ=0: k_march_m7)
        const char *eq = tuning("VR_M7_WQ");
        if (!(eq && std::atoi(eq) == 0)) {
            note_kernel("k_march_m7wq", B, method);
            Params Q = P;
            Q.wq_map = M7_WQ_MAP;
            if (const char *em = tuning("VR_WQ_MAP")) Q.wq_map = std::atoi(em) != 0;
            hipLaunchKernelGGL((k_march_m7wq<B>), grid, block, occupancy_lds(P), s, vol, Q);
            return hipGetLastError();
        }
    }
    if constexpr (B > 0 && B <= 8) {
        // pipelined corner gathers (VR_M7_PIPE=0: the plain march); oblique views
        // at 2 workgroups per CU (1024^3x8 C1: 8.53 -> 7.45 ms; C0 is fastest
        // uncapped, 1.53 ms; profiles/r02/m7_pipe.log)
        const char *ep = tuning("VR_M7_PIPE");
        if (!(ep && std::atoi(ep) == 0)) {
            note_kernel("k_march_m7_pipe", B, method);
            hipLaunchKernelGGL((k_march_m7_pipe<B>), grid, block,
                               cap_lds(P, P.wg_per_cu > 0 ? P.wg_per_cu
                                                          : (P.oblique && B == 8 ? 2 : 0)),
                               s, vol, P);
            return hipGetLastError();
        }
    }
    // oblique views at 3 workgroups per CU when B = 8 (the measured case): fewer
    // corner-mean refreshes in flight, fewer L2 re-reads (1024^3x8 C1 9.94 ->
    // 8.29 ms; row-aligned C0 is fastest uncapped)
    note_kernel("k_march_m7", B, method);
    hipLaunchKernelGGL((k_march_m7<B>), grid, block,
                       cap_lds(P, P.wg_per_cu > 0 ? P.wg_per_cu : (P.oblique && B == 8 ? 3 : 0)),
                       s, vol, P);
    return hipGetLastError();
}

hipError_t launch_march_m7(int nb, int method, const float *vol, const Params &P0,
                           uint32_t nslots, hipStream_t s) {
    if (nslots == 0) return hipSuccess;
    // the one-lane method-7 marches (k_march_m7_pipe / k_march_m7): a 16x4 pixel
    // block per wave, except 8+-bin row-aligned views of a fine volume (< 4 pixels
    // per voxel of the x-y face), which keep 64-pixel rows: 256^3 x 4 at 512^2 C0
    // 0.322 -> 0.222 ms, C1 0.201 -> 0.175; 512^3 x 8 1080p C0 1.201 -> 1.125;
    // 1024^3 x 4 C0 0.795 -> 0.775, C1 2.67 -> 2.39; 1024^3 x 8 C0 1.447 vs 1.468
    // (rows; profiles/r06/segmap/m7_*.log).  VR_M7_MAP=0/1 overrides.
    Params P = P0;
    P.seg_map = !(nb >= 8 && !P.oblique &&
                  (uint64_t)P.CW * P.CH < 4ull * (uint64_t)P.nx * (uint64_t)P.ny);
    if (const char *e = tuning("VR_M7_MAP")) P.seg_map = std::atoi(e) != 0;
    switch (nb) {
    case 1: return march_m7_b<1>(method, vol, P, nslots, s);
    case 2: return march_m7_b<2>(method, vol, P, nslots, s);
    case 4: return march_m7_b<4>(method, vol, P, nslots, s);
    case 8: return march_m7_b<8>(method, vol, P, nslots, s);
    case 16: return march_m7_b<16>(method, vol, P, nslots, s);
    case 32: return march_m7_b<32>(method, vol, P, nslots, s);
    default: return march_m7_b<0>(method, vol, P, nslots, s);
    }
}

}  // namespace vr
