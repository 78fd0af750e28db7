// vr_kernels.hip -- gfx950 marches of methods 1/2/3 (the d_render path,
// K:272-717) and the kernel choice between them (march_b).  One 64x4-pixel
// tile per 256-thread workgroup, XCD-aware tile order; per step the statistic
// is decoded from the 8 corner distribution records and blended with the
// texture unit's 8-bit filter weights.
//
//  k_march_pipe<B,M,GM>  one lane per ray, next step's 8 corners gathered
//                        while this one decodes (row-aligned views, B <= 8)
//  k_march<B,M,COUNT>    the wave's footprint box staged in LDS, every voxel
//                        decoded once per wave-step (coarse volumes, entropy);
//                        COUNT: the footprint-marking pass that counts U
//  k_march_duo<B,M,K>    the same box for K consecutive samples per lane
//  k_march_ws<B,M>       wave-staged exact footprint (entropy, 1-4 bins)
//  k_march_quad(2)<M,BR> quad-cooperative 64-B x-pair gathers (oblique, B = 8)
//  k_march_wide / _wq    16- and 32-bin records
//  k_synth, k_unscatter, k_popcount, k_logcheck
// Methods 7 and 4/5/6: vr_m7.hip, vr_codec.hip; ray-segmented marches:
// vr_seg.hip.  K = volumeRender_kernel.cu of the reference.
#include "vr_device.h"
#include "vr_internal.h"
#include "vr_march.h"
#include "vr_quad.h"

#include <algorithm>
#include <cstdlib>
#include <cstdio>

namespace vr {


static char g_last_kernel[64] = "";

void note_kernel(const char *kind, int B, int method) {
    snprintf(g_last_kernel, sizeof g_last_kernel, "%s<B=%d,M=%d>", kind, B, method);
}

const char *last_march_kernel() { return g_last_kernel; }





// the statistic of a record in the box / direct paths of k_march: wide entropy
// through the LDS column (st: this wave's, 64 * B floats), everything else as
// record_stat
template <int B, int M>
__device__ __forceinline__ float box_stat(const float (&p)[B], const Params &P, float *st,
                                          uint32_t lane, const LogEnt *tab) {
    if constexpr (M == 3 && B >= 8) {
        if (st) return entropy_stash<B>(p, st, lane, P.enorm, tab);
    }
    return record_stat<B, M>(p, P.enorm);  // (callers without an LDS column: k_march_ws's direct path)
}

// Compile-time tuning knob (tools/build_variants.sh builds sweeps of it).
#ifndef VR_BOX_G
#define VR_BOX_G 4          // box voxels per lane in flight, staged path
#endif

// Direct path: each lane gathers and decodes its own 8 corner records, up to
// min(64 / B, CGMAX) of them in flight.
template <int B, int M, int CGMAX = 8>
__device__ __forceinline__ float sample_direct(const float *__restrict__ vol, const Params &P,
                                               const Foot &f, const LogEnt *tab = nullptr,
                                               float *st = nullptr) {
    const uint64_t r00 = (uint64_t)f.z0 * P.sz + (uint64_t)f.y0 * P.sy;
    const uint64_t r10 = (uint64_t)f.z0 * P.sz + (uint64_t)f.y1 * P.sy;
    const uint64_t r01 = (uint64_t)f.z1 * P.sz + (uint64_t)f.y0 * P.sy;
    const uint64_t r11 = (uint64_t)f.z1 * P.sz + (uint64_t)f.y1 * P.sy;
    const uint64_t vidx[8] = {r00 + f.x0, r00 + f.x1, r10 + f.x0, r10 + f.x1,
                              r01 + f.x0, r01 + f.x1, r11 + f.x0, r11 + f.x1};
    float s[8];
    if constexpr (B > 0) {
        constexpr int CG0 = (B >= 64) ? 1 : ((64 / B) > 8 ? 8 : (64 / B));
        constexpr int CG = CG0 < CGMAX ? CG0 : CGMAX;
#pragma unroll
        for (int g = 0; g < 8; g += CG) {
            float rec[CG][B];
#pragma unroll
            for (int j = 0; j < CG; j++) load_rec<B>(vol, vidx[g + j], rec[j]);
#pragma unroll
            for (int j = 0; j < CG; j++) s[g + j] = box_stat<B, M>(rec[j], P, st, threadIdx.x & 63u, tab);
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++)
            s[j] = record_stat_rt<M>(vol + vidx[j] * (uint64_t)P.nb, P.nb, P.enorm);
    }
    return blend8(s, f);
}


// NG groups of 64 box voxels from position p0: all NG loads issue before the
// first decode waits on them
template <int B, int M, int NG>
__device__ __forceinline__ void box_chunk(const float *__restrict__ vbase, const Params &P,
                                          float *box, int dx, int dxy, int V, uint32_t lane,
                                          int p0, float rdx, float rdxy, const LogEnt *tab,
                                          float *st) {
    const uint32_t sy = (uint32_t)P.sy;
    float rec[NG][B];
#pragma unroll
    for (int g = 0; g < NG; g++) {
        const int p = min(p0 + g * 64 + (int)lane, V - 1);
        const int z = (int)(((float)p + 0.5f) * rdxy);
        const int r = p - z * dxy;
        const int y = (int)(((float)r + 0.5f) * rdx);
        const int x = r - y * dx;
        const uint64_t off = (uint64_t)(uint32_t)z * P.sz + (uint32_t)(y * sy + x);
        if constexpr (B == 16 || B == 32) {
            // wide records: the quad loads its 4 lanes' records as contiguous
            // 64-B runs (lane q reads chunk 4s + q of each) and a DPP transpose
            // hands every lane its own (k_march_wq); lane-owned 64 / 128-B
            // records made every 16-B wave load touch ~64 lines
            const uint32_t q = lane & 3u;
            const uint32_t lo = (uint32_t)off, hi = (uint32_t)(off >> 32);
            float4 Mq[B / 16][4];
#pragma unroll
            for (int R = 0; R < 4; R++) {
                const uint32_t l = (uint32_t)(R == 0 ? bcast_g<0>((int)lo) : R == 1 ? bcast_g<1>((int)lo)
                                            : R == 2 ? bcast_g<2>((int)lo) : bcast_g<3>((int)lo));
                const uint32_t h = (uint32_t)(R == 0 ? bcast_g<0>((int)hi) : R == 1 ? bcast_g<1>((int)hi)
                                            : R == 2 ? bcast_g<2>((int)hi) : bcast_g<3>((int)hi));
                const float4 *src = reinterpret_cast<const float4 *>(
                    vbase + (((uint64_t)h << 32) | l) * (uint64_t)B);
#pragma unroll
                for (int c = 0; c < B / 16; c++) Mq[c][R] = src[4 * c + q];
            }
#pragma unroll
            for (int c = 0; c < B / 16; c++) {
                quad_transpose(Mq[c], q);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    rec[g][16 * c + 4 * k + 0] = Mq[c][k].x;
                    rec[g][16 * c + 4 * k + 1] = Mq[c][k].y;
                    rec[g][16 * c + 4 * k + 2] = Mq[c][k].z;
                    rec[g][16 * c + 4 * k + 3] = Mq[c][k].w;
                }
            }
        } else {
            load_rec<B>(vbase, off, rec[g]);
        }
    }
#pragma unroll
    for (int g = 0; g < NG; g++) {
        const int p = p0 + g * 64 + (int)lane;
        if (p < V) box[p] = box_stat<B, M>(rec[g], P, st, lane, tab);
    }
}

// Staged path: the wave's footprint box for this step (every voxel any active
// lane's 8 corners touch) is loaded with consecutive lanes on consecutive
// voxels of a box row (coalesced), each voxel's statistic is decoded ONCE and
// parked in the wave's LDS slice, then every lane blends its 8 corners from
// LDS.  Position p -> (x,y,z) in the box uses float reciprocals, exact for
// p < 2^11 (box_max <= 1024).  Positions past the box end are clamped to its
// last voxel so every load is unconditional: all of a chunk's loads issue
// back-to-back before the first decode waits on them.  A chunk takes only the
// 64-voxel groups the box still needs (wave-uniform): a 140-voxel box decodes
// 192 slots, not 256 (512^3 x 8 at 1080p: boxes of ~130-210 voxels).
template <int B, int M>
__device__ __forceinline__ void decode_box(const float *__restrict__ vbase, const Params &P,
                                           float *box, int dx, int dxy, int V, uint32_t lane,
                                           const LogEnt *tab, float *st) {
#ifdef VR_BOX_CHECK
    // decode counts of the frame: box voxels and lane slots (64 per group) decoded
    if (lane == 0 && P.box_check) {
        atomicAdd(P.box_check + 3, (unsigned long long)V);
        atomicAdd(P.box_check + 4, (unsigned long long)((V + 63) / 64 * 64));
    }
#endif
    constexpr int G0 = B >= 32 ? 1 : (B >= 16 ? 2 : 4);
    constexpr int G = G0 < VR_BOX_G ? G0 : VR_BOX_G;  // voxels per lane in flight
    // hardware reciprocals (1 ulp) instead of two IEEE divisions per wave-step:
    // (p + 0.5) / d lies at least 0.5 / d from an integer, a relative gap of
    // >= 2^-12 for p < 2^11, far above the reciprocal's 2^-22 error, so the
    // truncations below give the same box coordinates
    const float rdx = __builtin_amdgcn_rcpf((float)dx), rdxy = __builtin_amdgcn_rcpf((float)dxy);
    for (int p0 = 0; p0 < V; p0 += 64 * G) {
        const int left = V - p0;  // wave-uniform
        if (G >= 4 && left > 192)
            box_chunk<B, M, (G >= 4 ? 4 : 1)>(vbase, P, box, dx, dxy, V, lane, p0, rdx, rdxy, tab, st);
        else if (G >= 3 && left > 128)
            box_chunk<B, M, (G >= 3 ? 3 : 1)>(vbase, P, box, dx, dxy, V, lane, p0, rdx, rdxy, tab, st);
        else if (G >= 2 && left > 64)
            box_chunk<B, M, (G >= 2 ? 2 : 1)>(vbase, P, box, dx, dxy, V, lane, p0, rdx, rdxy, tab, st);
        else
            box_chunk<B, M, 1>(vbase, P, box, dx, dxy, V, lane, p0, rdx, rdxy, tab, st);
    }
}

#ifndef VR_MARCH_MINW
#define VR_MARCH_MINW 1   // minimum waves per SIMD the register allocation must allow
#endif

#ifdef VR_BOX_CHECK
// Tooling build (-DVR_BOX_CHECK, vr_debug_box_check): the staged reads' bounds.
// A lane's 8 corners must lie inside the wave's box, the largest box index it
// reads, ((z1 - bz0) dy + (y1 - by0)) dx + (x1 - bx0), below the box's dx dy dz
// voxels (those the decode wrote this step), and the box inside the volume.  A
// violating read is counted and skipped (its sample is 0), never performed.
// hi: the largest box index the lane reads, V: the voxels decoded this step
// (dx dy dz)
__device__ __forceinline__ bool box_ok(const Params &P, const Foot &f, int bx0, int by0, int bz0,
                                       int dx, int dy, int dz, int hi, int V) {
    const bool ok = f.x0 >= bx0 && f.y0 >= by0 && f.z0 >= bz0 && f.x1 >= f.x0 &&
                    f.y1 >= f.y0 && f.z1 >= f.z0 && f.x1 < bx0 + dx && f.y1 < by0 + dy &&
                    f.z1 < bz0 + dz && hi < V && V <= P.box_max;
    if (!ok && P.box_check) {
        atomicAdd(P.box_check, 1ull);
        const long long over = (long long)hi + 1 - (long long)V;
        if (over > 0) atomicMax(P.box_check + 1, (unsigned long long)over);
    }
    return ok;
}
// (wave-uniform) false = the box is not inside the volume: counted, and the
// step takes the direct path instead, whose corners footprint() clamps
__device__ __forceinline__ bool box_in_volume(const Params &P, int bx0, int by0, int bz0, int dx,
                                              int dy, int dz, uint32_t lane) {
    const bool in = bx0 >= 0 && by0 >= 0 && bz0 >= 0 && bx0 + dx <= P.nx &&
                    by0 + dy <= P.ny && bz0 + dz <= P.nz;
    if (!in && lane == 0 && P.box_check)
        atomicAdd(P.box_check + 2, (unsigned long long)(dx * dy * dz));
    return in;
}
#endif
template <int B, int M, bool COUNT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_MARCH_MINW, 8))) void k_march(const float *__restrict__ vol, Params P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;  // whole workgroup uniform
    // entropy (method 3) of 8 / 16 / 32-bin records: the exact logarithm through
    // the LDS table (logf_fast_tabp: no f64 division) and the rolled per-bin sum
    // over the lane's record column (entropy_stash), behind the box slices
    const LogEnt *tab = nullptr;
    float *st = nullptr;
    if constexpr (M == 3 && B >= 8) {
        LogEnt *t = reinterpret_cast<LogEnt *>(lds + 4u * (uint32_t)P.box_max);
        copy_logtab(t);
        __syncthreads();
        tab = t;
        // this wave's bin-major record column (entropy_stash) behind the table
        st = lds + 4u * (uint32_t)P.box_max + (uint32_t)kLogTabN * (sizeof(LogEnt) / 4u) + (threadIdx.x >> 6) * 64u * B;
    }
    const uint32_t lane = threadIdx.x & 63u;
    float *box = lds + (threadIdx.x >> 6) * (uint32_t)P.box_max;
    uint32_t lx, ly;
    if (P.wq_map) {  // a wave takes a 16x4 pixel block (a compact footprint box)
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
    // every lane stays to the end: the staged decode needs all 64 lanes
    Ray r;
    bool alive = valid && make_ray(P, x, y, r);
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = r.tnear;
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
    int n = 0;
    for (int i = 0; i < kMaxSteps; i++) {
        if (!wave_any(alive)) break;
        const Foot f = footprint(P, px, py, pz);
        if constexpr (COUNT) {
            if (alive) mark_foot(P, f);
        }
        float sample = 0.0f;
        bool staged = false;
        if constexpr (B > 0) {
            if (P.box_max > 0) {
                const int bx0 = wave_min(alive ? f.x0 : 0x7FFFFFFF);
                const int by0 = wave_min(alive ? f.y0 : 0x7FFFFFFF);
                const int bz0 = wave_min(alive ? f.z0 : 0x7FFFFFFF);
                // x1 = min(x0 + 1, n - 1) except at the low clamp, so this is a
                // (tight or one-voxel-larger) superset of the upper corners
                const int bx1 = min(wave_max(alive ? f.x0 : -1) + 1, P.nx - 1);
                const int by1 = min(wave_max(alive ? f.y0 : -1) + 1, P.ny - 1);
                const int bz1 = min(wave_max(alive ? f.z0 : -1) + 1, P.nz - 1);
                const int dx = bx1 - bx0 + 1, dy = by1 - by0 + 1, dz = bz1 - bz0 + 1;
#ifdef VR_BOX_CHECK
                if (dx * dy * dz <= P.box_max && box_in_volume(P, bx0, by0, bz0, dx, dy, dz, lane)) {
#else
                if (dx * dy * dz <= P.box_max) {  // wave-uniform
#endif
                    staged = true;
                    const int dxy = dx * dy;
                    const float *vbase =
                        vol + ((uint64_t)bz0 * P.sz + (uint64_t)by0 * P.sy + (uint64_t)bx0) *
                                  (uint64_t)B;
                    decode_box<B, M>(vbase, P, box, dx, dxy, dxy * dz, lane, tab, st);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#ifdef VR_BOX_CHECK
                    if (alive && box_ok(P, f, bx0, by0, bz0, dx, dy, dz,
                                        ((f.z1 - bz0) * dy + (f.y1 - by0)) * dx + (f.x1 - bx0),
                                        dx * dy * dz)) {
#else
                    if (alive) {
#endif
                        const int b0 = ((f.z0 - bz0) * dy + (f.y0 - by0)) * dx + (f.x0 - bx0);
                        const int ox = f.x1 - f.x0, oy = (f.y1 - f.y0) * dx;
                        const int oz = (f.z1 - f.z0) * dxy;
                        float s[8];
                        s[0] = box[b0];
                        s[1] = box[b0 + ox];
                        s[2] = box[b0 + oy];
                        s[3] = box[b0 + oy + ox];
                        s[4] = box[b0 + oz];
                        s[5] = box[b0 + oz + ox];
                        s[6] = box[b0 + oz + oy];
                        s[7] = box[b0 + oz + oy + ox];
                        sample = blend8(s, f);
                    }
                    // the slice is rewritten next step: keep these reads ahead of it
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
            }
        }
        if (alive) {
            if (!staged) sample = sample_direct<B, M>(vol, P, f, tab, st);
            n = i + 1;
            if (composite(P, sample, sx, sy, sz, sw)) {
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
    if (n == 0) {  // miss (K:302-303): nothing written
        write_miss(P, o);
        return;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
}


// ---- the LDS-box march, two samples per box (k_march_duo) ----
// k_march decodes a footprint box for every sample; on coarse volumes (512^3 x
// 8 at 1080p: ~4 rays per voxel, ~70 box voxels per wave-step) most of a
// wave-step is the box's fixed cost -- six wave reductions, the box set-up,
// the barriers -- not the decode.  Here one box covers a sample and the next
// one of every lane (the union of both footprints; the next one only where the
// ray reaches it by tfar, K:700-705), so those costs are paid once per two
// samples.  The samples and their compositing are those of k_march in the same
// order (positions advanced by the same float adds; a ray that terminates on the
// first sample leaves the second unread): the frame is bit-identical.  Mean and
// variance only: the entropy's duo instance lost to k_march<B, 3>.
template <int B, int M, int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_MARCH_MINW, 8))) void k_march_duo(const float *__restrict__ vol, Params P) {
    static_assert(M >= 1 && M <= 2, "mean, variance");
    static_assert(K >= 2 && K <= 4, "samples per box");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;  // whole workgroup uniform
    const LogEnt *tab = nullptr;  // (mean / variance: no log table, no record columns)
    float *st = nullptr;
    const uint32_t lane = threadIdx.x & 63u;
    float *box = lds + (threadIdx.x >> 6) * (uint32_t)P.box_max;
    uint32_t lx, ly;
    if (P.wq_map) {
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
    Ray r;
    bool alive = valid && make_ray(P, x, y, r);
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = r.tnear;
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
    int n = 0;
    for (int i = 0; i < kMaxSteps; i += K) {
        if (!wave_any(alive)) break;
        // this sample's footprint and those of the next K - 1 the one-sample loop
        // would take if none ends the ray (same float adds; K:700-705)
        Foot f[K];
        f[0] = footprint(P, px, py, pz);
        int lo_x = alive ? f[0].x0 : 0x7FFFFFFF, lo_y = alive ? f[0].y0 : 0x7FFFFFFF;
        int lo_z = alive ? f[0].z0 : 0x7FFFFFFF;
        int hi_x = alive ? -f[0].x0 : 0x7FFFFFFF, hi_y = alive ? -f[0].y0 : 0x7FFFFFFF;
        int hi_z = alive ? -f[0].z0 : 0x7FFFFFFF;
        {
            bool reach = alive;
            float tq = t, qx = px, qy = py, qz = pz;
#pragma unroll
            for (int k = 1; k < K; k++) {
                tq = tq + kTStep;
                reach = reach && !(tq > r.tfar) && i + k < kMaxSteps;
                qx = qx + stx;
                qy = qy + sty;
                qz = qz + stz;
                f[k] = footprint(P, qx, qy, qz);
                if (reach) {
                    lo_x = min(lo_x, f[k].x0);
                    lo_y = min(lo_y, f[k].y0);
                    lo_z = min(lo_z, f[k].z0);
                    hi_x = min(hi_x, -f[k].x0);
                    hi_y = min(hi_y, -f[k].y0);
                    hi_z = min(hi_z, -f[k].z0);
                }
            }
        }
        dpp_min3(lo_x, lo_y, lo_z);
        dpp_min3(hi_x, hi_y, hi_z);
        const int bx0 = lo_x, by0 = lo_y, bz0 = lo_z;
        // x1 = min(x0 + 1, n - 1) except at the low clamp: a superset of the upper corners
        const int bx1 = min(-hi_x + 1, P.nx - 1);
        const int by1 = min(-hi_y + 1, P.ny - 1);
        const int bz1 = min(-hi_z + 1, P.nz - 1);
        const int dx = bx1 - bx0 + 1, dy = by1 - by0 + 1, dz = bz1 - bz0 + 1;
        const int dxy = dx * dy;
        const int V = dxy * dz;
#ifdef VR_BOX_CHECK
        const bool staged = V <= P.box_max && box_in_volume(P, bx0, by0, bz0, dx, dy, dz, lane);
#else
        const bool staged = V <= P.box_max;  // wave-uniform
#endif
        if (staged) {
            const float *vbase =
                vol + ((uint64_t)bz0 * P.sz + (uint64_t)by0 * P.sy + (uint64_t)bx0) * (uint64_t)B;
            decode_box<B, M>(vbase, P, box, dx, dxy, V, lane, tab, st);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            // alive here: the ray reached this sample (t <= tfar), so f[k] is in the box
            if (alive) {
                const Foot &fk = f[k];
                float sample = 0.0f;
                const int b0 = ((fk.z0 - bz0) * dy + (fk.y0 - by0)) * dx + (fk.x0 - bx0);
                const int ox = fk.x1 - fk.x0, oy = (fk.y1 - fk.y0) * dx;
                const int oz = (fk.z1 - fk.z0) * dxy;
#ifdef VR_BOX_CHECK
                if (staged && !box_ok(P, fk, bx0, by0, bz0, dx, dy, dz, b0 + oz + oy + ox, V)) {
                } else
#endif
                if (staged) {
                    float sv[8];
                    sv[0] = box[b0];
                    sv[1] = box[b0 + ox];
                    sv[2] = box[b0 + oy];
                    sv[3] = box[b0 + oy + ox];
                    sv[4] = box[b0 + oz];
                    sv[5] = box[b0 + oz + ox];
                    sv[6] = box[b0 + oz + oy];
                    sv[7] = box[b0 + oz + oy + ox];
                    sample = blend8(sv, fk);
                } else {
                    sample = sample_direct<B, M>(vol, P, fk, tab, st);
                }
                n = i + k + 1;
                if (composite(P, sample, sx, sy, sz, sw)) {
                    alive = false;
                } else {
                    t = t + kTStep;
                    if (t > r.tfar || i + k + 1 >= kMaxSteps) {
                        alive = false;
                    } else {
                        px = px + stx;
                        py = py + sty;
                        pz = pz + stz;
                    }
                }
            }
        }
        if (staged) {  // the slice is rewritten next step: keep these reads ahead of it
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    if (!valid) return;
    if (n == 0) {  // miss (K:302-303): nothing written
        write_miss(P, o);
        return;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
}


__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
    return v;
}

// ---- wave-staged march (B <= 8) ----
// Exact-footprint staging per wave (8x8 rays), wave-synchronous: no workgroup
// barriers (a workgroup-wide version with 5 barriers per step was latency-bound,
// DESIGN.md 4.4), so the 16-20 resident waves of a CU
// hide each other's HBM latency.  Per step: (y,z) row table by LDS atomics,
// compaction by DPP scans, row-start marks + a max-scan give every lane its
// (row, x) for consecutive records, so consecutive lanes load consecutive
// records (coalesced), each record's statistic is decoded once and parked in
// LDS, and every lane blends its 8 corners from there.
constexpr int kWsTbl = 256;   // (y,z) row-table entries per wave (4 per lane)
constexpr int kWsRows = 128;  // compacted rows per wave-step
constexpr int kWsRec = 512;   // staged record statistics per wave-step
#ifndef VR_WS_U3
#define VR_WS_U3 2            // 64-record blocks in flight per lane, entropy decode
#endif

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_incl_max(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x112, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x114, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x118, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x142, 0xA, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x143, 0xC, 0xF, false));
    return v;
}

#ifndef VR_WS_WAVES
#define VR_WS_WAVES 4       // the wave-staged march is latency-bound: keep >= 4 waves/SIMD
#endif

template <int B, int M>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_WS_WAVES, 8))) void k_march_ws(const float *__restrict__ vol, Params P) {
    __shared__ int s_xmn[4][kWsTbl], s_xmx[4][kWsTbl], s_toff[4][kWsTbl];
    __shared__ uint2 s_rows[4][kWsRows];  // x: ry | rz << 10 | loff << 20,  y: xmin
    __shared__ int s_mark[4][kWsRec];
    __shared__ float s_stat[4][kWsRec];
    extern __shared__ __attribute__((aligned(32))) LogEnt s_lt[];  // entropy's log table (M == 3)
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;  // whole workgroup uniform
    if constexpr (M == 3) {
        copy_logtab(s_lt);
        __syncthreads();
    }
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    int *xmn = s_xmn[wave], *xmx = s_xmx[wave], *toff = s_toff[wave], *mark = s_mark[wave];
    uint2 *rowv = s_rows[wave];
    float *stat = s_stat[wave];
    for (uint32_t e = lane; e < (uint32_t)kWsTbl; e += 64) {
        xmn[e] = 0x7FFFFFFF;
        xmx[e] = -1;
    }
    for (uint32_t q = lane; q < (uint32_t)kWsRec; q += 64) mark[q] = -1;
    wave_sync();
    uint32_t lx, ly;
    tile_pixel(tid, lx, ly);
    const uint32_t x = (tile % P.tiles_x) * kTileW + lx;
    const uint32_t y = (tile / P.tiles_x) * kTileH + ly;
    const bool valid = x < P.CW && y < P.CH;
    const uint64_t o = P.tile_list ? (uint64_t)slot * 256u + ly * kTileW + lx
                                   : (uint64_t)y * P.W + x;
    Ray r;
    bool alive = valid && make_ray(P, x, y, r);
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = r.tnear;
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
    int n = 0;
    for (int i = 0; i < kMaxSteps; i++) {
        if (!wave_any(alive)) break;
        Foot f = {0, 0, 0, 0, 0, 0, 0.0f, 0.0f, 0.0f};
        if (alive) f = footprint(P, px, py, pz);
        const int ymn = wave_min(alive ? f.y0 : 0x7FFFFFFF);
        const int ymx = wave_max(alive ? f.y1 : -1);
        const int zmn = wave_min(alive ? f.z0 : 0x7FFFFFFF);
        const int zmx = wave_max(alive ? f.z1 : -1);
        const int Y = ymx - ymn + 1, E = Y * (zmx - zmn + 1);
        bool staged = E <= kWsTbl;
        float sample = 0.0f;
        if (staged) {
            const int e00 = (f.y0 - ymn) + Y * (f.z0 - zmn);
            const int e10 = e00 + (f.y1 - f.y0), e01 = e00 + Y * (f.z1 - f.z0);
            const int e11 = e01 + (f.y1 - f.y0);
            if (alive) {
                atomicMin(&xmn[e00], f.x0); atomicMax(&xmx[e00], f.x1);
                atomicMin(&xmn[e10], f.x0); atomicMax(&xmx[e10], f.x1);
                atomicMin(&xmn[e01], f.x0); atomicMax(&xmx[e01], f.x1);
                atomicMin(&xmn[e11], f.x0); atomicMax(&xmx[e11], f.x1);
            }
            wave_sync();
            // compaction: lane owns table entries 4*lane .. 4*lane+3 (and resets them)
            int mn[4], ln[4], cnt = 0, rec = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int e = 4 * (int)lane + j;
                ln[j] = 0;
                mn[j] = 0;
                if (e < E) {
                    const int a = xmn[e], b = xmx[e];
                    if (b >= a) { mn[j] = a; ln[j] = b - a + 1; cnt++; rec += ln[j]; }
                    xmn[e] = 0x7FFFFFFF;
                    xmx[e] = -1;
                }
            }
            const int icnt = wave_incl_scan(cnt), irec = wave_incl_scan(rec);
            const int rows = __builtin_amdgcn_readlane(icnt, 63);
            const int R = __builtin_amdgcn_readlane(irec, 63);
            staged = rows <= kWsRows && R <= kWsRec;
            if (staged) {
                // row-start marks carry the step as a tag: stale marks never match
                const float rY = 1.0f / (float)Y;
                int rb = icnt - cnt, ob = irec - rec;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    if (ln[j] > 0) {
                        const int e = 4 * (int)lane + j;
                        const int rz = (int)(((float)e + 0.5f) * rY), ry = e - rz * Y;
                        rowv[rb] = make_uint2((uint32_t)ry | ((uint32_t)rz << 10) |
                                                  ((uint32_t)ob << 20),
                                              (uint32_t)mn[j]);
                        toff[e] = ob - mn[j];
                        mark[ob] = (i << 8) | rb;
                        rb++;
                        ob += ln[j];
                    }
                }
                wave_sync();
                // consecutive lanes on consecutive records; U x 64 records in flight
                // (fewer for the register-hungry entropy decode)
                constexpr int U = M == 3 ? VR_WS_U3 : 4;
                int carry = -1;
                for (int q0 = 0; q0 < R; q0 += 64 * U) {
                    float rr[U][B];
                    int li[U];
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        const int q = q0 + 64 * u + (int)lane;
                        uint64_t ga = 0;
                        li[u] = -1;
                        if (q0 + 64 * u < R) {  // wave-uniform
                            int m = -1;
                            if (q < R) {
                                const int v = mark[q];
                                if ((v >> 8) == i) m = v & 255;
                            }
                            m = max(wave_incl_max(m), carry);
                            carry = __builtin_amdgcn_readlane(m, 63);
                            if (q < R) {
                                const uint2 rw = rowv[m];
                                const int lo = (int)(rw.x >> 20);
                                ga = (uint64_t)(zmn + (int)((rw.x >> 10) & 1023u)) * P.sz +
                                     (uint64_t)(ymn + (int)(rw.x & 1023u)) * P.sy +
                                     (uint64_t)(rw.y + (uint32_t)(q - lo));
                                li[u] = q;
                            }
                        }
                        load_rec<B>(vol, ga, rr[u]);
                    }
#pragma unroll
                    for (int u = 0; u < U; u++)
                        if (li[u] >= 0)
                            stat[li[u]] = record_stat_p<B, M>(rr[u], P.enorm, s_lt);
                }
                wave_sync();
                if (alive) {
                    const int t00 = toff[e00], t10 = toff[e10];
                    const int t01 = toff[e01], t11 = toff[e11];
                    float sv[8];
                    sv[0] = stat[t00 + f.x0]; sv[1] = stat[t00 + f.x1];
                    sv[2] = stat[t10 + f.x0]; sv[3] = stat[t10 + f.x1];
                    sv[4] = stat[t01 + f.x0]; sv[5] = stat[t01 + f.x1];
                    sv[6] = stat[t11 + f.x0]; sv[7] = stat[t11 + f.x1];
                    sample = blend8(sv, f);
                }
                wave_sync();
            }
        }
        if (alive) {
            if (!staged) sample = sample_direct<B, M, 2>(vol, P, f);
            n = i + 1;
            if (composite(P, sample, sx, sy, sz, sw)) {
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
    if (n == 0) {  // miss (K:302-303): nothing written
        write_miss(P, o);
        return;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
}

// ---- software-pipelined march (B <= 8) ----
#ifndef VR_PIPE_WAVES
#define VR_PIPE_WAVES 1     // minimum waves per SIMD the register allocation must allow
#endif
// B = 8: at most 3 waves per SIMD.  The cap is a scheduling hint as much as
// an occupancy limit: it lets the compiler spend registers on keeping the next
// step's 16 gathers in flight; 1.41 -> 1.35 ms at 1024^3 x 8, C0 (8 waves
// allowed: the march also fits 4 waves, but runs slower).
#ifndef VR_PIPE_MAXWAVES
#define VR_PIPE_MAXWAVES(B) ((B) >= 8 ? 3 : 8)
#endif
template <int B, int M, int GM = kGatherMode<M>>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_PIPE_WAVES, VR_PIPE_MAXWAVES(B)))) void k_march_pipe(const float *__restrict__ vol, Params P) {
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;
    unsigned long long t0 = 0;
    if (P.wave_clock) t0 = wall_clock64();
    float *st = nullptr;
    const LogEnt *tab = nullptr;
    if constexpr (M == 3) {  // entropy: rolled per-bin sums over LDS record columns
        // (in the dynamic LDS, the launch requests sizeof(EntropyLds<B>) at least)
        extern __shared__ __attribute__((aligned(32))) float s_dyn[];
        EntropyLds<B> *el = reinterpret_cast<EntropyLds<B> *>(s_dyn);
        copy_logtab(el->tab);
        __syncthreads();
        st = el->col + (threadIdx.x >> 6) * 64u * B;
        tab = el->tab;
    }
    const int n = march_pipe_tile<B, M, GM>(vol, P, slot, tile, threadIdx.x, st, tab);
    if (P.tile_cost) record_tile_cost(P, tile, n);  // all lanes have reconverged here
    if (P.wave_clock && (threadIdx.x & 63) == 0) {
        unsigned long long *w = P.wave_clock + ((uint64_t)slot * 4u + threadIdx.x / 64u) * 3u;
        w[0] = t0;
        w[1] = wall_clock64();
        w[2] = __smid();  // XCC id in the high bits on gfx94x/gfx950
    }
}

// ---- wide records (B = 16, 32: the reference's own 32-bin histograms) ----
// One lane per ray, as k_march_pipe, but a step's 8 corner records (1 KiB per
// lane at B = 32) cannot sit in registers twice.  The corners go in batches of
// CG = 64 / B records (64 VGPRs): while batch k decodes, batch k + 1 -- after a
// step's last batch, the first batch of the next step's footprint, gathered
// unconditionally like k_march_pipe's next step -- is in flight, so every wave
// keeps loads outstanding through the f64 decode chains (32 dependent bins per
// record at B = 32).  A 32-bin record is exactly one 128-B line, so every byte
// a gather fetches is used.  Arithmetic and blend order are those of k_march's
// direct path (record_stat per corner, blend8).
__device__ __forceinline__ uint64_t corner_index(const Params &P, const Foot &f, int j) {
    const uint64_t z = (j & 4) ? (uint64_t)f.z1 : (uint64_t)f.z0;
    const uint64_t y = (j & 2) ? (uint64_t)f.y1 : (uint64_t)f.y0;
    const uint64_t x = (j & 1) ? (uint64_t)f.x1 : (uint64_t)f.x0;
    return z * P.sz + y * P.sy + x;
}

// one batch: gather corners jn .. jn + CG - 1 of fl into nxt, then decode cur
template <int B, int M>
__device__ __forceinline__ void wide_batch(const float *__restrict__ vol, const Params &P,
                                           const Foot &fl, int jn, float (&nxt)[64 / B][B],
                                           const float (&cur)[64 / B][B], float *sv,
                                           const LogEnt *lt) {
    constexpr int CG = 64 / B;
#pragma unroll
    for (int j = 0; j < CG; j++) load_rec<B>(vol, corner_index(P, fl, jn + j), nxt[j]);
#pragma unroll
    for (int j = 0; j < CG; j++) sv[j] = record_stat_p<B, M>(cur[j], P.enorm, lt);
}

template <int B, int M>
__device__ __forceinline__ int march_wide_tile(const float *__restrict__ vol, const Params &P,
                                               uint32_t slot, uint32_t tile, uint32_t tid,
                                               const LogEnt *lt) {
    constexpr int CG = 64 / B, NB = 8 / CG;
    static_assert(NB % 2 == 0, "batches alternate between two register sets");
    uint32_t lx, ly;
    lane_pixel(P, tid, lx, ly);
    const uint32_t x = (tile % P.tiles_x) * kTileW + lx;
    const uint32_t y = (tile / P.tiles_x) * kTileH + ly;
    if (x >= P.CW || y >= P.CH) return -1;  // no cross-lane work in this kernel
    const uint64_t o = P.tile_list ? (uint64_t)slot * 256u + ly * kTileW + lx
                                   : (uint64_t)y * P.W + x;
    Ray r;
    if (!make_ray(P, x, y, r)) {
        write_miss(P, o);
        return -1;
    }
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = r.tnear;
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
    int n = 0;
    Foot fc = footprint(P, px, py, pz);
    float ra[CG][B], rb[CG][B];
#pragma unroll
    for (int j = 0; j < CG; j++) load_rec<B>(vol, corner_index(P, fc, j), ra[j]);
    for (int i = 0; i < kMaxSteps; i++) {
        const float tn = t + kTStep;                               // K:701
        const bool cont = !(tn > r.tfar) && (i + 1 < kMaxSteps);  // K:703, K:381
        const float nx = px + stx, ny = py + sty, nz = pz + stz;   // K:706
        const Foot fn = footprint(P, nx, ny, nz);
        float sv[8];
#pragma unroll
        for (int k = 0; k < NB; k += 2) {
            wide_batch<B, M>(vol, P, fc, (k + 1) * CG, rb, ra, sv + k * CG, lt);
            const Foot &fl = k + 2 < NB ? fc : fn;
            wide_batch<B, M>(vol, P, fl, ((k + 2) % NB) * CG, ra, rb, sv + (k + 1) * CG, lt);
        }
        const float sample = blend8(sv, fc);
        n = i + 1;
        if (composite(P, sample, sx, sy, sz, sw) || !cont) break;
        t = tn;
        px = nx;
        py = ny;
        pz = nz;
        fc = fn;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
    return n;
}

// At most VR_WIDE_WAVES waves per SIMD: the register budget that keeps a batch
// of loads in flight through the decode (as k_march_pipe's cap; without it the
// scheduler sinks the loads below the decode to save registers).
template <int B, int M>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_WIDE_MINW, VR_WIDE_WAVES))) void k_march_wide(const float *__restrict__ vol, Params P) {
    static_assert(M == 1 || M == 2, "mean and variance (entropy: k_march)");
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;
    const int n = march_wide_tile<B, M>(vol, P, slot, tile, threadIdx.x, nullptr);
    if (P.tile_cost) record_tile_cost(P, tile, n);  // all lanes have reconverged here
}

#ifndef VR_QUAD_MAP
#define VR_QUAD_MAP 0
#endif

// ---- quad-cooperative pipelined march (B == 8) ----
// Lane l = 4q + g of a wave is the home of the ray at pixel (q, g) of the
// wave's 16x4 pixel block (the 4 waves of a workgroup sit side by side in the
// 64x4 tile).  For
// the gathers the four lanes of quad q work for ray (G, q), G = 0..3 in turn:
// per (y,z) corner combo they read that ray's x0/x1 record pair as ONE
// contiguous 64-byte run (lane g takes 16-byte chunk g), so every 4-lane group
// of a gather instruction is one contiguous request.  This is the cheapest
// pattern for the texture-address path, which bounds per-ray 16-byte gathers
// at 32-byte strides (tools/ta_rates.hip, tools/replay_loads.hip, PMC
// TA_TA_BUSY ~90 %).  A pair swap with the xor-1 neighbour then gives each
// lane two complete records -- corner (x = g>>1, y = g&1) at z0 and z1 -- so
// every corner is still decoded exactly once, and the blend runs inside the
// quad in the reference's lerp order (x, then y, then z).  Next-step gathers
// are issued group by group into the registers the current group has just
// released (rolling prefetch).


// ---- wide records, quad-cooperative gathers (B = 16, 32) ----
// k_march_wide is bound by the texture-address path (PMC TA_BUSY 95-100 % at
// 1024^3 x 32, C0): each 16-byte wave-instruction of a lane-owned 128-B record
// touches 64 lines.  Here the 4 lanes of a quad (4 neighbouring rays) load
// each other's records together: for corner j and quad ray R, lane g reads
// chunk 4s + g of R's record (s = 0 .. B/16 - 1), so every 4-lane group of an
// instruction is one contiguous 64-byte run, 16 runs per instruction.  A 4x4
// transpose over (ray, lane) with quad_perm DPP (two butterfly stages, the
// xor-2 and xor-1 exchanges) then leaves each lane with its own ray's whole
// record, which it decodes exactly as k_march_wide does.  The loop is
// wave-uniform (the quads exchange data every step); corner batches are
// double-buffered as in k_march_wide.
// the 4 rays' packed footprints of a quad (pack_foot: x0 | y0 << 16, z0 | dx << 16 |
// dy << 17 | dz << 18 | live << 19)
struct QuadFeet {
    int w0[4], w1[4];
};
__device__ __forceinline__ QuadFeet quad_feet(const Foot &f, bool live) {
    const FootPacked p = pack_foot(f, live);
    QuadFeet q;
    q.w0[0] = bcast_g<0>(p.w0); q.w1[0] = bcast_g<0>(p.w1);
    q.w0[1] = bcast_g<1>(p.w0); q.w1[1] = bcast_g<1>(p.w1);
    q.w0[2] = bcast_g<2>(p.w0); q.w1[2] = bcast_g<2>(p.w1);
    q.w0[3] = bcast_g<3>(p.w0); q.w1[3] = bcast_g<3>(p.w1);
    return q;
}

// Gather corner j of the quad's 4 rays (lane g: chunks 4s + g) into M[s][R];
// rays not live skip their loads.
template <int B>
__device__ __forceinline__ void wq_gather(const float *__restrict__ vol, const Params &P,
                                          const QuadFeet &q, int j, uint32_t g,
                                          float4 (&M)[B / 16][4]) {
#pragma unroll
    for (int R = 0; R < 4; R++) {
        const uint32_t w0 = (uint32_t)q.w0[R], w1 = (uint32_t)q.w1[R];
        if ((w1 >> 19) & 1u) {
            const uint64_t x = (w0 & 0xFFFFu) + ((j & 1) ? ((w1 >> 16) & 1u) : 0u);
            const uint64_t y = (w0 >> 16) + ((j & 2) ? ((w1 >> 17) & 1u) : 0u);
            const uint64_t z = (w1 & 0xFFFFu) + ((j & 4) ? ((w1 >> 18) & 1u) : 0u);
            const float4 *rec =
                reinterpret_cast<const float4 *>(vol + (z * P.sz + y * P.sy + x) * (uint64_t)B);
#pragma unroll
            for (int s = 0; s < B / 16; s++) M[s][R] = rec[4 * s + g];
        }
    }
}

// transpose a gathered corner and decode this lane's record
template <int B, int M>
__device__ __forceinline__ float wq_decode(float4 (&Mc)[B / 16][4], uint32_t g, bool alive,
                                           float enorm, const LogEnt *lt, float *col) {
#pragma unroll
    for (int s = 0; s < B / 16; s++) quad_transpose(Mc[s], g);
    float st = 0.0f;
    if (alive) {
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
        // 32-bin entropy: the rolled per-bin sum over this lane's LDS column
        // (entropy_stash; 1024^3 x 32 C1 m3 ~51 -> 26.8 ms); 16 bins keep the
        // unrolled sum (13.4 ms rolled vs 12.5)
        if constexpr (M == 3 && B >= 32) st = entropy_stash<B>(p, col, threadIdx.x & 63u, enorm, lt);
        else st = record_stat_p<B, M>(p, enorm, lt);
    }
    return st;
}

// batches K (in A) and K + 1 (in Bf) of a step: batch K decodes while batch
// K + 1 loads into Bf, then batch K + 1 decodes while the next batch -- of this
// step or, after the step's last, the next step's first -- loads into A.
// Compile-time K keeps every array index static (registers, no scratch).
template <int B, int M, int K>
__device__ __forceinline__ void wq_pair(const float *__restrict__ vol, const Params &P,
                                        const QuadFeet &qc, const QuadFeet &qn, uint32_t g,
                                        bool alive, float4 (&A)[64 / B][B / 16][4],
                                        float4 (&Bf)[64 / B][B / 16][4], float (&sv)[8],
                                        const LogEnt *lt, float *col) {
    constexpr int CG = 64 / B, NB = 8 / CG;
#pragma unroll
    for (int c = 0; c < CG; c++) wq_gather<B>(vol, P, qc, (K + 1) * CG + c, g, Bf[c]);
#pragma unroll
    for (int c = 0; c < CG; c++) sv[K * CG + c] = wq_decode<B, M>(A[c], g, alive, P.enorm, lt, col);
    if constexpr (K + 2 < NB) {
#pragma unroll
        for (int c = 0; c < CG; c++) wq_gather<B>(vol, P, qc, (K + 2) * CG + c, g, A[c]);
    } else {
#pragma unroll
        for (int c = 0; c < CG; c++) wq_gather<B>(vol, P, qn, c, g, A[c]);
    }
#pragma unroll
    for (int c = 0; c < CG; c++) sv[(K + 1) * CG + c] = wq_decode<B, M>(Bf[c], g, alive, P.enorm, lt, col);
}

template <int B, int M>
__device__ __forceinline__ int march_wq_tile(const float *__restrict__ vol, const Params &P,
                                             uint32_t slot, uint32_t tile, uint32_t tid,
                                             const LogEnt *lt, float *col) {
    constexpr int S = B / 16;        // 16-byte chunks per lane per record
    constexpr int CG = 64 / B;       // corners per batch (64 VGPRs)
    constexpr int NB = 8 / CG;       // batches per step
    static_assert(NB % 2 == 0, "batches alternate between two register sets");
    uint32_t lx, ly;
    if (P.wq_map) {  // oblique views: a wave takes a 16x4 block, a quad one pixel column
        lx = (tid >> 6) * 16u + ((tid & 63u) >> 2);
        ly = tid & 3u;
    } else {
        tile_pixel(tid, lx, ly);
    }
    const uint32_t x = (tile % P.tiles_x) * kTileW + lx;
    const uint32_t y = (tile / P.tiles_x) * kTileH + ly;
    const bool valid = x < P.CW && y < P.CH;
    const uint64_t o = P.tile_list ? (uint64_t)slot * 256u + ly * kTileW + lx
                                   : (uint64_t)y * P.W + x;
    const uint32_t g = tid & 3u;
    // every lane stays to the end: the quads exchange records every step
    Ray r = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    bool alive = valid && make_ray(P, x, y, r);
    const bool hit = alive;
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = r.tnear;
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
    int n = 0;
    Foot fc = footprint(P, px, py, pz);
    QuadFeet qc = quad_feet(fc, alive);
    float4 A[CG][S][4], Bf[CG][S][4];
#pragma unroll
    for (int c = 0; c < CG; c++) wq_gather<B>(vol, P, qc, c, g, A[c]);
    for (int i = 0; i < kMaxSteps; i++) {
        if (!wave_any(alive)) break;
        const float tn = t + kTStep;                                        // K:701
        const bool cont = alive && !(tn > r.tfar) && (i + 1 < kMaxSteps);  // K:703, K:381
        const float nx = px + stx, ny = py + sty, nz = pz + stz;            // K:706
        const Foot fn = footprint(P, nx, ny, nz);
        const QuadFeet qn = quad_feet(fn, cont);
        float sv[8];
        wq_pair<B, M, 0>(vol, P, qc, qn, g, alive, A, Bf, sv, lt, col);
        if constexpr (NB == 4) wq_pair<B, M, 2>(vol, P, qc, qn, g, alive, A, Bf, sv, lt, col);
        if (alive) {
            n = i + 1;
            if (composite(P, blend8(sv, fc), sx, sy, sz, sw) || !cont) {
                alive = false;
            } else {
                t = tn;
                px = nx;
                py = ny;
                pz = nz;
            }
        }
        fc = fn;
        qc = qn;
    }
    if (!valid) return -1;
    if (!hit) {
        write_miss(P, o);
        return -1;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
    return n;
}

template <int B, int M>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_WIDE_MINW, M == 3 && B >= 32 ? 8 : VR_WIDE_WAVES))) void k_march_wq(const float *__restrict__ vol, Params P) {
    __shared__ LogEnt s_lt[M == 3 ? kLogTabN : 1];  // entropy: the exact-log table (copy_logtab)
    // entropy: each wave's bin-major record columns (entropy_stash)
    __shared__ float s_col[M == 3 && B >= 32 ? 4 * 64 * B : 1];
    if constexpr (M == 3) {
        copy_logtab(s_lt);
        __syncthreads();
    }
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;
    const int n = march_wq_tile<B, M>(vol, P, slot, tile, threadIdx.x, s_lt,
                                      s_col + (threadIdx.x >> 6) * 64u * B);
    if (P.tile_cost) record_tile_cost(P, tile, n);  // all lanes have reconverged here
}

// Gather ray (G, q)'s four x-pairs: L[c] = chunk g of the pair at combo c =
// (y = c & 1, z = c >> 1).  A pair clamped at the x edge (x1 == x0) repeats x0.
// BR: the volume is the 2x2 (x, y) micro-brick copy (P.bvol): lane g reads
// half g & 1 of record x0 (g < 2) or x1 (g >= 2) of each (y, z) combo, so a
// footprint's four (x, y) corners at one z share a line when x0 and y0 are
// even (oblique views: fewer distinct lines per wave step).
template <int G, bool BR = false>
__device__ __forceinline__ bool qc_gather(const float *__restrict__ vol, const Params &P,
                                          const FootPacked &fp, uint32_t g, float4 (&L)[4]) {
    const int w0 = bcast_g<G>(fp.w0), w1 = bcast_g<G>(fp.w1);
    const bool live = (w1 >> 19) & 1;
    if (BR && live) {
        const uint64_t x0 = (uint32_t)w0 & 0xFFFFu, y0 = (uint32_t)w0 >> 16;
        const uint64_t z0 = (uint32_t)w1 & 0xFFFFu;
        const uint64_t ddx = (w1 >> 16) & 1, ddy = (w1 >> 17) & 1, ddz = (w1 >> 18) & 1;
        const uint64_t xg = x0 + (ddx & (g >> 1)), y1 = y0 + ddy;
        const uint64_t bx = (xg >> 1) * 4u + (xg & 1u);
        const uint64_t ry0 = (y0 >> 1) * P.sy + (y0 & 1u) * 2u + bx;
        const uint64_t ry1 = (y1 >> 1) * P.sy + (y1 & 1u) * 2u + bx;
        const uint64_t rz0 = z0 * P.sz, rz1 = rz0 + ddz * P.sz;
        const uint32_t half = g & 1u;
        L[0] = reinterpret_cast<const float4 *>(vol + (rz0 + ry0) * 8)[half];
        L[1] = reinterpret_cast<const float4 *>(vol + (rz0 + ry1) * 8)[half];
        L[2] = reinterpret_cast<const float4 *>(vol + (rz1 + ry0) * 8)[half];
        L[3] = reinterpret_cast<const float4 *>(vol + (rz1 + ry1) * 8)[half];
    } else if (live) {
        const uint64_t x0 = (uint32_t)w0 & 0xFFFFu, y0 = (uint32_t)w0 >> 16;
        const uint64_t z0 = (uint32_t)w1 & 0xFFFFu;
        const uint64_t ddy = (w1 >> 17) & 1, ddz = (w1 >> 18) & 1;
        const uint32_t chunk = ((w1 >> 16) & 1) ? g : (g & 1u);
        const uint64_t r00 = z0 * P.sz + y0 * P.sy + x0;
        const uint64_t r10 = r00 + ddy * P.sy, r01 = r00 + ddz * P.sz, r11 = r10 + ddz * P.sz;
        L[0] = reinterpret_cast<const float4 *>(vol + r00 * 8)[chunk];
        L[1] = reinterpret_cast<const float4 *>(vol + r10 * 8)[chunk];
        L[2] = reinterpret_cast<const float4 *>(vol + r01 * 8)[chunk];
        L[3] = reinterpret_cast<const float4 *>(vol + r11 * 8)[chunk];
    }
    return live;
}


template <int G, int M, bool BR>
__device__ __forceinline__ float qc_group(const float *__restrict__ vol, const Params &P,
                                          const FootPacked &fc, bool lc, const FootPacked &fn,
                                          bool &ln, uint32_t g, float4 (&L)[4],
                                          const LogEnt *lt) {
    // this step's records of ray (G, q) out of the chunk registers ...
    const bool odd = g & 1u;
    float r0[8], r1[8];
    pair_swap(L[0], L[1], odd, r0);  // combo (y = g&1, z0)
    pair_swap(L[2], L[3], odd, r1);  // combo (y = g&1, z1)
    // ... which frees them for the next step's gathers of the same group
    ln = qc_gather<G, BR>(vol, P, fn, g, L);
    float s0 = 0.0f, s1 = 0.0f;
    if (lc) {
        // (the rolled LDS-column entropy measured slower here: 1024^3 x 8 C1 m3
        // 8.37 -> 9.44 ms, profiles/r04/variants_1024x8_m3.log)
        s0 = record_stat_p<8, M>(r0, P.enorm, lt);
        s1 = record_stat_p<8, M>(r1, P.enorm, lt);
    }
    return qc_blend<G>(fc, s0, s1);
}

template <int M, bool BR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_QUAD_WAVES, 8))) void k_march_quad(const float *__restrict__ vol, Params P) {
    // entropy: the exact log's table in LDS (the launch's occupancy request
    // reserves far more than its 2 KiB); a load from there is an LDS read, not
    // a constant-memory gather on the march's critical path
    extern __shared__ __attribute__((aligned(32))) LogEnt s_lt[];
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;  // uniform per workgroup
    if constexpr (M == 3) {
        copy_logtab(s_lt);
        __syncthreads();
    }
    unsigned long long t0 = 0;
    if (P.wave_clock) t0 = wall_clock64();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t q = lane >> 2, g = lane & 3u;
#if VR_QUAD_MAP == 1  // wave = one 64-pixel row, quad = 4 consecutive pixels
    const uint32_t lx = lane, ly = wave;
#else                 // 16x4 block per wave, quad = a column
    const uint32_t lx = wave * 16u + q, ly = g;
#endif
    const uint32_t x = (tile % P.tiles_x) * kTileW + lx;
    const uint32_t y = (tile / P.tiles_x) * kTileH + ly;
    const bool valid = x < P.CW && y < P.CH;
    const uint64_t o = P.tile_list ? (uint64_t)slot * 256u + ly * kTileW + lx
                                   : (uint64_t)y * P.W + x;
    // every lane stays to the end: quads cooperate on each other's rays
    Ray r;
    bool alive = valid && make_ray(P, x, y, r);
    const bool hit = alive;
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = r.tnear;
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
    int n = 0;
    float4 L0[4], L1[4], L2[4], L3[4];  // chunk registers of groups 0..3
    FootPacked fc = pack_foot(footprint(P, px, py, pz), alive);
    bool lc[4];
    lc[0] = qc_gather<0, BR>(vol, P, fc, g, L0);
    lc[1] = qc_gather<1, BR>(vol, P, fc, g, L1);
    lc[2] = qc_gather<2, BR>(vol, P, fc, g, L2);
    lc[3] = qc_gather<3, BR>(vol, P, fc, g, L3);
    for (int i = 0; i < kMaxSteps; i++) {
        if (!wave_any(alive)) break;
        // next step of this lane's own ray (speculative: assumes no early exit)
        const float tn = t + kTStep;                                        // K:701
        const bool cont = alive && !(tn > r.tfar) && (i + 1 < kMaxSteps);  // K:703, 381
        const float nx = px + stx, ny = py + sty, nz = pz + stz;            // K:706
        const FootPacked fn = pack_foot(footprint(P, nx, ny, nz), cont);
        bool ln[4];
        const float b0 = qc_group<0, M, BR>(vol, P, fc, lc[0], fn, ln[0], g, L0, s_lt);
        const float b1 = qc_group<1, M, BR>(vol, P, fc, lc[1], fn, ln[1], g, L1, s_lt);
        const float b2 = qc_group<2, M, BR>(vol, P, fc, lc[2], fn, ln[2], g, L2, s_lt);
        const float b3 = qc_group<3, M, BR>(vol, P, fc, lc[3], fn, ln[3], g, L3, s_lt);
        const float sample = g == 0 ? b0 : (g == 1 ? b1 : (g == 2 ? b2 : b3));
        if (alive) {
            n = i + 1;
            if (composite(P, sample, sx, sy, sz, sw) || !cont) {
                alive = false;
            } else {
                t = tn;
                px = nx;
                py = ny;
                pz = nz;
            }
        }
        fc = fn;
#pragma unroll
        for (int k = 0; k < 4; k++) lc[k] = ln[k];
    }
    if (P.wave_clock && lane == 0) {  // tooling (vr_debug_wave_clock, tools/wave_timeline.py)
        unsigned long long *w = P.wave_clock + ((uint64_t)slot * 4u + wave) * 3u;
        w[0] = t0;
        w[1] = wall_clock64();
        w[2] = __smid();
    }
    if (!valid) return;
    if (!hit) {
        write_miss(P, o);
        return;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
}

// ---- the quad march with two lanes per ray (short launches: a rank's list) ----
// The halves h = lane >> 5 of a wave take alternate steps of the same 8x4-pixel
// block: h = 0 gathers and decodes the even steps of its quad's rays, h = 1 the
// odd ones, each half with k_march_quad's quad gathers, pair swaps and blends.
// Every lane keeps its ray's even-step chain (t and position accumulated one
// step at a time, K:701, 706), so both halves hold the same float values; after
// one cross-half exchange of the two samples both composite them in order and
// end the ray at the same step -- the one-lane march's float operations in the
// same order.  A ray's chain of dependent gathers is halved, which is what
// bounds a short launch: at N = 8 a C1 rank's longest wave took 0.55 of its
// 0.59 ms (tools/wave_timeline.py).  A 64x4 tile is two workgroups; workgroup b
// renders half (b >> 3) & 1 of launch slot (b >> 4) * 8 + (b & 7), on XCD b % 8
// = the slot's XCD.
template <int M, bool BR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_QUAD_WAVES, 8))) void k_march_quad2(const float *__restrict__ vol, Params P) {
    extern __shared__ __attribute__((aligned(32))) LogEnt s_lt2[];
    const uint32_t vb = (blockIdx.x >> 4) * 8u + (blockIdx.x & 7u), part = (blockIdx.x >> 3) & 1u;
    if (vb >= P.n_tiles) return;  // uniform per workgroup
    const uint32_t slot = (P.tile_list || P.perm) ? vb : xcd_slot(vb, P.n_tiles);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;
    if constexpr (M == 3) {
        copy_logtab(s_lt2);
        __syncthreads();
    }
    unsigned long long t0 = 0;
    if (P.wave_clock) t0 = wall_clock64();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t h = lane >> 5, q = (lane >> 2) & 7u, g = lane & 3u;
    const uint32_t lx = part * 32u + wave * 8u + q, ly = g;
    const uint32_t x = (tile % P.tiles_x) * kTileW + lx;
    const uint32_t y = (tile / P.tiles_x) * kTileH + ly;
    const bool valid = x < P.CW && y < P.CH;
    const uint64_t o = P.tile_list ? (uint64_t)slot * 256u + ly * kTileW + lx
                                   : (uint64_t)y * P.W + x;
    Ray r;
    bool alive = valid && make_ray(P, x, y, r);
    const bool hit = alive;
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = r.tnear;  // the chain at the iteration's even step i
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
    int n = 0;
    float4 L0[4], L1[4], L2[4], L3[4];
    FootPacked fc;
    {
        const float t1 = t + kTStep;
        const bool live = h ? alive && !(t1 > r.tfar) && (1 < kMaxSteps) : alive;
        fc = h ? pack_foot(footprint(P, px + stx, py + sty, pz + stz), live)
               : pack_foot(footprint(P, px, py, pz), live);
    }
    bool lc[4];
    lc[0] = qc_gather<0, BR>(vol, P, fc, g, L0);
    lc[1] = qc_gather<1, BR>(vol, P, fc, g, L1);
    lc[2] = qc_gather<2, BR>(vol, P, fc, g, L2);
    lc[3] = qc_gather<3, BR>(vol, P, fc, g, L3);
    for (int i = 0; i < kMaxSteps; i += 2) {
        if (!wave_any(alive)) break;
        // steps i+1, i+2, i+3 of the chain; this half's next gather is step
        // i+2 (h = 0) or i+3 (h = 1), speculative (assumes no early exit)
        const float ta = t + kTStep, tb = ta + kTStep, tc = tb + kTStep;   // K:701
        const float ax = px + stx, ay = py + sty, az = pz + stz;            // K:706
        const float bx = ax + stx, by = ay + sty, bz = az + stz;
        const float nx = h ? bx + stx : bx, ny = h ? by + sty : by, nz = h ? bz + stz : bz;
        const bool nl = h ? alive && !(tc > r.tfar) && (i + 3 < kMaxSteps)
                          : alive && !(tb > r.tfar) && (i + 2 < kMaxSteps);
        const FootPacked fn = pack_foot(footprint(P, nx, ny, nz), nl);
        bool ln[4];
        const float b0 = qc_group<0, M, BR>(vol, P, fc, lc[0], fn, ln[0], g, L0, s_lt2);
        const float b1 = qc_group<1, M, BR>(vol, P, fc, lc[1], fn, ln[1], g, L1, s_lt2);
        const float b2 = qc_group<2, M, BR>(vol, P, fc, lc[2], fn, ln[2], g, L2, s_lt2);
        const float b3 = qc_group<3, M, BR>(vol, P, fc, lc[3], fn, ln[3], g, L3, s_lt2);
        const float mine = g == 0 ? b0 : (g == 1 ? b1 : (g == 2 ? b2 : b3));
        const float other = __shfl_xor(mine, 32);
        const float s_even = h ? other : mine, s_odd = h ? mine : other;
        if (alive) {
            n = i + 1;
            if (composite(P, s_even, sx, sy, sz, sw) || !(!(ta > r.tfar) && (i + 1 < kMaxSteps))) {
                alive = false;  // K:698, 703, 381
            } else {
                n = i + 2;
                if (composite(P, s_odd, sx, sy, sz, sw) || !(!(tb > r.tfar) && (i + 2 < kMaxSteps))) {
                    alive = false;
                } else {
                    t = tb;
                    px = bx;
                    py = by;
                    pz = bz;
                }
            }
        }
        fc = fn;
#pragma unroll
        for (int k = 0; k < 4; k++) lc[k] = ln[k];
    }
    if (P.wave_clock && lane == 0) {  // tooling (vr_debug_wave_clock, tools/wave_timeline.py)
        unsigned long long *w = P.wave_clock + ((uint64_t)slot * 8u + part * 4u + wave) * 3u;
        w[0] = t0;
        w[1] = wall_clock64();
        w[2] = __smid();
    }
    if (!valid || h) return;
    if (!hit) {
        write_miss(P, o);
        return;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
}




// ---- synthetic volume ----

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
        float *dst = vol + ((uint64_t)z * a.sz + (uint64_t)y * a.sy + x) * (uint64_t)nb;
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
    const uint32_t px = (tile % tiles_x) * kTileW + (threadIdx.x & (kTileW - 1));
    const uint32_t py = (tile / tiles_x) * kTileH + threadIdx.x / kTileW;
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

// Exhaustive check of logf_canon against (float)log((double)x) over every
// positive finite float, for both fast forms (series and table); cnt[0] =
// mismatches of either, cnt[1] = inputs either form left to the double-log
// fallback (summed over the two).
__global__ __launch_bounds__(256) void k_logcheck(unsigned long long *cnt) {
    unsigned long long bad = 0, slow = 0;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t b = 1 + blockIdx.x * blockDim.x + threadIdx.x; b < 0x7F800000u; b += stride) {
        const float x = __uint_as_float(b);
        float r;
        slow += !logf_fast_series(x, r);
        slow += !logf_fast_tab(x, r);
        const uint32_t want = __float_as_uint((float)log((double)x));
        bad += __float_as_uint(logf_canon<false>(x)) != want;
        bad += __float_as_uint(logf_canon<true>(x)) != want;
    }
    if (bad) atomicAdd(&cnt[0], bad);
    if (slow) atomicAdd(&cnt[1], slow);
}

hipError_t launch_logcheck(unsigned long long *cnt, hipStream_t s) {
    hipLaunchKernelGGL(k_logcheck, dim3(8192), dim3(256), 0, s, cnt);
    return hipGetLastError();
}

// ------------------------------ launchers ---------------------------------


template <int B, bool COUNT>
static hipError_t march_b(int method, const float *vol, Params P, uint32_t nslots,
                          hipStream_t s) {
    const dim3 grid(nslots), block(256);
    // one f32 box slice of box_max voxels per wave (4 waves); a larger request
    // caps the workgroups resident per CU (160 KiB of LDS per CU)
    // (+ the log table and the record columns of the wide entropy march, k_march)
    const size_t lds = cap_lds(P, P.wg_per_cu, B > 0 ? (size_t)P.box_max * 4u * sizeof(float) +
                                                   (B >= 8 && method == 3 ? kLogTabN * sizeof(LogEnt) + 4u * 64u * B * sizeof(float) : 0) : 0);
    if constexpr (!COUNT && B > 0 && B <= 8) {
        if (P.path == 7) {
            hipError_t err = hipSuccess;
            if (launch_march_seg(B, method, P.seg_lanes, vol, P, nslots, s, err)) return err;
            P.path = 2;
        }
        if (B == 8 && P.path == 0 && method >= 1 && method <= 3) {
            note_kernel(P.bvol ? "k_march_quad_brick" : "k_march_quad", B, method);
            // The quad march uses no LDS; an LDS request caps it at 2 workgroups
            // (2 waves per SIMD) per CU, which trims the oblique view's line
            // re-reads: 1024^3x8 C1 3.73 -> 3.52 ms (3 per CU by registers, 1 per
            // CU 3.91).  VR_WG_PER_CU overrides.
            // A rank's tile list of <= 400 K rays (8 GPUs at 1080p) runs at 1 per
            // CU: its tiles are scattered over the frame, and fewer rays in flight
            // re-read fewer lines (cost-dealt C1 lists, max over 8 ranks: 0.71 ->
            // 0.59 ms; 3 per CU 0.68; tools/rank_sim.py)
            const int qcap = P.wg_per_cu > 0 ? P.wg_per_cu
                             : (P.tile_list && (uint64_t)nslots * 256u <= 400000u) ? 1 : 2;
            // entropy: the log table (qc_group) at the front
            const size_t qlds = cap_lds(P, qcap, method == 3 ? kLogTabN * sizeof(LogEnt) : 0);
            if (P.quad2) {  // two lanes per ray, two workgroups per tile
                note_kernel(P.bvol ? "k_march_quad2_brick" : "k_march_quad2", B, method);
                const dim3 grid2(((nslots + 7u) / 8u) * 16u);
                Params Q = P;
                if (P.bvol) {
                    Q.sy = P.bsy;
                    Q.sz = P.bsz;
                }
                const float *v = P.bvol ? P.bvol : vol;
                switch (method * 2 + (P.bvol ? 1 : 0)) {
                case 2: hipLaunchKernelGGL((k_march_quad2<1, false>), grid2, block, qlds, s, v, Q); break;
                case 3: hipLaunchKernelGGL((k_march_quad2<1, true>), grid2, block, qlds, s, v, Q); break;
                case 4: hipLaunchKernelGGL((k_march_quad2<2, false>), grid2, block, qlds, s, v, Q); break;
                case 5: hipLaunchKernelGGL((k_march_quad2<2, true>), grid2, block, qlds, s, v, Q); break;
                case 6: hipLaunchKernelGGL((k_march_quad2<3, false>), grid2, block, qlds, s, v, Q); break;
                case 7: hipLaunchKernelGGL((k_march_quad2<3, true>), grid2, block, qlds, s, v, Q); break;
                }
                return hipGetLastError();
            }
            if (P.bvol) {
                Params Q = P;
                Q.sy = P.bsy;
                Q.sz = P.bsz;
                switch (method) {
                case 1: hipLaunchKernelGGL((k_march_quad<1, true>), grid, block, qlds, s, P.bvol, Q); break;
                case 2: hipLaunchKernelGGL((k_march_quad<2, true>), grid, block, qlds, s, P.bvol, Q); break;
                case 3: hipLaunchKernelGGL((k_march_quad<3, true>), grid, block, qlds, s, P.bvol, Q); break;
                }
            } else {
                switch (method) {
                case 1: hipLaunchKernelGGL((k_march_quad<1, false>), grid, block, qlds, s, vol, P); break;
                case 2: hipLaunchKernelGGL((k_march_quad<2, false>), grid, block, qlds, s, vol, P); break;
                case 3: hipLaunchKernelGGL((k_march_quad<3, false>), grid, block, qlds, s, vol, P); break;
                }
            }
            return hipGetLastError();
        }
        if (P.path == 4 && method >= 1 && method <= 3) {
            note_kernel("k_march_ws", B, method);
            switch (method) {
            case 1: hipLaunchKernelGGL((k_march_ws<B, 1>), grid, block, 0, s, vol, P); break;
            case 2: hipLaunchKernelGGL((k_march_ws<B, 2>), grid, block, 0, s, vol, P); break;
            case 3: hipLaunchKernelGGL((k_march_ws<B, 3>), grid, block, kLogTabN * sizeof(LogEnt), s, vol, P); break;
            }
            return hipGetLastError();
        }
        if (B < 8 && P.path == 0) P.path = 2;  // per-ray pipelined for narrow records
        if constexpr (B == 1) {  // baked statistics (vr_stats.hip, bricked planes): paths 2, 7 only
            if (method <= 0) P.path = 2;
        }
        if (P.path == 2 && P.avol && method >= 1 && method <= 3) {
            // views along the volume's y / z on the axis-rows copy (vr_api.cpp
            // ensure_axis_copy): the same march, gathers addressed with its strides
            note_kernel(P.asy == 1 ? "k_march_pipe_yrows" : "k_march_pipe_zrows", B, method);
            Params Q = P;
            Q.sx = P.asx;
            Q.sy = P.asy;
            Q.sz = P.asz;
            switch (method) {
            case 1: hipLaunchKernelGGL((k_march_pipe<B, 1, 3>), grid, block, occupancy_lds(P), s, P.avol, Q); break;
            case 2: hipLaunchKernelGGL((k_march_pipe<B, 2, 3>), grid, block, occupancy_lds(P), s, P.avol, Q); break;
            // (the entropy march's LDS columns and table are part of the request)
            case 3: hipLaunchKernelGGL((k_march_pipe<B, 3, 3>), grid, block, cap_lds(P, P.wg_per_cu, sizeof(EntropyLds<B>)), s, P.avol, Q); break;
            }
            return hipGetLastError();
        }
        if (P.path == 2 && method >= -1 && method <= 3) {
            note_kernel("k_march_pipe", B, method);
            switch (method) {
            case 0:
                if constexpr (B == 1) {
                    // a baked plane's y- / z-rows copy (side and top views, gather8 MODE 4 / 5)
                    if (P.plane_axis == 1) {
                        note_kernel("k_march_pipe_plane_yrows", B, method);
                        hipLaunchKernelGGL((k_march_pipe<1, 0, 4>), grid, block, occupancy_lds(P), s, vol, P);
                    } else if (P.plane_axis == 2) {
                        note_kernel("k_march_pipe_plane_zrows", B, method);
                        hipLaunchKernelGGL((k_march_pipe<1, 0, 5>), grid, block, occupancy_lds(P), s, vol, P);
                    } else if (P.plane_axis == 3) {  // 8 x 2 x 2 brick copy (MODE 6)
                        note_kernel("k_march_pipe_plane8", B, method);
                        hipLaunchKernelGGL((k_march_pipe<1, 0, 6>), grid, block, occupancy_lds(P), s, vol, P);
                    } else {
                        hipLaunchKernelGGL((k_march_pipe<1, 0>), grid, block, occupancy_lds(P), s, vol, P);
                    }
                    break;
                }
                return hipErrorInvalidValue;
            case -1:
                if constexpr (B == 1) {
                    hipLaunchKernelGGL((k_march_pipe<1, -1>), grid, block, occupancy_lds(P), s, vol, P);
                    break;
                }
                return hipErrorInvalidValue;
            case 1: hipLaunchKernelGGL((k_march_pipe<B, 1>), grid, block, occupancy_lds(P), s, vol, P); break;
            case 2: hipLaunchKernelGGL((k_march_pipe<B, 2>), grid, block, occupancy_lds(P), s, vol, P); break;
            case 3: hipLaunchKernelGGL((k_march_pipe<B, 3>), grid, block, cap_lds(P, P.wg_per_cu, sizeof(EntropyLds<B>)), s, vol, P); break;
            }
            return hipGetLastError();
        }
    }
    if constexpr (!COUNT && (B == 16 || B == 32)) {
        // wide records, mean / variance: the quad-cooperative march (k_march_wq),
        // except row-aligned views of 16-bin records, whose lane-owned 64-B records
        // already sit side by side (k_march_wide; 1024^3 x 16 C0 2.79 vs 3.90 ms;
        // profiles/r02/wide_records.log).  VR_WIDE=1 / 2 forces one; VR_PATH=1 and
        // coarse row-aligned full frames keep the LDS box (vr_api.cpp).  Entropy
        // stays on k_march: unrolled over a batch its per-bin logarithms need more
        // than 256 VGPRs (B = 16: 512 + spills).
        if (P.path != 1 && (method == 1 || method == 2 || (method == 3 && WQ3))) {
            // an occupancy cap's LDS request leaves room for the kernel's static LDS
            // (the entropy march's log table and record columns)
            const size_t wl = cap_lds(P, P.wg_per_cu, 0,
                                      method == 3 ? kLogTabN * sizeof(LogEnt) + (B >= 32 ? 4 * 64 * B * sizeof(float) : 4) : 64);
            int kind = (B == 16 && !P.oblique && method != 3) ? 1 : 2;
            if (const char *ew = tuning("VR_WIDE")) {
                const int v = std::atoi(ew);
                if (v == 1 || v == 2) kind = v;
            }
            if (method == 3) kind = 2;  // k_march_wide: mean and variance only
            // k_march_wq pixels: 16x4 blocks per wave (a quad = a pixel column) beat a
            // 64-pixel row per wave: 1024^3 x 32 C1 12.44 -> 11.77 ms, C0 6.64 -> 6.56,
            // 1024^3 x 16 C1 6.78 -> 6.65 (profiles/r02/wide_records.log); VR_WQ_MAP=0: rows
            P.wq_map = 1;
            if (const char *em = tuning("VR_WQ_MAP")) P.wq_map = std::atoi(em) != 0;
            if (kind == 1) {
                note_kernel("k_march_wide", B, method);
                // a 16x4 pixel block per wave (1024^3 x 16 1080p C0 m1 2.719 -> 2.673
                // ms, profiles/r06/segmap/wide_1024x16.log); VR_WIDE_MAP=0: rows
                P.seg_map = 1;
                if (const char *em = tuning("VR_WIDE_MAP")) P.seg_map = std::atoi(em) != 0;
                if (method == 1)
                    hipLaunchKernelGGL((k_march_wide<B, 1>), grid, block, wl, s, vol, P);
                else
                    hipLaunchKernelGGL((k_march_wide<B, 2>), grid, block, wl, s, vol, P);
            } else {
                note_kernel("k_march_wq", B, method);
                if (method == 1)
                    hipLaunchKernelGGL((k_march_wq<B, 1>), grid, block, wl, s, vol, P);
                else if (method == 2)
                    hipLaunchKernelGGL((k_march_wq<B, 2>), grid, block, wl, s, vol, P);
                else if constexpr (WQ3)
                    hipLaunchKernelGGL((k_march_wq<B, 3>), grid, block, wl, s, vol, P);
            }
            return hipGetLastError();
        }
    }
    if (!COUNT) note_kernel("k_march", B, method);
    if (method >= 1 && method <= 3) {
        // the LDS-box march: a wave takes a 16x4-pixel block, whose footprint box is
        // compact (512^3 x 8 C0 1080p: ~70 voxels per wave-step instead of
        // ~140-210 for a 64-pixel row): m1 0.869 -> 0.723 ms, m2 0.760 -> 0.627
        // (profiles/r03/box_map.log); VR_BOX_MAP=0 keeps the rows
        P.wq_map = 1;
        if (const char *em = tuning("VR_BOX_MAP")) P.wq_map = std::atoi(em) != 0;
    }
    if constexpr (!COUNT && B > 0 && B <= 8) {
        // P.duo samples per footprint box (k_march_duo; fill_params: coarse
        // row-aligned 8-bin full frames, VR_DUO)
        const int k = P.duo;
        if (k >= 2 && k <= 4 && (method == 1 || method == 2) && P.box_max > 0) {
            note_kernel(k == 2 ? "k_march_duo" : k == 3 ? "k_march_duo3" : "k_march_duo4", B, method);
#define VR_DUO_L(MM, KK) hipLaunchKernelGGL((k_march_duo<B, MM, KK>), grid, block, lds, s, vol, P)
            switch (k * 4 + method) {
            case 9: VR_DUO_L(1, 2); break;
            case 10: VR_DUO_L(2, 2); break;
            case 13: VR_DUO_L(1, 3); break;
            case 14: VR_DUO_L(2, 3); break;
            case 17: VR_DUO_L(1, 4); break;
            case 18: VR_DUO_L(2, 4); break;
            }
#undef VR_DUO_L
            return hipGetLastError();
        }
    }
    switch (method) {
    case 0:
    case -1:  // baked statistics: the pipelined / segmented marches only (bricked planes)
        return hipErrorInvalidValue;
    case 1: hipLaunchKernelGGL((k_march<B, 1, COUNT>), grid, block, lds, s, vol, P); break;
    case 2: hipLaunchKernelGGL((k_march<B, 2, COUNT>), grid, block, lds, s, vol, P); break;
    case 3: hipLaunchKernelGGL((k_march<B, 3, COUNT>), grid, block, lds, s, vol, P); break;
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
    if (method == 7 || method == -7)  // corner-mean state along the ray: vr_m7.hip
        return count ? hipErrorInvalidValue : launch_march_m7(nb, method, vol, P, nslots, s);
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
