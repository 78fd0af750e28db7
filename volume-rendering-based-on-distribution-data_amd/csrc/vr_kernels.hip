// vr_kernels.hip -- gfx950 kernels of the distribution-volume ray caster.
//
//  k_march<B, M, COUNT>  the d_render per-ray march (K:272-717) for methods
//                        1/2/3: one lane per ray, one 8x8 ray block per wave,
//                        one 64x4-pixel tile per 256-thread workgroup,
//                        XCD-aware tile order.  Per step the statistic is
//                        decoded from the 8 corner distribution records and
//                        blended with 8-bit filter weights; when the wave's
//                        footprint box fits its LDS slice the box is loaded
//                        coalesced and every voxel decoded once (staged path),
//                        otherwise each lane gathers its own corners.
//  k_march_m7<B>         method 7, software-interpolated corner means
//                        (K:320-367, 395-480), stateful along the ray.
//  k_synth               the synthetic distribution volume, written in HBM.
//  k_unscatter           rank-0 frame assembly of gathered tiles.
//  k_popcount            footprint bitset -> U.
//
// K = volumeRender_kernel.cu of the reference.
#include "vr_device.h"
#include "vr_internal.h"
#include "vr_march.h"

#include <algorithm>
#include <cstdlib>
#include <cstdio>

namespace vr {


static char g_last_kernel[64] = "";

void note_kernel(const char *kind, int B, int method) {
    snprintf(g_last_kernel, sizeof g_last_kernel, "%s<B=%d,M=%d>", kind, B, method);
}

const char *last_march_kernel() { return g_last_kernel; }

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

// Compile-time tuning knobs (tools/build_variants.sh builds sweeps of them).
#ifndef VR_DIRECT_CG
#define VR_DIRECT_CG 8      // corners gathered before decoding, direct path
#endif
#ifndef VR_BOX_G
#define VR_BOX_G 4          // box voxels per lane in flight, staged path
#endif

// Direct path: each lane gathers and decodes its own 8 corner records, CGMAX
// corners in flight.
template <int B, int M, int CGMAX = VR_DIRECT_CG>
__device__ __forceinline__ float sample_direct_cg(const float *__restrict__ vol, const Params &P,
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

template <int B, int M>
__device__ __forceinline__ float sample_direct(const float *__restrict__ vol, const Params &P,
                                               const Foot &f, const LogEnt *tab = nullptr,
                                               float *st = nullptr) {
    return sample_direct_cg<B, M, VR_DIRECT_CG>(vol, P, f, tab, st);
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

// NG groups of 64 box voxels from position p0: all NG loads issue before the
// first decode waits on them
// ZT: the box's slices are a subset of its z range (k_march_duo, slice_table):
// slot z of the box holds slice (ztab >> 4 z) & 15 of the range
template <int B, int M, int NG, bool ZT = false>
__device__ __forceinline__ void box_chunk(const float *__restrict__ vbase, const Params &P,
                                          float *box, int dx, int dxy, int V, uint32_t lane,
                                          int p0, float rdx, float rdxy, const LogEnt *tab,
                                          float *st, uint64_t ztab = 0) {
    const uint32_t sy = (uint32_t)P.sy;
    float rec[NG][B];
#pragma unroll
    for (int g = 0; g < NG; g++) {
        const int p = min(p0 + g * 64 + (int)lane, V - 1);
        const int zs = (int)(((float)p + 0.5f) * rdxy);
        const int r = p - zs * dxy;
        const int y = (int)(((float)r + 0.5f) * rdx);
        const int x = r - y * dx;
        const int z = ZT ? (int)((ztab >> (4 * zs)) & 15u) : zs;
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
template <int B, int M, bool ZT = false>
__device__ __forceinline__ void decode_box(const float *__restrict__ vbase, const Params &P,
                                           float *box, int dx, int dxy, int V, uint32_t lane,
                                           const LogEnt *tab, float *st, uint64_t ztab = 0) {
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
            box_chunk<B, M, (G >= 4 ? 4 : 1), ZT>(vbase, P, box, dx, dxy, V, lane, p0, rdx, rdxy, tab, st, ztab);
        else if (G >= 3 && left > 128)
            box_chunk<B, M, (G >= 3 ? 3 : 1), ZT>(vbase, P, box, dx, dxy, V, lane, p0, rdx, rdxy, tab, st, ztab);
        else if (G >= 2 && left > 64)
            box_chunk<B, M, (G >= 2 ? 2 : 1), ZT>(vbase, P, box, dx, dxy, V, lane, p0, rdx, rdxy, tab, st, ztab);
        else
            box_chunk<B, M, 1, ZT>(vbase, P, box, dx, dxy, V, lane, p0, rdx, rdxy, tab, st, ztab);
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
// (dx dy dz, or dx dy x the used slices of a slice-compacted box); slices:
// the footprint's slices are among the box's (slice-compacted boxes)
__device__ __forceinline__ bool box_ok(const Params &P, const Foot &f, int bx0, int by0, int bz0,
                                       int dx, int dy, int dz, int hi, int V, bool slices = true) {
    const bool ok = slices && f.x0 >= bx0 && f.y0 >= by0 && f.z0 >= bz0 && f.x1 >= f.x0 &&
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
        st = lds + 4u * (uint32_t)P.box_max + 65u * (sizeof(LogEnt) / 4u) + (threadIdx.x >> 6) * 64u * B;
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

// OR over the 64 lanes (DPP row shifts, then row broadcasts; lane 63 holds it)
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
    int x = (int)v;
    x |= __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);
    x |= __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);
    x |= __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);
    x |= __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);
    x |= __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);
    x |= __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);
    return (uint32_t)__builtin_amdgcn_readlane(x, 63);
}

// the used slices of a box's z range (bit z of mask) packed as 4-bit offsets,
// slot s -> slice (table >> 4 s) & 15 (wave-uniform; ranges of <= 16 slices)
__device__ __forceinline__ uint64_t slice_table(uint32_t mask) {
    uint64_t t = 0;
    int s = 0;
    for (int z = 0; z < 16; z++)
        if ((mask >> z) & 1u) t |= (uint64_t)z << (4 * s++);
    return t;
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
// first sample leaves the second unread): the frame is bit-identical.  Entropy
// (M = 3) decodes through the LDS log table and the rolled record columns of
// k_march (same LDS request); its round-4 fault is DESIGN.md 4.2.1.
template <int B, int M, int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_MARCH_MINW, 8))) void k_march_duo(const float *__restrict__ vol, Params P) {
    static_assert(M >= 1 && M <= 3, "mean, variance, entropy");
    static_assert(K >= 2 && K <= 4, "samples per box");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;  // whole workgroup uniform
    const LogEnt *tab = nullptr;
    float *st = nullptr;
    if constexpr (M == 3 && B >= 8) {  // k_march's entropy layout behind the box slices
        LogEnt *tb = reinterpret_cast<LogEnt *>(lds + 4u * (uint32_t)P.box_max);
        copy_logtab(tb);
        __syncthreads();
        tab = tb;
        st = lds + 4u * (uint32_t)P.box_max + 65u * (sizeof(LogEnt) / 4u) + (threadIdx.x >> 6) * 64u * B;
    }
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
        uint32_t incl = alive ? 1u : 0u;  // the samples whose footprints the box covers
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
                    incl |= 1u << k;
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
        // P.duo_compact (VR_DUO_COMPACT=1, off by default): the box keeps only
        // the slices some footprint reads -- K samples a step apart leave
        // slices between them that none does (512^3: a step is 2.56 slices, so
        // {z, z+1} and {z+3, z+4} skip z+2).  Ranges of <= 16 slices are
        // compacted (slot -> slice through slice_table).  It decodes 6 % fewer
        // voxels at 512^3 C0 but the table and slot counts cost more: 0.624 ->
        // 0.681 ms.
        const bool compact = dz <= 16 && P.duo_compact;  // wave-uniform
        uint32_t zmask = (1u << min(dz, 31)) - 1u;
        uint64_t ztab = 0;
        if (compact) {
            uint32_t m = 0;
#pragma unroll
            for (int k = 0; k < K; k++)
                if ((incl >> k) & 1u) m |= (1u << (f[k].z0 - bz0)) | (1u << (f[k].z1 - bz0));
            zmask = wave_or(m);
            ztab = slice_table(zmask);
        }
        const int nzs = compact ? __builtin_popcount(zmask) : dz;
        const int dxy = dx * dy;
        const int V = dxy * nzs;
#ifdef VR_BOX_CHECK
        const bool staged = V <= P.box_max && box_in_volume(P, bx0, by0, bz0, dx, dy, dz, lane);
#else
        const bool staged = V <= P.box_max;  // wave-uniform
#endif
        if (staged) {
            const float *vbase =
                vol + ((uint64_t)bz0 * P.sz + (uint64_t)by0 * P.sy + (uint64_t)bx0) * (uint64_t)B;
            if (compact)
                decode_box<B, M, true>(vbase, P, box, dx, dxy, V, lane, tab, st, ztab);
            else
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
                // the footprint's slices z0, z1 (= z0 or z0 + 1) sit in adjacent slots
                const int zs0 = compact ? __builtin_popcount(zmask & ((1u << (fk.z0 - bz0)) - 1u))
                                        : fk.z0 - bz0;
                const int b0 = (zs0 * dy + (fk.y0 - by0)) * dx + (fk.x0 - bx0);
                const int ox = fk.x1 - fk.x0, oy = (fk.y1 - fk.y0) * dx;
                const int oz = (fk.z1 - fk.z0) * dxy;
#ifdef VR_BOX_CHECK
                if (staged && !box_ok(P, fk, bx0, by0, bz0, dx, dy, dz, b0 + oz + oy + ox, V,
                                      !compact || ((zmask >> (fk.z0 - bz0)) &
                                                   (zmask >> (fk.z1 - bz0)) & 1u))) {
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

// ---- the workgroup-box march (k_march_wgbox) ----
// k_march_duo's boxes are per wave (16 x 4 pixels).  At 512^3 x 8, 1080p, C0 a
// wave's ~8 x 2 footprint centres need a box of ~9 x 3.4 voxels per slice, and
// the rows it shares with the tile below -- another workgroup, steps ahead or
// behind -- are fetched again: the frame decodes ~2.1 voxels per voxel of U
// and its fabric traffic is 1.98 x the algorithmic bytes.
// Here a workgroup of R x 256 lanes takes R vertically adjacent tiles (64 x 4R
// pixels, a 16 x 4 block per wave) and marches them in lockstep: per step the
// union box of all its lanes' K footprints is fetched and decoded once, by all
// lanes together, into one LDS box; then every lane blends its own samples.
// Samples, their order and the compositing are k_march_duo's (bit-identical).
// Each step: the waves' bounds meet through LDS minima (three rotating sets:
// set s is cleared two steps before its reuse, so one barrier orders it),
// a barrier, the decode, a barrier, the samples.  A union box larger than
// P.box_wg voxels (the first steps of rays entering far apart) samples directly.
template <int B, int M, int NG>
__device__ __forceinline__ void wg_chunk(const float *__restrict__ vbase, const Params &P, float *box,
                                         int dx, int dxy, int V, int p0, int nt, uint32_t tid,
                                         float rdx, float rdxy, const LogEnt *tab = nullptr,
                                         float *st = nullptr) {
    const uint32_t sy = (uint32_t)P.sy;
    float rec[NG][B];
#pragma unroll
    for (int g = 0; g < NG; g++) {
        const int p = min(p0 + g * nt + (int)tid, V - 1);  // clamped: every load issues
        const int z = (int)(((float)p + 0.5f) * rdxy);
        const int r = p - z * dxy;
        const int y = (int)(((float)r + 0.5f) * rdx);
        const int x = r - y * dx;
        load_rec<B>(vbase, (uint64_t)(uint32_t)z * P.sz + (uint32_t)(y * sy + x), rec[g]);
    }
#pragma unroll
    for (int g = 0; g < NG; g++) {
        const int p = p0 + g * nt + (int)tid;
        if (p < V) box[p] = box_stat<B, M>(rec[g], P, st, tid & 63u, tab);
    }
}

// Entropy (M = 3, 8 bins, K = 1: one sample per box, as k_march<8,3>): the
// decode is most of the frame's VALU, and the union box of R tile rows decodes
// ~20 % fewer slots per wave-step than the per-wave boxes;
// k_march's LDS log table and per-wave record columns (entropy_stash) sit at
// the front of the LDS.
template <int B, int M, int K, int R>
__global__ __launch_bounds__(256 * R) __attribute__((amdgpu_waves_per_eu(M == 3 ? 4 : 1, 8))) void k_march_wgbox(const float *__restrict__ vol, Params P) {
    static_assert(M == 1 || M == 2 || (M == 3 && B == 8 && K == 1), "mean, variance; 8-bin entropy");
    static_assert(K >= 1 && K <= 4 && (R == 2 || R == 4), "samples per box, tile rows");
    constexpr int NT = 256 * R;
    // voxels per lane in flight (entropy: one, within 128 VGPRs)
    constexpr int G = M == 3 ? 1 : (B >= 8 ? 2 : 4);
    extern __shared__ __attribute__((aligned(32))) float lds[];
    const LogEnt *tab = nullptr;
    float *st = nullptr;
    float *base = lds;
    if constexpr (M == 3) {  // [log table][R x 4 waves' record columns][bounds][box]
        LogEnt *tb = reinterpret_cast<LogEnt *>(lds);
        copy_logtab(tb);
        tab = tb;
        st = lds + 65u * (sizeof(LogEnt) / 4u) + (threadIdx.x >> 6) * 64u * B;
        base = lds + 65u * (sizeof(LogEnt) / 4u) + 4u * R * 64u * B;
    }
    int *red = reinterpret_cast<int *>(base);  // 3 sets x 8: min lo x/y/z, min -hi x/y/z
    float *box = base + 24;
    // the group's top tile: an entry of the grouped frame order, or raster groups
    uint32_t top;
    if (P.perm) {
        top = P.perm[blockIdx.x];
    } else {
        const uint32_t gi = xcd_slot(blockIdx.x, gridDim.x);
        top = (gi / P.tiles_x) * R * P.tiles_x + gi % P.tiles_x;
    }
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    const uint32_t lx = (w & 3u) * 16u + (lane >> 2), ly = (w >> 2) * kTileH + (lane & 3u);
    const uint32_t x = (top % P.tiles_x) * kTileW + lx;
    const uint32_t y = (top / P.tiles_x) * kTileH + ly;
    const bool valid = x < P.CW && y < P.CH;
    const uint64_t o = (uint64_t)y * P.W + x;
    if (tid < 24) red[tid] = 0x7FFFFFFF;
    Ray r;
    bool alive = valid && make_ray(P, x, y, r);
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = r.tnear;
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
    int n = 0;
    __syncthreads();
    int set = 0;
    for (int i = 0; i < kMaxSteps; i += K) {
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
        int *rs = red + 8 * set;
        if (lane == 0 && lo_x != 0x7FFFFFFF) {  // a wave with a live lane
            atomicMin(rs + 0, lo_x);
            atomicMin(rs + 1, lo_y);
            atomicMin(rs + 2, lo_z);
            atomicMin(rs + 3, hi_x);
            atomicMin(rs + 4, hi_y);
            atomicMin(rs + 5, hi_z);
        }
        __syncthreads();
        // workgroup-uniform: scalar registers
        const int bx0 = __builtin_amdgcn_readfirstlane(rs[0]);
        const int by0 = __builtin_amdgcn_readfirstlane(rs[1]);
        const int bz0 = __builtin_amdgcn_readfirstlane(rs[2]);
        const int nhx = __builtin_amdgcn_readfirstlane(rs[3]);
        const int nhy = __builtin_amdgcn_readfirstlane(rs[4]);
        const int nhz = __builtin_amdgcn_readfirstlane(rs[5]);
        // set + 2 (mod 3) was read last step, before this barrier, and is next
        // written two steps on, after the next barrier
        const int clr = set == 0 ? 2 : set - 1;
        if (tid < 6) red[8 * clr + tid] = 0x7FFFFFFF;
        set = set == 2 ? 0 : set + 1;
        if (bx0 == 0x7FFFFFFF) break;  // no live ray in the workgroup (uniform)
        const int bx1 = min(-nhx + 1, P.nx - 1);
        const int by1 = min(-nhy + 1, P.ny - 1);
        const int bz1 = min(-nhz + 1, P.nz - 1);
        const int dx = bx1 - bx0 + 1, dy = by1 - by0 + 1, dz = bz1 - bz0 + 1;
        const int dxy = dx * dy;
        const int V = dxy * dz;
        const bool staged = V <= P.box_wg;  // workgroup-uniform
        if (staged) {
            const float *vbase =
                vol + ((uint64_t)bz0 * P.sz + (uint64_t)by0 * P.sy + (uint64_t)bx0) * (uint64_t)B;
            const float rdx = __builtin_amdgcn_rcpf((float)dx), rdxy = __builtin_amdgcn_rcpf((float)dxy);
            for (int p0 = 0; p0 < V; p0 += NT * G) {
                if (V - p0 > NT)
                    wg_chunk<B, M, G>(vbase, P, box, dx, dxy, V, p0, NT, tid, rdx, rdxy, tab, st);
                else
                    wg_chunk<B, M, 1>(vbase, P, box, dx, dxy, V, p0, NT, tid, rdx, rdxy, tab, st);
            }
            __syncthreads();
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            if (alive) {  // the ray reached this sample (t <= tfar): f[k] is in the box
                const Foot &fk = f[k];
                float sample;
                if (staged) {
                    const int b0 = ((fk.z0 - bz0) * dy + (fk.y0 - by0)) * dx + (fk.x0 - bx0);
                    const int ox = fk.x1 - fk.x0, oy = (fk.y1 - fk.y0) * dx;
                    const int oz = (fk.z1 - fk.z0) * dxy;
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
                    sample = sample_direct_cg<B, M, M == 3 ? 2 : VR_DIRECT_CG>(vol, P, fk, tab, st);  // (rare: registers)
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
        // the next step's decode rewrites the box only after its barrier, which
        // every wave reaches after these reads
    }
    if (!valid) return;
    if (n == 0) {  // miss (K:302-303): nothing written
        write_miss(P, o);
        return;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
}

// Union bounds (minima of lo, minima of -hi, per axis) of the footprints of
// samples skip .. skip + K - 1 ahead of this lane's current one, over those the
// ray reaches by tfar (K:700-705) -- the same float adds the samples take, so
// the footprints are the ones the march will read.  Rays that end by opacity
// before them are still counted (a superset: a box is never too small).
template <int K>
__device__ __forceinline__ void union_feet(const Params &P, bool alive, float t, float tfar,
                                           float px, float py, float pz, float stx, float sty,
                                           float stz, int i, int skip, int (&lo)[3], int (&nhi)[3]) {
    lo[0] = lo[1] = lo[2] = nhi[0] = nhi[1] = nhi[2] = 0x7FFFFFFF;
    bool reach = alive;
    float tq = t, qx = px, qy = py, qz = pz;
    for (int m = 0; m < skip + K; m++) {
        if (m > 0) {
            tq = tq + kTStep;
            reach = reach && !(tq > tfar) && i + m < kMaxSteps;
            qx = qx + stx;
            qy = qy + sty;
            qz = qz + stz;
        }
        if (m >= skip && reach) {
            const Foot f = footprint(P, qx, qy, qz);
            lo[0] = min(lo[0], f.x0);
            lo[1] = min(lo[1], f.y0);
            lo[2] = min(lo[2], f.z0);
            nhi[0] = min(nhi[0], -f.x0);
            nhi[1] = min(nhi[1], -f.y0);
            nhi[2] = min(nhi[2], -f.z0);
        }
    }
    dpp_min3(lo[0], lo[1], lo[2]);
    dpp_min3(nhi[0], nhi[1], nhi[2]);
}

// The workgroup box march with the next box in flight (k_march_wgpipe, R = 2):
// k_march_wgbox waits, every step, for the slowest of its waves' box loads
// behind two barriers with nothing to overlap them.  Here the union box of the
// NEXT K samples is bounded first (positions K steps ahead, same float adds),
// its first 512 G voxels are loaded into registers (G per lane), this step's
// samples are blended from the current decoded box while those loads fly, and
// only then are they decoded into the other LDS box (a larger box's remaining
// voxels, up to P.box_wg, are loaded and decoded after them).  One step:
// bounds -> barrier -> issue loads -> samples -> decode -> barrier.
// Bit-identical to k_march_duo.
template <int B, int M, int K, int R>
__global__ __launch_bounds__(256 * R) __attribute__((amdgpu_waves_per_eu(M == 1 || B < 8 ? 4 : 2, 8))) void k_march_wgpipe(const float *__restrict__ vol, Params P) {
    static_assert(M == 1 || M == 2, "mean, variance");
    static_assert(K >= 2 && K <= 4 && R == 2, "samples per box, tile rows");
    constexpr int NT = 256 * R;
    constexpr int G = B >= 8 ? 2 : 4;  // voxels per lane in flight during the samples
    constexpr int PRE = NT * G;
    const int CAP = P.box_wg;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    int *red = reinterpret_cast<int *>(lds);  // 3 sets x 8 (k_march_wgbox)
    float *stat = lds + 24;                   // two decoded boxes of CAP voxels
    uint32_t top;
    if (P.perm) {
        top = P.perm[blockIdx.x];
    } else {
        const uint32_t gi = xcd_slot(blockIdx.x, gridDim.x);
        top = (gi / P.tiles_x) * R * P.tiles_x + gi % P.tiles_x;
    }
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    const uint32_t lx = (w & 3u) * 16u + (lane >> 2), ly = (w >> 2) * kTileH + (lane & 3u);
    const uint32_t x = (top % P.tiles_x) * kTileW + lx;
    const uint32_t y = (top / P.tiles_x) * kTileH + ly;
    const bool valid = x < P.CW && y < P.CH;
    const uint64_t o = (uint64_t)y * P.W + x;
    if (tid < 24) red[tid] = 0x7FFFFFFF;
    Ray r;
    bool alive = valid && make_ray(P, x, y, r);
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    float t = r.tnear;
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
    int n = 0;
    const uint32_t syp = (uint32_t)P.sy;
    float rec[G][B];
    // the box a step reads: origin, extent, voxels; V = 0 = sample directly
    int bx0 = 0, by0 = 0, bz0 = 0, dx = 1, dy = 1, V = 0;
    bool more = true;  // some lane reaches the box
    // bounds of the box `skip` steps ahead -> set s; the next box's origin /
    // extent / voxels (0 when larger than CAP) and whether any lane reaches it
    int set = 0;
    auto next_box = [&](int i, int skip, int &nx0, int &ny0, int &nz0, int &ndx, int &ndy, int &nV) {
        int lo[3], nhi[3];
        union_feet<K>(P, alive, t, r.tfar, px, py, pz, stx, sty, stz, i, skip, lo, nhi);
        int *rs = red + 8 * set;
        if (lane == 0 && lo[0] != 0x7FFFFFFF) {
            atomicMin(rs + 0, lo[0]);
            atomicMin(rs + 1, lo[1]);
            atomicMin(rs + 2, lo[2]);
            atomicMin(rs + 3, nhi[0]);
            atomicMin(rs + 4, nhi[1]);
            atomicMin(rs + 5, nhi[2]);
        }
        __syncthreads();
        // workgroup-uniform: scalar registers
        nx0 = __builtin_amdgcn_readfirstlane(rs[0]);
        ny0 = __builtin_amdgcn_readfirstlane(rs[1]);
        nz0 = __builtin_amdgcn_readfirstlane(rs[2]);
        const int hx = __builtin_amdgcn_readfirstlane(rs[3]);
        const int hy = __builtin_amdgcn_readfirstlane(rs[4]);
        const int hz = __builtin_amdgcn_readfirstlane(rs[5]);
        const int clr = set == 0 ? 2 : set - 1;  // read last step, written two steps on
        if (tid < 6) red[8 * clr + tid] = 0x7FFFFFFF;
        set = set == 2 ? 0 : set + 1;
        if (nx0 == 0x7FFFFFFF) return false;
        ndx = min(-hx + 1, P.nx - 1) - nx0 + 1;
        ndy = min(-hy + 1, P.ny - 1) - ny0 + 1;
        const int ndz = min(-hz + 1, P.nz - 1) - nz0 + 1;
        nV = ndx * ndy * ndz;
        if (nV > CAP) nV = 0;
        return true;
    };
    auto issue = [&](int nx0, int ny0, int nz0, int ndx, int ndy, int nV, int p0) {
        const float *vbase =
            vol + ((uint64_t)nz0 * P.sz + (uint64_t)ny0 * P.sy + (uint64_t)nx0) * (uint64_t)B;
        const int ndxy = ndx * ndy;
        const float rdx = __builtin_amdgcn_rcpf((float)ndx), rdxy = __builtin_amdgcn_rcpf((float)ndxy);
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int p = min(p0 + g * NT + (int)tid, nV - 1);  // clamped: every load issues
            const int z = (int)(((float)p + 0.5f) * rdxy);
            const int rr = p - z * ndxy;
            const int yy = (int)(((float)rr + 0.5f) * rdx);
            const int xx = rr - yy * ndx;
            load_rec<B>(vbase, (uint64_t)(uint32_t)z * P.sz + (uint32_t)(yy * syp + xx), rec[g]);
        }
    };
    auto decode = [&](float *dst, int nV, int p0) {
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int p = p0 + g * NT + (int)tid;
            if (p < nV) dst[p] = record_stat<B, M>(rec[g], P.enorm);
        }
    };
    // the voxels past the first PRE (boxes larger than the registers hold)
    auto rest = [&](float *dst, int nx0, int ny0, int nz0, int ndx, int ndy, int nV) {
        for (int p0 = PRE; p0 < nV; p0 += PRE) {
            issue(nx0, ny0, nz0, ndx, ndy, nV, p0);
            decode(dst, nV, p0);
        }
    };
    __syncthreads();  // the bound sets are initialised
    {  // prologue: the first box, loaded and decoded synchronously
        int nx0 = 0, ny0 = 0, nz0 = 0, ndx = 1, ndy = 1, nV = 0;
        more = next_box(0, 0, nx0, ny0, nz0, ndx, ndy, nV);
        if (more && nV) {
            issue(nx0, ny0, nz0, ndx, ndy, nV, 0);
            decode(stat, nV, 0);
            rest(stat, nx0, ny0, nz0, ndx, ndy, nV);
        }
        bx0 = nx0; by0 = ny0; bz0 = nz0; dx = ndx; dy = ndy; V = more ? nV : 0;
        __syncthreads();
    }
    int cur = 0;
    for (int i = 0; more && i < kMaxSteps; i += K) {
        // the next box: bounded, then its loads in flight during this step's samples
        int nx0 = 0, ny0 = 0, nz0 = 0, ndx = 1, ndy = 1, nV = 0;
        const bool next = i + K < kMaxSteps && next_box(i, K, nx0, ny0, nz0, ndx, ndy, nV);
        if (next && nV) issue(nx0, ny0, nz0, ndx, ndy, nV, 0);
        const float *box = stat + cur * CAP;
        const int dxy = dx * dy;
#pragma unroll 1  // (unrolled, the 8-bin mean needs one VGPR too many at 4 waves per SIMD)
        for (int k = 0; k < K; k++) {
            if (alive) {  // the ray reached this sample: its footprint is in the box
                const Foot fk = footprint(P, px, py, pz);
                float sample;
                if (V) {
                    const int b0 = ((fk.z0 - bz0) * dy + (fk.y0 - by0)) * dx + (fk.x0 - bx0);
                    const int ox = fk.x1 - fk.x0, oy = (fk.y1 - fk.y0) * dx;
                    const int oz = (fk.z1 - fk.z0) * dxy;
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
                    sample = sample_direct<B, M>(vol, P, fk);
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
        if (next && nV) {
            decode(stat + (cur ^ 1) * CAP, nV, 0);
            rest(stat + (cur ^ 1) * CAP, nx0, ny0, nz0, ndx, ndy, nV);
        }
        __syncthreads();  // the next box is decoded; this one is free
        cur ^= 1;
        more = next;
        bx0 = nx0; by0 = ny0; bz0 = nz0; dx = ndx; dy = ndy; V = next ? nV : 0;
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
// DESIGN.md 4.3), so the 16-20 resident waves of a CU
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
            if (!staged) sample = sample_direct_cg<B, M, 2>(vol, P, f);
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
    tile_pixel(tid, lx, ly);
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
    __shared__ LogEnt s_lt[M == 3 ? 65 : 1];  // entropy: the exact-log table (copy_logtab)
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

#ifndef VR_QUAD_WAVES
#define VR_QUAD_WAVES 1  // minimum waves per SIMD the register allocation must allow
#endif
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

// ---- methods 4/5/6: fractal/template codec volume ----
// The reference pre-bakes the decoded statistics into fractalQueryTex
// (K:775-871) and samples it with the texture trilinear (K:639-652); here, as
// for methods 1/2/3, each of the 8 corners is decoded from its codebook entry,
// template and sparse errors at every step and blended with the quantised
// weights.  One lane per ray.
//
// Decode of one corner (codec_decode_pre's arithmetic, vr_device.h): the
// template row -- from LDS when the table is staged there (TL), read with LDS
// instructions rather than generic loads -- flipped and circularly shifted
// (fractalDecoding, K:195-222); the NE sparse errors (K:805-823) are applied
// through the thread's own LDS scratch column (bin i at scr[i * 256]: a lane's
// dynamic bin index never conflicts with another lane's bank), one
// read-add-clamp-write per error instead of a compare-and-select over every
// bin; then renormalised (K:826-835).
template <int B, bool TL>
__device__ __forceinline__ void codec_decode_scr(const Params &P, const float *s_tpl, float *scr,
                                                 const int4 c, const float4 (&pre)[2],
                                                 const float2 *e, float (&dec)[B]) {
    const uint32_t row = (uint32_t)c.x * B;
#pragma unroll
    for (int m = 0; m < B; m++) {
        int i = m - c.y;                    // dec[(i + shift) mod B] = src[i]
        if (i < 0) i += B;
        const uint32_t k = row + (uint32_t)(c.z ? B - 1 - i : i);
        dec[m] = TL ? s_tpl[k] : P.tpl[k];
    }
    if (c.w > 0) {
#pragma unroll
        for (int m = 0; m < B; m++) scr[m * 256] = dec[m];
        for (int j = 0; j < c.w; j++) {
            float2 ev;
            if (j < kCodecPre) {
                const float4 h = pre[j >> 1];
                ev = (j & 1) ? make_float2(h.z, h.w) : make_float2(h.x, h.y);
            } else {
                ev = e[j];
            }
            const int idx = (int)ev.x;
            if (idx >= 0 && idx < B) {      // bin ids outside [0, B) skipped
                float v = scr[idx * 256] + ev.y;
                if (v < 0) v = 0;
                scr[idx * 256] = v;
            }
        }
#pragma unroll
        for (int m = 0; m < B; m++) dec[m] = scr[m * 256];
    }
    float total = 0.0f;
#pragma unroll
    for (int i = 0; i < B; i++) total = total + dec[i];
    if (total > 0) {
#pragma unroll
        for (int i = 0; i < B; i++) dec[i] = dec[i] / total;
    }
}

template <int B, int C, bool COUNT, bool TL>
__global__ __launch_bounds__(256) void k_march_codec(const float *__restrict__ unused, Params P) {
    (void)unused;
    extern __shared__ __attribute__((aligned(16))) float s_lds[];
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;  // whole workgroup
    if constexpr (TL) {  // small template tables live in LDS: no gathers for them
        const uint32_t n = (uint32_t)P.tpl_lds / 4;
        for (uint32_t i = threadIdx.x; i < n; i += 256) s_lds[i] = P.tpl[i];
        __syncthreads();
    }
    // this thread's error scratch column, after the (16-byte aligned) template table
    const uint32_t scr0 = TL ? ((uint32_t)P.tpl_lds / 4 + 3u) & ~3u : 0u;
    float *scr = s_lds + scr0 + threadIdx.x;
    // entropy (C == 2): the exact log's table after the scratch (32-byte aligned)
    LogEnt *lt = reinterpret_cast<LogEnt *>(s_lds + ((scr0 + (uint32_t)B * 256u + 7u) & ~7u));
    if constexpr (C == 2) {
        copy_logtab(lt);
        __syncthreads();
    }
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
    // the first kCodecPre error pairs of a voxel are gathered with its codebook
    // entry as two 16-byte loads when the per-voxel block allows (even slot count)
    const bool pre16 = P.err_slots >= kCodecPre && (P.err_slots & 1) == 0;
    const int npre = P.err_slots < kCodecPre ? P.err_slots : kCodecPre;
    int n = 0;
    for (int i = 0; i < kMaxSteps; i++) {
        const Foot f = footprint(P, px, py, pz);
        if constexpr (COUNT) mark_foot(P, f);
        const uint64_t r00 = (uint64_t)f.z0 * P.sz + (uint64_t)f.y0 * P.sy;
        const uint64_t r10 = (uint64_t)f.z0 * P.sz + (uint64_t)f.y1 * P.sy;
        const uint64_t r01 = (uint64_t)f.z1 * P.sz + (uint64_t)f.y0 * P.sy;
        const uint64_t r11 = (uint64_t)f.z1 * P.sz + (uint64_t)f.y1 * P.sy;
        const uint64_t v[8] = {r00 + f.x0, r00 + f.x1, r10 + f.x0, r10 + f.x1,
                               r01 + f.x0, r01 + f.x1, r11 + f.x0, r11 + f.x1};
        // all 8 codebook entries and their first error pairs in one batch
        int4 c[8];
        float4 pre[8][2];
#pragma unroll
        for (int j = 0; j < 8; j++) c[j] = P.cb[v[j]];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float2 *e = P.err + v[j] * (uint64_t)P.err_slots;
            if (pre16) {
                pre[j][0] = reinterpret_cast<const float4 *>(e)[0];
                pre[j][1] = reinterpret_cast<const float4 *>(e)[1];
            } else {
                float2 q[kCodecPre];
#pragma unroll
                for (int k = 0; k < kCodecPre; k++) q[k] = k < npre ? e[k] : make_float2(0.f, 0.f);
                pre[j][0] = make_float4(q[0].x, q[0].y, q[1].x, q[1].y);
                pre[j][1] = make_float4(q[2].x, q[2].y, q[3].x, q[3].y);
            }
        }
        float sv[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            float dec[B];
            codec_decode_scr<B, TL>(P, s_lds, scr, c[j], pre[j],
                                    P.err + v[j] * (uint64_t)P.err_slots, dec);
            // entropy: rolled per-bin sum over the thread's LDS scratch column
            sv[j] = C == 2 ? entropy_col<B, 256>(dec, scr, P.enorm, lt) : codec_stat_of<B, C>(dec, P.enorm);
        }
        n = i + 1;
        if (composite(P, blend8(sv, f), sx, sy, sz, sw)) break;
        t = t + kTStep;
        if (t > r.tfar) break;
        px = px + stx;
        py = py + sty;
        pz = pz + stz;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
}

// ---- methods 4/5/6, quad-cooperative (B == 8, oblique views) ----
// The codec march with the quad march's lane roles (k_march_quad): the 4
// lanes of a quad take turns on their 4 rays; for ray G, lane g fetches and
// decodes the two corners (x = g>>1, y = g&1) at z0 and z1 -- codebook entry
// plus the first 4 error pairs each -- so a quad's loads land on two rows of
// adjacent voxels instead of the 8 scattered corners one lane would fetch
// for its own ray, and every corner is decoded once.  The blend runs inside
// the quad (qc_blend, the reference's lerp order); the next step's corner
// data of group G is fetched into the registers group G has just released.
struct CqPart {
    int4 c[2];
    float4 e[2][2];
};

template <int G>
__device__ __forceinline__ bool cq_gather(const Params &P, const FootPacked &fp, uint32_t g,
                                          bool pre16, int npre, CqPart &d) {
    const int w0 = bcast_g<G>(fp.w0), w1 = bcast_g<G>(fp.w1);
    const bool live = (w1 >> 19) & 1;
    if (live) {
        const uint64_t x = ((uint32_t)w0 & 0xFFFFu) + (g >> 1) * (((uint32_t)w1 >> 16) & 1u);
        const uint64_t y = ((uint32_t)w0 >> 16) + (g & 1u) * (((uint32_t)w1 >> 17) & 1u);
        const uint64_t z0 = (uint32_t)w1 & 0xFFFFu;
        const uint64_t v0 = z0 * P.sz + y * P.sy + x;
        const uint64_t v1 = v0 + (((uint32_t)w1 >> 18) & 1u) * P.sz;
        const uint64_t v[2] = {v0, v1};
#pragma unroll
        for (int k = 0; k < 2; k++) {
            d.c[k] = P.cb[v[k]];
            const float2 *e = P.err + v[k] * (uint64_t)P.err_slots;
            if (pre16) {
                d.e[k][0] = reinterpret_cast<const float4 *>(e)[0];
                d.e[k][1] = reinterpret_cast<const float4 *>(e)[1];
            } else {
                float2 q[kCodecPre];
#pragma unroll
                for (int j = 0; j < kCodecPre; j++) q[j] = j < npre ? e[j] : make_float2(0.f, 0.f);
                d.e[k][0] = make_float4(q[0].x, q[0].y, q[1].x, q[1].y);
                d.e[k][1] = make_float4(q[2].x, q[2].y, q[3].x, q[3].y);
            }
        }
    }
    return live;
}

template <int C, bool TL>
__device__ __forceinline__ float cq_stat(const Params &P, const float *s_tpl, float *scr,
                                         const LogEnt *lt, const int4 c, const float4 (&pre)[2],
                                         uint64_t vox) {
    float dec[8];
    codec_decode_scr<8, TL>(P, s_tpl, scr, c, pre, P.err + vox * (uint64_t)P.err_slots, dec);
    if constexpr (C == 2) return entropy_col<8, 256>(dec, scr, P.enorm, lt);  // rolled, LDS column
    else return codec_stat_of<8, C>(dec, P.enorm);
}

template <int G, int C, bool TL>
__device__ __forceinline__ float cq_group(const Params &P, const float *s_tpl, float *scr,
                                          const LogEnt *lt, const FootPacked &fc, bool lc,
                                          const FootPacked &fn, bool &ln, uint32_t g, bool pre16,
                                          int npre, CqPart &D) {
    // this step's corner data of ray (G, q) out of the registers ...
    const CqPart cur = D;
    // ... which then take the next step's fetches of the same group
    ln = cq_gather<G>(P, fn, g, pre16, npre, D);
    float s0 = 0.0f, s1 = 0.0f;
    if (lc) {
        // the corners' voxel indices again (errors beyond the first 4 pairs are read directly)
        const int w0 = bcast_g<G>(fc.w0), w1 = bcast_g<G>(fc.w1);
        const uint64_t x = ((uint32_t)w0 & 0xFFFFu) + (g >> 1) * (((uint32_t)w1 >> 16) & 1u);
        const uint64_t y = ((uint32_t)w0 >> 16) + (g & 1u) * (((uint32_t)w1 >> 17) & 1u);
        const uint64_t v0 = ((uint32_t)w1 & 0xFFFFu) * P.sz + y * P.sy + x;
        const uint64_t v1 = v0 + (((uint32_t)w1 >> 18) & 1u) * P.sz;
        s0 = cq_stat<C, TL>(P, s_tpl, scr, lt, cur.c[0], cur.e[0], v0);
        s1 = cq_stat<C, TL>(P, s_tpl, scr, lt, cur.c[1], cur.e[1], v1);
    }
    return qc_blend<G>(fc, s0, s1);
}

template <int C, bool TL>
__global__ __launch_bounds__(256) void k_march_codec_quad(const float *__restrict__ unused, Params P) {
    (void)unused;
    extern __shared__ __attribute__((aligned(16))) float s_lds[];
    const uint32_t slot = launch_slot(P);
    const uint32_t tile = tile_of(P, slot);
    if (tile == kPad) return;  // uniform per workgroup
    if constexpr (TL) {
        const uint32_t n = (uint32_t)P.tpl_lds / 4;
        for (uint32_t i = threadIdx.x; i < n; i += 256) s_lds[i] = P.tpl[i];
    }
    const uint32_t scr0 = TL ? ((uint32_t)P.tpl_lds / 4 + 3u) & ~3u : 0u;
    float *scr = s_lds + scr0 + threadIdx.x;
    LogEnt *lt = reinterpret_cast<LogEnt *>(s_lds + ((scr0 + 8u * 256u + 7u) & ~7u));
    if constexpr (C == 2) copy_logtab(lt);
    if constexpr (TL || C == 2) __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t q = lane >> 2, g = lane & 3u;
    const uint32_t lx = wave * 16u + q, ly = g;  // 16x4 block per wave, quad = a column
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
    const bool pre16 = P.err_slots >= kCodecPre && (P.err_slots & 1) == 0;
    const int npre = P.err_slots < kCodecPre ? P.err_slots : kCodecPre;
    int n = 0;
    CqPart D0, D1, D2, D3;
    FootPacked fc = pack_foot(footprint(P, px, py, pz), alive);
    bool lc[4];
    lc[0] = cq_gather<0>(P, fc, g, pre16, npre, D0);
    lc[1] = cq_gather<1>(P, fc, g, pre16, npre, D1);
    lc[2] = cq_gather<2>(P, fc, g, pre16, npre, D2);
    lc[3] = cq_gather<3>(P, fc, g, pre16, npre, D3);
    for (int i = 0; i < kMaxSteps; i++) {
        if (!wave_any(alive)) break;
        const float tn = t + kTStep;                                        // K:701
        const bool cont = alive && !(tn > r.tfar) && (i + 1 < kMaxSteps);  // K:703, 381
        const float nx = px + stx, ny = py + sty, nz = pz + stz;            // K:706
        const FootPacked fn = pack_foot(footprint(P, nx, ny, nz), cont);
        bool ln[4];
        const float b0 = cq_group<0, C, TL>(P, s_lds, scr, lt, fc, lc[0], fn, ln[0], g, pre16, npre, D0);
        const float b1 = cq_group<1, C, TL>(P, s_lds, scr, lt, fc, lc[1], fn, ln[1], g, pre16, npre, D1);
        const float b2 = cq_group<2, C, TL>(P, s_lds, scr, lt, fc, lc[2], fn, ln[2], g, pre16, npre, D2);
        const float b3 = cq_group<3, C, TL>(P, s_lds, scr, lt, fc, lc[3], fn, ln[3], g, pre16, npre, D3);
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
    if (!valid) return;
    if (!hit) {
        write_miss(P, o);
        return;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
}

template <int B, bool COUNT>
static hipError_t march_codec_b(int method, Params P, uint32_t nslots, hipStream_t s) {
    const dim3 grid(nslots), block(256);
    if (!COUNT) note_kernel("k_march_codec", B, method);
    // template table (if staged) at the front of the request, then the error
    // scratch (B floats per thread); VR_WG_PER_CU caps
    const size_t need = (((((size_t)P.tpl_lds + 15) & ~(size_t)15) + (size_t)B * 256u * 4u + 31) &
                         ~(size_t)31) + (method == 6 ? 65 * sizeof(LogEnt) : 0);
    const size_t lds = cap_lds(P, P.wg_per_cu, need);
    const bool tl = P.tpl_lds != 0;
    if constexpr (B == 8 && !COUNT) {
        // oblique views: the quad-cooperative codec march (VR_CODEC_QUAD=0 disables)
        const char *eq = tuning("VR_CODEC_QUAD");
        if (P.oblique && !(eq && std::atoi(eq) == 0)) {
            note_kernel("k_march_codec_quad", B, method);
            switch (method * 2 + (tl ? 1 : 0)) {
            case 8: hipLaunchKernelGGL((k_march_codec_quad<0, false>), grid, block, lds, s, nullptr, P); break;
            case 9: hipLaunchKernelGGL((k_march_codec_quad<0, true>), grid, block, lds, s, nullptr, P); break;
            case 10: hipLaunchKernelGGL((k_march_codec_quad<1, false>), grid, block, lds, s, nullptr, P); break;
            case 11: hipLaunchKernelGGL((k_march_codec_quad<1, true>), grid, block, lds, s, nullptr, P); break;
            case 12: hipLaunchKernelGGL((k_march_codec_quad<2, false>), grid, block, lds, s, nullptr, P); break;
            case 13: hipLaunchKernelGGL((k_march_codec_quad<2, true>), grid, block, lds, s, nullptr, P); break;
            default: return hipErrorInvalidValue;
            }
            return hipGetLastError();
        }
    }
    switch (method * 2 + (tl ? 1 : 0)) {
    case 8: hipLaunchKernelGGL((k_march_codec<B, 0, COUNT, false>), grid, block, lds, s, nullptr, P); break;
    case 9: hipLaunchKernelGGL((k_march_codec<B, 0, COUNT, true>), grid, block, lds, s, nullptr, P); break;
    case 10: hipLaunchKernelGGL((k_march_codec<B, 1, COUNT, false>), grid, block, lds, s, nullptr, P); break;
    case 11: hipLaunchKernelGGL((k_march_codec<B, 1, COUNT, true>), grid, block, lds, s, nullptr, P); break;
    case 12: hipLaunchKernelGGL((k_march_codec<B, 2, COUNT, false>), grid, block, lds, s, nullptr, P); break;
    case 13: hipLaunchKernelGGL((k_march_codec<B, 2, COUNT, true>), grid, block, lds, s, nullptr, P); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <bool COUNT>
static hipError_t march_codec_dispatch(int nb, int method, const Params &P, uint32_t nslots,
                                       hipStream_t s) {
    switch (nb) {
    case 1: return march_codec_b<1, COUNT>(method, P, nslots, s);
    case 2: return march_codec_b<2, COUNT>(method, P, nslots, s);
    case 4: return march_codec_b<4, COUNT>(method, P, nslots, s);
    case 8: return march_codec_b<8, COUNT>(method, P, nslots, s);
    case 16: return march_codec_b<16, COUNT>(method, P, nslots, s);
    case 32: return march_codec_b<32, COUNT>(method, P, nslots, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_march_codec(int nb, int method, const Params &P, uint32_t nslots, bool count,
                              hipStream_t s) {
    if (nslots == 0) return hipSuccess;
    return count ? march_codec_dispatch<true>(nb, method, P, nslots, s)
                 : march_codec_dispatch<false>(nb, method, P, nslots, s);
}

// Algorithmic bytes of the marked codec voxels: a 16-byte codebook entry and
// NE 8-byte error pairs each.
__global__ __launch_bounds__(256) void k_codec_bytes(const unsigned long long *__restrict__ bits,
                                                     uint64_t nvox, const int4 *__restrict__ cb,
                                                     unsigned long long *total) {
    unsigned long long acc = 0;
    for (uint64_t v = blockIdx.x * 256ull + threadIdx.x; v < nvox; v += gridDim.x * 256ull)
        if ((bits[v >> 6] >> (v & 63)) & 1ull) acc += 16ull + 8ull * (unsigned)cb[v].w;
    if (acc) atomicAdd(total, acc);
}

hipError_t launch_codec_bytes(const unsigned long long *bits, uint64_t nvox, const int4 *cb,
                              unsigned long long *total, hipStream_t s) {
    uint64_t blocks = (nvox + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(k_codec_bytes, dim3((uint32_t)blocks), dim3(256), 0, s, bits, nvox, cb,
                       total);
    return hipGetLastError();
}

// Codec validation: counts codebook entries the decode cannot take (template
// id outside [0, ntpl), shift outside [0, nb), NE outside [0, err_slots]).
__global__ __launch_bounds__(256) void k_codec_check(const int4 *__restrict__ cb, uint64_t n,
                                                     int ntpl, int nb, int slots,
                                                     unsigned long long *bad) {
    unsigned long long b = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        const int4 c = cb[i];
        b += c.x < 0 || c.x >= ntpl || c.y < 0 || c.y >= nb || c.w < 0 || c.w > slots;
    }
    if (b) atomicAdd(bad, b);
}

hipError_t launch_codec_check(const int4 *cb, uint64_t n, int ntpl, int nb, int slots,
                              unsigned long long *bad, hipStream_t s) {
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_codec_check, dim3((uint32_t)blocks), dim3(256), 0, s, cb, n, ntpl, nb,
                       slots, bad);
    return hipGetLastError();
}

template <int B, bool BK = false>
__global__ __launch_bounds__(256) void k_march_m7(const float *__restrict__ vol, Params P) {
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

// Synthetic codec volume: the section-5 scalar field f
// encoded against templates of mean (t + 0.5) / T; per voxel
// h = splitmix64(seed ^ v): shift (h >> 8) & 1 (mod B), flip when
// ((h >> 16) & 7) == 0, NE = (h >> 24) % (min(slots, 3) + 1); error j is
// bin h2 % B, value (u01(h2) - 0.5) / 10 with h2 = splitmix64(seed +
// 0x5bd1e995 + v * slots + j).
__global__ __launch_bounds__(256) void k_synth_codec(int4 *__restrict__ cb, float2 *__restrict__ err,
                                                     SynthArgs a, int ntpl, int slots) {
    const uint64_t nvox = (uint64_t)a.nx * a.ny * a.nz;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const int nemax = (slots < 3 ? slots : 3) + 1;
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
        int t = (int)(f * (float)ntpl);
        if (t > ntpl - 1) t = ntpl - 1;
        const uint64_t h = splitmix64(a.seed ^ v);
        cb[v] = make_int4(t, (int)((h >> 8) & 1) % a.nb, ((h >> 16) & 7) == 0 ? 1 : 0,
                          (int)((h >> 24) % (uint64_t)nemax));
        for (int j = 0; j < slots; j++) {
            const uint64_t h2 = splitmix64(a.seed + 0x5bd1e995ull + v * (uint64_t)slots + j);
            err[v * (uint64_t)slots + j] =
                make_float2((float)(h2 % (uint64_t)a.nb),
                            (float)(((double)(h2 >> 11) * 0x1.0p-53 - 0.5) / 10.0));
        }
    }
}

hipError_t launch_synth_codec(int4 *cb, float2 *err, const SynthArgs &a, int ntpl, int slots,
                              hipStream_t s) {
    const uint64_t nvox = (uint64_t)a.nx * a.ny * a.nz;
    uint64_t blocks = (nvox + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_synth_codec, dim3((uint32_t)blocks), dim3(256), 0, s, cb, err, a, ntpl,
                       slots);
    return hipGetLastError();
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
                                                   (B >= 8 && method == 3 ? 65 * sizeof(LogEnt) + 4u * 64u * B * sizeof(float) : 0) : 0);
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
            const size_t qlds = cap_lds(P, qcap, method == 3 ? 65 * sizeof(LogEnt) : 0);
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
            case 3: hipLaunchKernelGGL((k_march_ws<B, 3>), grid, block, 65 * sizeof(LogEnt), s, vol, P); break;
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
                                      method == 3 ? 65 * sizeof(LogEnt) + (B >= 32 ? 4 * 64 * B * sizeof(float) : 4) : 64);
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
    if (!COUNT) note_kernel(method == 7 ? "k_march_m7" : "k_march", B, method);
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
        // workgroup boxes of P.wg_rows tile rows (fill_params: full frames, 4 / 8 bins)
        if constexpr (B == 4 || B == 8) {
            if (B == 8 && method == 3 && k <= 1 && !P.tile_list && (P.wg_rows == 2 || P.wg_rows == 4) &&
                P.box_wg > 0) {  // 8-bin entropy, one sample per box
                note_kernel(P.wg_rows == 4 ? "k_march_wgbox4_k1" : "k_march_wgbox2_k1", B, method);
                const size_t el = cap_lds(P, P.wg_per_cu, 65 * sizeof(LogEnt) + 4u * P.wg_rows * 64u * B * sizeof(float) +
                                                              (24u + (size_t)P.box_wg) * sizeof(float));
                if (P.wg_rows == 4)
                    hipLaunchKernelGGL((k_march_wgbox<8, 3, 1, 4>), grid, dim3(1024), el, s, vol, P);
                else
                    hipLaunchKernelGGL((k_march_wgbox<8, 3, 1, 2>), grid, dim3(512), el, s, vol, P);
                return hipGetLastError();
            }
            if ((k == 2 || k == 4) && (method == 1 || method == 2) && !P.tile_list &&
                (P.wg_rows == 2 || P.wg_rows == 4) && P.box_wg > 0 &&
                !(B == 8 && k == 4 && P.wg_rows == 4)) {  // (1024 lanes: 128 VGPRs, would spill)
                if (P.wg_pipe && P.wg_rows == 2) {  // next box in flight (k_march_wgpipe)
                    note_kernel(k == 2 ? "k_march_wgpipe2_k2" : "k_march_wgpipe2_k4", B, method);
                    const size_t pl = cap_lds(P, P.wg_per_cu, (24u + 2u * (size_t)P.box_wg) * sizeof(float));
#define VR_WGP_L(MM, KK) hipLaunchKernelGGL((k_march_wgpipe<B, MM, KK, 2>), grid, dim3(512), pl, s, vol, P)
                    switch ((k == 4 ? 4 : 0) + method) {
                    case 1: VR_WGP_L(1, 2); break;
                    case 2: VR_WGP_L(2, 2); break;
                    case 5: VR_WGP_L(1, 4); break;
                    case 6: VR_WGP_L(2, 4); break;
                    }
#undef VR_WGP_L
                    return hipGetLastError();
                }
                static const char *names[2][2] = {{"k_march_wgbox2_k2", "k_march_wgbox2_k4"},
                                                  {"k_march_wgbox4_k2", "k_march_wgbox4_k4"}};
                note_kernel(names[P.wg_rows == 4][k == 4], B, method);
                const size_t wl = cap_lds(P, P.wg_per_cu, (24u + (size_t)P.box_wg) * sizeof(float));
                const dim3 wblock(256u * (uint32_t)P.wg_rows);
#define VR_WG_L(MM, KK, RR) hipLaunchKernelGGL((k_march_wgbox<B, MM, KK, RR>), grid, wblock, wl, s, vol, P)
                switch ((P.wg_rows == 4 ? 8 : 0) + (k == 4 ? 4 : 0) + method) {
                case 1: VR_WG_L(1, 2, 2); break;
                case 2: VR_WG_L(2, 2, 2); break;
                case 5: VR_WG_L(1, 4, 2); break;
                case 6: VR_WG_L(2, 4, 2); break;
                case 9: VR_WG_L(1, 2, 4); break;
                case 10: VR_WG_L(2, 2, 4); break;
                case 13: if constexpr (B != 8) VR_WG_L(1, 4, 4); break;
                case 14: if constexpr (B != 8) VR_WG_L(2, 4, 4); break;
                }
#undef VR_WG_L
                return hipGetLastError();
            }
        }
        // a grouped launch (fill_params: grid and order by groups of rows) that no
        // instance above took would cover only some of the tiles
        if (P.wg_rows) return hipErrorInvalidValue;
        if (k >= 2 && k <= 4 && method >= 1 && method <= 3 && P.box_max > 0) {
            note_kernel(k == 2 ? "k_march_duo" : k == 3 ? "k_march_duo3" : "k_march_duo4", B, method);
#define VR_DUO_L(MM, KK) hipLaunchKernelGGL((k_march_duo<B, MM, KK>), grid, block, lds, s, vol, P)
            switch (k * 4 + method) {
            case 9: VR_DUO_L(1, 2); break;
            case 10: VR_DUO_L(2, 2); break;
            case 11: VR_DUO_L(3, 2); break;
            case 13: VR_DUO_L(1, 3); break;
            case 14: VR_DUO_L(2, 3); break;
            case 15: VR_DUO_L(3, 3); break;
            case 17: VR_DUO_L(1, 4); break;
            case 18: VR_DUO_L(2, 4); break;
            case 19: VR_DUO_L(3, 4); break;
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
    case -7:  // method 7 over the baked corner means (plane 3, vr_stats.hip)
        if constexpr (B == 1 && !COUNT) {
            // 4-byte corners: the plain march (the look-ahead gather of
            // k_march_m7_pipe, VR_M7_PIPE=1, only adds loads), 4 workgroups per CU
            // on row-aligned views, 2 on oblique ones (1024^3 C0 0.68 -> 0.64 ms,
            // C1 2.03 -> 1.67; profiles/r02/baked_m7.log)
            const char *ep = tuning("VR_M7_PIPE");
            const size_t lds =
                cap_lds(P, P.wg_per_cu > 0 ? P.wg_per_cu : (P.oblique ? 2 : 4));
            if (ep && std::atoi(ep) != 0) {
                note_kernel("k_march_m7_pipe", B, method);
                hipLaunchKernelGGL((k_march_m7_pipe<1, true>), grid, block, lds, s, vol, P);
            } else {
                note_kernel("k_march_m7", B, method);
                hipLaunchKernelGGL((k_march_m7<1, true>), grid, block, lds, s, vol, P);
            }
            break;
        }
        return hipErrorInvalidValue;
    case 7:
        if (COUNT) return hipErrorInvalidValue;
        // oblique views run method 7 at 3 workgroups per CU when B = 8 (the
        // measured case): fewer corner-mean refreshes in flight, fewer L2
        // re-reads (1024^3x8 C1 9.94 -> 8.29 ms; row-aligned C0 is fastest
        // uncapped).  Keyed on the view, not on P.path, which
        // the B < 8 rewrite above has already changed.
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
                break;
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
                break;
            }
        }
        if constexpr (B > 0 && B <= 8) {
            // pipelined corner gathers (VR_M7_PIPE=0: the plain march)
            const char *ep = tuning("VR_M7_PIPE");
            const bool pipe = !(ep && std::atoi(ep) == 0);
            if (pipe) {
                // oblique views at 2 workgroups per CU (1024^3x8 C1: 8.53 -> 7.45 ms;
                // C0 is fastest uncapped, 1.53 ms; profiles/r02/m7_pipe.log)
                note_kernel("k_march_m7_pipe", B, method);
                hipLaunchKernelGGL((k_march_m7_pipe<B>), grid, block,
                                   cap_lds(P, P.wg_per_cu > 0 ? P.wg_per_cu
                                                              : (P.oblique && B == 8 ? 2 : 0)),
                                   s, vol, P);
                break;
            }
        }
        hipLaunchKernelGGL((k_march_m7<B>), grid, block,
                           cap_lds(P, P.wg_per_cu > 0 ? P.wg_per_cu : (P.oblique && B == 8 ? 3 : 0)),
                           s, vol, P);
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
