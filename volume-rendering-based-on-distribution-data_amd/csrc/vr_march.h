// vr_march.h -- device helpers shared by the march kernels (vr_kernels.hip,
// vr_seg.hip): launch-slot -> tile mapping, ray generation + box test,
// footprint + filter blend, composite, output writes, corner gathers.
// K = volumeRender_kernel.cu of the reference.
#pragma once

#include "vr_device.h"

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

// Workgroup b runs on XCD b % 8.  Tile lists (multi-GPU) and the host-built
// full-frame order P.perm are already XCD-interleaved by their producers
// (tiles.py / frame_order), so workgroup b takes entry b; without either, the
// raster order is split into one contiguous run per XCD (xcd_slot).
__device__ __forceinline__ uint32_t launch_slot(const Params &P) {
    return (P.tile_list || P.perm) ? blockIdx.x : xcd_slot(blockIdx.x, gridDim.x);
}
__device__ __forceinline__ uint32_t tile_of(const Params &P, uint32_t slot) {
    if (P.tile_list) return P.tile_list[slot];
    if (P.perm) return P.perm[slot];
    return slot;
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

// Pixel of this thread inside its tile: wave w renders tile row w, lane = x.
// Wide, short tiles: a footprint row of records is x-contiguous, so a tile edge
// along y (left/right neighbour) splits every 128-B line of the rows it
// crosses between two workgroups, while an edge along x costs only the records
// of one voxel row.  64x4 tiles fetch 12 % fewer lines per frame than 16x16
// (tools/footprint_sim.c, C0 at 1024^3 x 8) and each wave's gathers cover one
// contiguous x run.
static_assert(kTileW == 64 && kTileH * kTileW == 256, "one wave per 64-pixel tile row");
__device__ __forceinline__ void tile_pixel(uint32_t t, uint32_t &lx, uint32_t &ly) {
    lx = t & (kTileW - 1);
    ly = t / kTileW;
}
// P.seg_map: a wave's 64 lanes take a 16x4 pixel block of the tile instead of a
// 64-pixel row (compact footprints per load instruction; where it is the default:
// vr_api.cpp fill_params)
__device__ __forceinline__ void lane_pixel(const Params &P, uint32_t t, uint32_t &lx, uint32_t &ly) {
    if (P.seg_map) {
        lx = (t >> 6) * 16u + (t & 15u);
        ly = (t >> 4) & 3u;
    } else {
        tile_pixel(t, lx, ly);
    }
}

__device__ __forceinline__ void write_miss(const Params &P, uint64_t o) {
    if (P.out_n) P.out_n[o] = -1;
    if (P.tile_list) P.out[o] = 0u;  // packed tile slots are cleared (see write_pixel)
}

__device__ __forceinline__ void write_pixel(const Params &P, uint64_t o, int n, float r,
                                            float g, float b, float a) {
    if (P.out_n) P.out_n[o] = n;
    if (n < 0) {  // a miss leaves a full frame untouched (K:302-303) but clears a packed
        if (P.tile_list) P.out[o] = 0u;  // tile slot, so tile buffers need no memset
        return;
    }
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
// ---- wave-level helpers (64 lanes, DPP) ----
// min over the 64 lanes: row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast 15 / 31 across rows; lane 63 holds the result.
__device__ __forceinline__ int dpp_min(int v, int ident) {
    v = min(v, __builtin_amdgcn_update_dpp(ident, v, 0x111, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(ident, v, 0x112, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(ident, v, 0x114, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(ident, v, 0x118, 0xF, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(ident, v, 0x142, 0xA, 0xF, false));
    v = min(v, __builtin_amdgcn_update_dpp(ident, v, 0x143, 0xC, 0xF, false));
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int wave_min(int v) { return dpp_min(v, 0x7FFFFFFF); }
__device__ __forceinline__ int wave_max(int v) { return -dpp_min(-v, 0x7FFFFFFF); }

// three wave minima at once: each DPP level is issued for the three values back
// to back, so the DPP read-after-write hazard of one chain is covered by the
// other two instead of by s_nop wait states
__device__ __forceinline__ void dpp_min3(int &a, int &b, int &c) {
    constexpr int I = 0x7FFFFFFF;
#define VR_DPP3(CTRL, ROWM)                                                  \
    a = min(a, __builtin_amdgcn_update_dpp(I, a, CTRL, ROWM, 0xF, false));   \
    b = min(b, __builtin_amdgcn_update_dpp(I, b, CTRL, ROWM, 0xF, false));   \
    c = min(c, __builtin_amdgcn_update_dpp(I, c, CTRL, ROWM, 0xF, false));
    VR_DPP3(0x111, 0xF)
    VR_DPP3(0x112, 0xF)
    VR_DPP3(0x114, 0xF)
    VR_DPP3(0x118, 0xF)
    VR_DPP3(0x142, 0xA)
    VR_DPP3(0x143, 0xC)
#undef VR_DPP3
    a = __builtin_amdgcn_readlane(a, 63);
    b = __builtin_amdgcn_readlane(b, 63);
    c = __builtin_amdgcn_readlane(c, 63);
}

__device__ __forceinline__ bool wave_any(bool b) { return __ballot(b) != 0; }

// Corners of one sample (K:601 texture footprint): texel indices + 8-bit weights.
struct Foot {
    int x0, x1, y0, y1, z0, z1;
    float ax, ay, az;
};

__device__ __forceinline__ Foot footprint(const Params &P, float px, float py, float pz) {
    Foot f;
    lin_axis(px * 0.5f + 0.5f, P.nx, f.x0, f.x1, f.ax);
    lin_axis(py * 0.5f + 0.5f, P.ny, f.y0, f.y1, f.ay);
    lin_axis(pz * 0.5f + 0.5f, P.nz, f.z0, f.z1, f.az);
    return f;
}

__device__ __forceinline__ float blend8(const float (&s)[8], const Foot &f) {
    const float c00 = lerpq(s[0], s[1], f.ax);
    const float c10 = lerpq(s[2], s[3], f.ax);
    const float c01 = lerpq(s[4], s[5], f.ax);
    const float c11 = lerpq(s[6], s[7], f.ax);
    const float c0 = lerpq(c00, c10, f.ay);
    const float c1 = lerpq(c01, c11, f.ay);
    return lerpq(c0, c1, f.az);
}
// a baked plane's x-pair in one 8-byte load at 4-byte alignment (one address
// per lane for both x corners; bricks keep every pair inside one line)
typedef float vr_f2a4 __attribute__((ext_vector_type(2), aligned(4)));
__device__ __forceinline__ vr_f2a4 load_pair64(const float *__restrict__ vol, uint64_t i) {
    return *reinterpret_cast<const vr_f2a4 *>(vol + i);
}
// MODE 0: records in x rows (P.sy / P.sz record pitches).  MODE 3: an axis-rows
// copy (P.sx / P.sy / P.sz strides; axis_copy_strides).  MODE 4 / 5: a baked
// plane's y- / z-rows copy (P.sy / P.sz its pitches).  MODE 1 / 2: a baked
// statistics plane (B = 1) in 16 x 2 x 1 bricks (plane_index; P.sy / P.sz the
// plane pitches): each (y, z) row's x-pair is one 8-byte load; MODE 1 forms the
// index with 24-bit multiplies in 32 bits (pitches < 2^24, plane < 2^32 floats:
// vr_api.cpp plane_narrow), MODE 2 in 64 bits.
template <int B, int MODE = 0>
__device__ __forceinline__ void gather8(const float *__restrict__ vol, const Params &P,
                                        const Foot &f, float (&rec)[8][B]) {
    if constexpr (MODE == 1 || MODE == 2) {
        static_assert(B == 1, "baked planes hold one float per voxel");
        const uint32_t bx = plane_bx((uint32_t)f.x0);
        const bool ox = f.x1 != f.x0;
        uint64_t i00, i10, i01, i11;
        if constexpr (MODE == 1) {
            const uint32_t sy = (uint32_t)P.sy, sz = (uint32_t)P.sz;
            const uint32_t z0 = __umul24((uint32_t)f.z0, sz), z1 = __umul24((uint32_t)f.z1, sz);
            const uint32_t y0 = __umul24((uint32_t)f.y0 >> 1, sy) + ((uint32_t)f.y0 & 1u) * 16u + bx;
            const uint32_t y1 = __umul24((uint32_t)f.y1 >> 1, sy) + ((uint32_t)f.y1 & 1u) * 16u + bx;
            i00 = z0 + y0; i10 = z0 + y1; i01 = z1 + y0; i11 = z1 + y1;
        } else {
            const uint32_t sy = (uint32_t)P.sy;  // a slice is < 2^32 floats
            const uint32_t y0 = ((uint32_t)f.y0 >> 1) * sy + ((uint32_t)f.y0 & 1u) * 16u + bx;
            const uint32_t y1 = ((uint32_t)f.y1 >> 1) * sy + ((uint32_t)f.y1 & 1u) * 16u + bx;
            i00 = (uint64_t)f.z0 * P.sz + y0; i10 = (uint64_t)f.z0 * P.sz + y1;
            i01 = (uint64_t)f.z1 * P.sz + y0; i11 = (uint64_t)f.z1 * P.sz + y1;
        }
        const vr_f2a4 a = load_pair64(vol, i00), b = load_pair64(vol, i10);
        const vr_f2a4 c = load_pair64(vol, i01), d = load_pair64(vol, i11);
        rec[0][0] = a.x;
        rec[1][0] = ox ? a.y : a.x;
        rec[2][0] = b.x;
        rec[3][0] = ox ? b.y : b.x;
        rec[4][0] = c.x;
        rec[5][0] = ox ? c.y : c.x;
        rec[6][0] = d.x;
        rec[7][0] = ox ? d.y : d.x;
        return;
    }
    if constexpr (MODE == 4 || MODE == 5) {
        // a baked plane's axis copy (vr_stats.hip k_plane_axis): the same 16 x 2 x 1
        // bricks with the axis the view's screen x runs along in the brick rows --
        // MODE 4: y rows (y fast, x pairs, z slices), MODE 5: z rows (z fast, y
        // pairs, x slices).  The four pair loads carry y- or z-pairs and are
        // assigned to the same 8 corners, so the blend is unchanged.
        static_assert(B == 1, "baked planes hold one float per voxel");
        const uint32_t sy = (uint32_t)P.sy;  // a slice of the copy is < 2^32 floats
        if constexpr (MODE == 5) {
            const uint32_t bz = plane_bx((uint32_t)f.z0);
            const bool oz = f.z1 != f.z0;
            const uint32_t y0 = ((uint32_t)f.y0 >> 1) * sy + ((uint32_t)f.y0 & 1u) * 16u + bz;
            const uint32_t y1 = ((uint32_t)f.y1 >> 1) * sy + ((uint32_t)f.y1 & 1u) * 16u + bz;
            const uint64_t x0 = (uint64_t)f.x0 * P.sz, x1 = (uint64_t)f.x1 * P.sz;
            const vr_f2a4 a = load_pair64(vol, x0 + y0), b = load_pair64(vol, x1 + y0);
            const vr_f2a4 c = load_pair64(vol, x0 + y1), d = load_pair64(vol, x1 + y1);
            rec[0][0] = a.x; rec[4][0] = oz ? a.y : a.x;
            rec[1][0] = b.x; rec[5][0] = oz ? b.y : b.x;
            rec[2][0] = c.x; rec[6][0] = oz ? c.y : c.x;
            rec[3][0] = d.x; rec[7][0] = oz ? d.y : d.x;
        } else {
            const uint32_t by = plane_bx((uint32_t)f.y0);
            const bool oy = f.y1 != f.y0;
            const uint32_t x0 = ((uint32_t)f.x0 >> 1) * sy + ((uint32_t)f.x0 & 1u) * 16u + by;
            const uint32_t x1 = ((uint32_t)f.x1 >> 1) * sy + ((uint32_t)f.x1 & 1u) * 16u + by;
            const uint64_t z0 = (uint64_t)f.z0 * P.sz, z1 = (uint64_t)f.z1 * P.sz;
            const vr_f2a4 a = load_pair64(vol, z0 + x0), b = load_pair64(vol, z0 + x1);
            const vr_f2a4 c = load_pair64(vol, z1 + x0), d = load_pair64(vol, z1 + x1);
            rec[0][0] = a.x; rec[2][0] = oy ? a.y : a.x;
            rec[1][0] = b.x; rec[3][0] = oy ? b.y : b.x;
            rec[4][0] = c.x; rec[6][0] = oy ? c.y : c.x;
            rec[5][0] = d.x; rec[7][0] = oy ? d.y : d.x;
        }
        return;
    }
    if constexpr (MODE == 6) {
        // a baked plane's 8 x 2 x 2 brick copy (oblique views, vr_stats.hip
        // k_plane8): the four pair loads of MODE 1 with the z pair inside the
        // brick (offset 16) -- a footprint whose z0 is even reads one line per y
        // row pair instead of two
        static_assert(B == 1, "baked planes hold one float per voxel");
        const uint32_t bx = plane8_bx((uint32_t)f.x0);
        const bool ox = f.x1 != f.x0;
        const uint32_t sy = (uint32_t)P.sy;  // a slice pair of the copy is < 2^32 floats
        const uint32_t y0 = ((uint32_t)f.y0 >> 1) * sy + ((uint32_t)f.y0 & 1u) * 8u + bx;
        const uint32_t y1 = ((uint32_t)f.y1 >> 1) * sy + ((uint32_t)f.y1 & 1u) * 8u + bx;
        const uint64_t z0 = (uint64_t)((uint32_t)f.z0 >> 1) * P.sz + ((uint32_t)f.z0 & 1u) * 16u;
        const uint64_t z1 = (uint64_t)((uint32_t)f.z1 >> 1) * P.sz + ((uint32_t)f.z1 & 1u) * 16u;
        const vr_f2a4 a = load_pair64(vol, z0 + y0), b = load_pair64(vol, z0 + y1);
        const vr_f2a4 c = load_pair64(vol, z1 + y0), d = load_pair64(vol, z1 + y1);
        rec[0][0] = a.x;
        rec[1][0] = ox ? a.y : a.x;
        rec[2][0] = b.x;
        rec[3][0] = ox ? b.y : b.x;
        rec[4][0] = c.x;
        rec[5][0] = ox ? c.y : c.x;
        rec[6][0] = d.x;
        rec[7][0] = ox ? d.y : d.x;
        return;
    }
    if constexpr (MODE == 3) {  // axis-rows copy: all three axes strided
        const uint64_t x0 = (uint64_t)f.x0 * P.sx, x1 = (uint64_t)f.x1 * P.sx;
        const uint64_t y0 = (uint64_t)f.y0 * P.sy, y1 = (uint64_t)f.y1 * P.sy;
        const uint64_t z0 = (uint64_t)f.z0 * P.sz, z1 = (uint64_t)f.z1 * P.sz;
        load_rec<B>(vol, x0 + y0 + z0, rec[0]);
        load_rec<B>(vol, x1 + y0 + z0, rec[1]);
        load_rec<B>(vol, x0 + y1 + z0, rec[2]);
        load_rec<B>(vol, x1 + y1 + z0, rec[3]);
        load_rec<B>(vol, x0 + y0 + z1, rec[4]);
        load_rec<B>(vol, x1 + y0 + z1, rec[5]);
        load_rec<B>(vol, x0 + y1 + z1, rec[6]);
        load_rec<B>(vol, x1 + y1 + z1, rec[7]);
        return;
    }
    const uint64_t r00 = (uint64_t)f.z0 * P.sz + (uint64_t)f.y0 * P.sy;
    const uint64_t r10 = (uint64_t)f.z0 * P.sz + (uint64_t)f.y1 * P.sy;
    const uint64_t r01 = (uint64_t)f.z1 * P.sz + (uint64_t)f.y0 * P.sy;
    const uint64_t r11 = (uint64_t)f.z1 * P.sz + (uint64_t)f.y1 * P.sy;
    load_rec<B>(vol, r00 + f.x0, rec[0]);
    load_rec<B>(vol, r00 + f.x1, rec[1]);
    load_rec<B>(vol, r10 + f.x0, rec[2]);
    load_rec<B>(vol, r10 + f.x1, rec[3]);
    load_rec<B>(vol, r01 + f.x0, rec[4]);
    load_rec<B>(vol, r01 + f.x1, rec[5]);
    load_rec<B>(vol, r11 + f.x0, rec[6]);
    load_rec<B>(vol, r11 + f.x1, rec[7]);
}

// gather8's MODE for statistic template M (0 / -1: a baked plane)
template <int M>
constexpr int kGatherMode = M == 0 ? 1 : (M == -1 ? 2 : 0);

// Entropy (K:761-769) of a record with few registers: the lane parks
// its record in its own bin-major LDS column (st[i * 64 + lane]: conflict-free)
// and runs the per-bin sum as a rolled loop over it, the exact logarithm from
// the LDS table -- the same operations in the same order as entropy_p, so the
// same float.  Unrolled over 32 bins the decode held ~430 registers (1 wave per
// SIMD); rolled, the march keeps several waves per SIMD to hide its loads.  The
// 8-bin marches use it too (their unrolled 8 x 8 logarithms per step held
// 360-470 registers, or spilled).
template <int B, int STRIDE = 64>
__device__ __forceinline__ float entropy_col(const float (&p)[B], float *col, float enorm,
                                             const LogEnt *tab) {
#pragma unroll
    for (int i = 0; i < B; i++) col[i * STRIDE] = p[i];
    constexpr int N = B < kEntChunk ? B : kEntChunk;
    float ent = 0.0f;
#pragma unroll 1
    for (int i = 0; i < B; i += N) {  // N bins per iteration (ent_terms)
        float q[N];
        double t[N];
#pragma unroll
        for (int k = 0; k < N; k++) q[k] = col[(i + k) * STRIDE];  // this lane's writes
        ent_terms<N>(q, tab, t);
#pragma unroll
        for (int k = 0; k < N; k++) ent = (float)((double)ent + (double)q[k] * t[k]);
    }
    ent = -ent;
    return ent / enorm;
}
// st: the wave's 64 * B-float region, bin-major (st[i * 64 + lane])
template <int B>
__device__ __forceinline__ float entropy_stash(const float (&p)[B], float *st, uint32_t lane,
                                               float enorm, const LogEnt *tab) {
    return entropy_col<B, 64>(p, st + lane, enorm, tab);
}

// an entropy march's LDS: the log table (kLogTabN entries) + 4 waves' record columns
template <int B>
struct EntropyLds {
    LogEnt tab[kLogTabN];
    float col[4 * 64 * B];
};

// (st, tab): this wave's record column and the LDS log table of an entropy
// march (EntropyLds), nullptr for the other methods
template <int B, int M>
__device__ __forceinline__ float decode8(const Params &P, const float (&rec)[8][B],
                                         const Foot &f, float *st = nullptr,
                                         const LogEnt *tab = nullptr) {
    float s[8];
    if constexpr (M == 3) {
        if (st) {
#pragma unroll
            for (int j = 0; j < 8; j++) s[j] = entropy_stash<B>(rec[j], st, threadIdx.x & 63u, P.enorm, tab);
            return blend8(s, f);
        }
    }
#pragma unroll
    for (int j = 0; j < 8; j++) s[j] = record_stat<B, M>(rec[j], P.enorm);
    return blend8(s, f);
}

// Same arithmetic as k_march's direct path, but the 8 corner records of step
// i+1 are gathered into a second register set BEFORE step i is decoded, so
// every wave always has a step's gathers in flight while its f64 decode runs.
// The prefetch assumes the ray continues; a ray that terminates (early, or at
// tfar) wastes one step of gathers.  The loop is unrolled by two so
// the two register sets swap roles without copies.  t: thread index inside
// the 256-thread tile; slot: the tile's launch slot (packed output position).
template <int B, int M, int GM = kGatherMode<M>>
__device__ __forceinline__ int march_pipe_tile(const float *__restrict__ vol, const Params &P,
                                               uint32_t slot, uint32_t tile, uint32_t tid,
                                               float *st = nullptr, const LogEnt *tab = nullptr) {
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
    bool alive = true;
    Foot fa = footprint(P, px, py, pz), fb;
    float ra[8][B], rb[8][B];
    gather8<B, GM>(vol, P, fa, ra);
    // one step: decode (fc, rc) while the gathers of the next step go to (fn, rn)
    auto step = [&](int i, const Foot &fc, const float (&rc)[8][B], Foot &fn,
                    float (&rn)[8][B]) {
        const float tn = t + kTStep;                               // K:701
        const bool cont = !(tn > r.tfar) && (i + 1 < kMaxSteps);  // K:703, K:381
        const float nx = px + stx, ny = py + sty, nz = pz + stz;   // K:706
        // The next step is gathered unconditionally: the footprint's indices
        // are clamped, so a ray past tfar reads one valid step it discards
        // (early-terminated rays already did).  Without a divergent branch
        // around the loads they need no copies at the join and the compiler
        // keeps the march small (B = 8: 107 VGPRs for the mean, 168 for the
        // variance) with all 16 in flight.  (Re-gathering the current
        // footprint instead -- cache hits -- measured 2.4 ms against 1.36:
        // the select changed the schedule again.)
        fn = footprint(P, nx, ny, nz);
        gather8<B, GM>(vol, P, fn, rn);
        const float sample = decode8<B, M>(P, rc, fc, st, tab);
        n = i + 1;
        if (composite(P, sample, sx, sy, sz, sw) || !cont) {
            alive = false;
        } else {
            t = tn;
            px = nx;
            py = ny;
            pz = nz;
        }
    };
    for (int i = 0; i < kMaxSteps; i += 2) {
        step(i, fa, ra, fb, rb);
        if (!alive) break;
        step(i + 1, fb, rb, fa, ra);
        if (!alive) break;
    }
    write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                sw * P.brightness);
    return n;
}

// Cost record of the adaptive tile order (vr_api.cpp frame_order): every wave
// adds (its longest ray's samples + 2) to its tile's entry, i.e. the wave's
// step-chain length plus a fixed launch/ray-setup share.  n = this lane's
// samples (-1: miss or outside the image); call with all 64 lanes converged.
__device__ __forceinline__ void record_tile_cost(const Params &P, uint32_t tile, int n) {
    const int mx = wave_max(n);
    if ((threadIdx.x & 63u) == 0) atomicAdd(P.tile_cost + tile, (uint32_t)(mx + 2));
}

// Dynamic LDS request that caps resident workgroups per CU at `cap` (0 = no
// cap) and is never below `need` (the kernel's own dynamic LDS, kept at the
// front of the buffer).  P.lds_cu / P.lds_wg are the device's LDS per CU and
// per workgroup (160 KiB each on gfx950, read once by vr_api.cpp); the request
// is clamped to the per-workgroup limit minus the kernel's static LDS.
// Host-side helper.
inline size_t cap_lds(const Params &P, int cap, size_t need = 0, size_t static_lds = 0) {
    size_t r = cap > 0 ? (size_t)(P.lds_cu / cap) & ~(size_t)255 : 0;
    if (r < need) r = need;
    const size_t room = (size_t)P.lds_wg > static_lds ? (size_t)P.lds_wg - static_lds : 0;
    return r > room && need <= room ? room : r;
}

// The VR_WG_PER_CU cap (P.wg_per_cu) for kernels without static LDS.
inline size_t occupancy_lds(const Params &P) { return cap_lds(P, P.wg_per_cu); }

}  // namespace vr
