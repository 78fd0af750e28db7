// vr_seg.hip -- ray-segmented march: S lanes share one ray (methods 1/2/3).
//
// The per-ray march (K:309-707) is a chain of dependent steps: gather the 8
// corner records, decode, composite, advance.  When a GPU has few rays (a rank
// of the multi-GPU tile split, small viewports) the frame time is the length
// of that chain for the longest rays, not HBM bandwidth.  Here a group of S
// consecutive lanes marches one ray in windows of S steps: lane k samples step
// base + k, so S steps' gathers are in flight at once, then the group
// composites the S samples in step order (front to back, K:690-699) with the
// early exit tested after every step (K:700-705).
//
// Bit-identical to the one-lane march: each lane keeps its own copy of the
// accumulated t and pos (K:701, K:706) and advances it by the same sequence of
// float additions (lane k starts k additions ahead, then adds S per window),
// so step s sees exactly the t_s and pos_s of the reference's loop; a step is
// taken iff s < 500 (K:381) and t_s <= tfar (t is non-decreasing, so that is
// the reference's "no earlier break"); composite order and expressions are the
// same.  Samples past an early exit inside a window are gathered but dropped.
#include "vr_internal.h"
#include "vr_march.h"

#include <cstdio>

namespace vr {

// value of lane r + J*R of the wave (ds_bpermute; R = 64/S rays per wave)
template <int S, int J>
__device__ __forceinline__ float group_bcast(float v, uint32_t r) {
    constexpr uint32_t R = 64u / S;
    return __int_as_float(__builtin_amdgcn_ds_bpermute((int)((r + J * R) << 2), __float_as_int(v)));
}

// front-to-back composite of the group's S samples in step order (K:683-705):
// every lane of the group classifies and composites the sample of step
// base + J, taken from the lane that gathered it
template <int S, int J>
__device__ __forceinline__ void composite_window(const Params &P, float smp, uint64_t vm,
                                                 uint32_t r, int base, bool &alive, int &n,
                                                 float &sx, float &sy, float &sz, float &sw) {
    if constexpr (J < S) {
        constexpr uint32_t R = 64u / S;
        const float sj = group_bcast<S, J>(smp, r);
        const bool vj = (vm >> (r + J * R)) & 1ull;
        if (alive) {
            if (vj) {
                n = base + J + 1;
                if (composite(P, sj, sx, sy, sz, sw)) alive = false;  // K:700
            } else {
                alive = false;  // t > tfar or 500 steps (K:381, K:703)
            }
        }
        composite_window<S, J + 1>(P, smp, vm, r, base, alive, n, sx, sy, sz, sw);
    }
}

// Workgroup b: tile slot (b % 8) + 8 (b / 8S), part (b / 8) % S.  Slot s runs on
// XCD s % 8 like every other march (the tile lists and the full-frame order
// are XCD-interleaved by their producers), and the S parts of a tile are
// consecutive workgroups of the same XCD.
//
// PIPE: the next window's corner records are gathered before this window is
// decoded (one window of gathers always in flight, twice the record
// registers); a group that exits early wastes one window of gathers.
#ifndef VR_SEG_WAVES
#define VR_SEG_WAVES 1   // minimum waves per SIMD the register allocation must allow
#endif
// part `part` (256/S of its rays) of the tile in launch slot `slot`
template <int B, int M, int S, bool PIPE, int GM>
__device__ __forceinline__ void march_seg_part(const float *__restrict__ vol, const Params &P,
                                               uint32_t slot, uint32_t part) {
    constexpr int RPW = 256 / S;  // rays per workgroup
    if (slot >= P.n_tiles) return;
    const uint32_t tile = P.tile_list ? P.tile_list[slot]
                        : P.perm      ? P.perm[slot]
                                      : xcd_slot(slot, P.n_tiles);
    if (tile == kPad) return;
    // lane = k*R + r: the 4-lane groups the L1 serves together hold adjacent rays
    // at the same step (adjacent records), as in the one-lane march
    constexpr uint32_t R = 64u / S;
    const uint32_t lane = threadIdx.x & 63u, rl = lane % R, k = lane / R;
    uint32_t lx, ly;
    if (P.seg_map) {
        // a wave's R rays as an (R/4) x 4 pixel block, the workgroup's as a
        // (RPW/4) x 4 column block of the tile: compact footprints per load
        constexpr uint32_t BW = R / 4u;
        lx = part * (RPW / 4u) + (threadIdx.x >> 6) * BW + rl % BW;
        ly = rl / BW;
    } else {
        const uint32_t p = part * RPW + (threadIdx.x >> 6) * R + rl;  // pixel inside the 64x4 tile
        lx = p % kTileW;
        ly = p / kTileW;
    }
    const uint32_t x = (tile % P.tiles_x) * kTileW + lx;
    const uint32_t y = (tile / P.tiles_x) * kTileH + ly;
    if (x >= P.CW || y >= P.CH) return;  // the whole group leaves
    const uint64_t o = P.tile_list ? (uint64_t)slot * 256u + ly * kTileW + lx
                                   : (uint64_t)y * P.W + x;
    Ray r;
    if (!make_ray(P, x, y, r)) {
        if (k == 0) write_miss(P, o);
        return;
    }
    float t = r.tnear;
    float px = r.ox + r.dx * r.tnear, py = r.oy + r.dy * r.tnear, pz = r.oz + r.dz * r.tnear;
    const float stx = r.dx * kTStep, sty = r.dy * kTStep, stz = r.dz * kTStep;
#pragma unroll
    for (int j = 0; j < S - 1; j++) {
        if ((uint32_t)j < k) {
            t = t + kTStep;
            px = px + stx;
            py = py + sty;
            pz = pz + stz;
        }
    }
    float sx = 0.0f, sy = 0.0f, sz = 0.0f, sw = 0.0f;
    int n = 0, base = 0;
    bool alive = true;
    // step s is taken iff s < 500 and t_s <= tfar (and no early exit before it)
    auto geom = [&](int s, float ts) { return s < kMaxSteps && (s == 0 || !(ts > r.tfar)); };
    auto advance = [&](float &tt, float &qx, float &qy, float &qz) {
#pragma unroll
        for (int j = 0; j < S; j++) {
            tt = tt + kTStep;
            qx = qx + stx;
            qy = qy + sty;
            qz = qz + stz;
        }
    };
    if constexpr (!PIPE) {
        while (true) {
            const bool valid = alive && geom(base + (int)k, t);
            float smp = 0.0f;
            if (valid) {
                const Foot f = footprint(P, px, py, pz);
                float rec[8][B];
                gather8<B, GM>(vol, P, f, rec);
                smp = decode8<B, M>(P, rec, f);
            }
            const uint64_t vm = __ballot(valid);
            composite_window<S, 0>(P, smp, vm, rl, base, alive, n, sx, sy, sz, sw);
            if (!__ballot(alive)) break;
            base += S;
            advance(t, px, py, pz);
        }
    } else {
        Foot fa, fb;
        float ra[8][B], rb[8][B];
        bool va = geom((int)k, t), vb = false;
#ifndef VR_SEG_COND
        fa = footprint(P, px, py, pz);
        gather8<B, GM>(vol, P, fa, ra);
#else
        if (va) {
            fa = footprint(P, px, py, pz);
            gather8<B, GM>(vol, P, fa, ra);
        }
#endif
        // one window: gather the next into (fn, rn, vn) while (fc, rc, vc) decodes
        auto window = [&](const Foot &fc, const float (&rc)[8][B], bool vc, Foot &fn,
                          float (&rn)[8][B], bool &vn) {
            float tn = t, nx = px, ny = py, nz = pz;
            advance(tn, nx, ny, nz);
            vn = alive && geom(base + S + (int)k, tn);
#ifndef VR_SEG_COND
            // Gathered unconditionally: without a divergent branch around the
            // loads the march needs no register copies at the join (B = 8,
            // mean: 208 -> 170 VGPRs, fewer instructions per window); a lane with no next
            // step re-reads its current footprint (cache hits), not new lines.
            // 1024^3 x 8 C0 cost-dealt lists, max over ranks: N = 4 0.405 ->
            // 0.380 ms, N = 8 0.212 -> 0.213, the longest tile alone 0.154 ->
            // 0.121 (profiles/r04/rank_sim_C0_uncond.log; VR_SEG_COND builds the
            // branch)
            fn = footprint(P, vn ? nx : px, vn ? ny : py, vn ? nz : pz);
            gather8<B, GM>(vol, P, fn, rn);
#else
            if (vn) {
                fn = footprint(P, nx, ny, nz);
                gather8<B, GM>(vol, P, fn, rn);
            }
#endif
            // (decoding unconditionally as well frees registers -- 170 -> 143
            // VGPRs, 3 waves per SIMD -- but lets the scheduler sink the next
            // window's loads into the decode: N = 8 lists 0.213 -> 0.254 ms,
            // profiles/r04/rank_sim_C0_uncond_decode.log)
            float smp = 0.0f;
            if (vc && alive) smp = decode8<B, M>(P, rc, fc);
            const uint64_t vm = __ballot(vc);
            composite_window<S, 0>(P, smp, vm, rl, base, alive, n, sx, sy, sz, sw);
            base += S;
            t = tn;
            px = nx;
            py = ny;
            pz = nz;
        };
        while (true) {
            window(fa, ra, va, fb, rb, vb);
            if (!__ballot(alive)) break;
            window(fb, rb, vb, fa, ra, va);
            if (!__ballot(alive)) break;
        }
    }
    if (k == 0)
        write_pixel(P, o, n, sx * P.brightness, sy * P.brightness, sz * P.brightness,
                    sw * P.brightness);
}

// GM: gather8's addressing (kGatherMode<M>; 3 = an axis-rows copy of the records,
// the views whose screen x runs along the volume's z or y)
template <int B, int M, int S, bool PIPE, int GM = kGatherMode<M>>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_SEG_WAVES, 8))) void k_march_seg(const float *__restrict__ vol, Params P) {
    const uint32_t b = blockIdx.x;
    const uint32_t slot = (b & 7u) + 8u * (b / (8u * S)), part = (b >> 3) % S;
    unsigned long long t0 = 0;
    if (P.wave_clock) t0 = wall_clock64();
    march_seg_part<B, M, S, PIPE, GM>(vol, P, slot, part);
    if (P.wave_clock && (threadIdx.x & 63u) == 0 && slot < P.n_tiles) {  // tooling
        unsigned long long *w = P.wave_clock + ((uint64_t)slot * 16u + part * 4u + threadIdx.x / 64u) * 3u;
        w[0] = t0;
        w[1] = wall_clock64();
        w[2] = __smid();
    }
}

// A tile list whose longest tiles set the launch time (a rank's list at 4-8
// GPUs): those tiles take SH lanes per ray, the rest ST, in ONE launch -- two
// kernels' worth of workgroups, the head's dispatched first.  Both bodies
// have about the same register need (one window of 8 corner records per lane),
// so sharing a kernel costs no occupancy.  Slots [0, head_slots) are the
// first entries of every XCD sublist (entry s runs on XCD s % 8 and each
// sublist is longest first, tiles.py / frame_order); head_slots is a multiple
// of 8, so the tail's workgroup b keeps b % 8 = its slot % 8.
template <int B, int M, int SH, int ST, int GM = kGatherMode<M>>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_SEG_WAVES, 8))) void k_march_seg_head(const float *__restrict__ vol, Params P) {
    const uint32_t hw = P.head_slots * (uint32_t)SH;  // head workgroups
    uint32_t b = blockIdx.x, slot, part;
    unsigned long long t0 = 0;
    if (P.wave_clock) t0 = wall_clock64();
    if (b < hw) {
        slot = (b & 7u) + 8u * (b / (8u * SH));
        part = (b >> 3) % SH;
        march_seg_part<B, M, SH, true, GM>(vol, P, slot, part);
    } else {
        b -= hw;
        slot = P.head_slots + (b & 7u) + 8u * (b / (8u * ST));
        part = (b >> 3) % ST;
        march_seg_part<B, M, ST, true, GM>(vol, P, slot, part);
    }
    if (P.wave_clock && (threadIdx.x & 63u) == 0 && slot < P.n_tiles && part < 4) {  // tooling
        unsigned long long *w = P.wave_clock + ((uint64_t)slot * 16u + part * 4u + threadIdx.x / 64u) * 3u;
        w[0] = t0;
        w[1] = wall_clock64();
        w[2] = __smid();
    }
}

// The same split with the one-lane pipelined march (march_pipe_tile, one
// 256-ray tile per workgroup) for the tail: the tail's rays are short enough
// that one lane per ray is the cheaper issue, the head's long chains take SH
// lanes.  Tail workgroup b' = b - head workgroups renders slot head_slots + b'
// (b' % 8 = b % 8: the tile list's XCD interleave holds).
template <int B, int M, int SH, int GM = kGatherMode<M>>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_SEG_WAVES, 8))) void k_march_pipe_head(const float *__restrict__ vol, Params P) {
    const uint32_t hw = P.head_slots * (uint32_t)SH;
    const uint32_t b = blockIdx.x;
    if (b < hw) {
        march_seg_part<B, M, SH, true, GM>(vol, P, (b & 7u) + 8u * (b / (8u * SH)), (b >> 3) % SH);
        return;
    }
    const uint32_t slot = P.head_slots + (b - hw);
    if (slot >= P.n_tiles) return;
    const uint32_t tile = P.tile_list[slot];
    if (tile == kPad) return;
    march_pipe_tile<B, M, GM>(vol, P, slot, tile, threadIdx.x);
}

template <int B, int SH>
static hipError_t pipe_head_launch(int method, const float *vol, const Params &P, uint32_t nslots,
                                   hipStream_t s) {
    const dim3 grid(P.head_slots * (uint32_t)SH + (nslots - P.head_slots)), block(256);
    if (P.avol) {
        Params Q = P;
        Q.sx = P.asx;
        Q.sy = P.asy;
        Q.sz = P.asz;
        switch (method) {
        case 1: hipLaunchKernelGGL((k_march_pipe_head<B, 1, SH, 3>), grid, block, occupancy_lds(P), s, P.avol, Q); break;
        case 2: hipLaunchKernelGGL((k_march_pipe_head<B, 2, SH, 3>), grid, block, occupancy_lds(P), s, P.avol, Q); break;
        default: return hipErrorInvalidValue;
        }
    } else {
        switch (method) {
        case 1: hipLaunchKernelGGL((k_march_pipe_head<B, 1, SH>), grid, block, occupancy_lds(P), s, vol, P); break;
        case 2: hipLaunchKernelGGL((k_march_pipe_head<B, 2, SH>), grid, block, occupancy_lds(P), s, vol, P); break;
        default: return hipErrorInvalidValue;
        }
    }
    return hipGetLastError();
}

template <int B, int SH>
static hipError_t seg_head_launch(int method, const float *vol, const Params &P, uint32_t nslots,
                                  hipStream_t s) {
    const uint32_t tail = nslots - P.head_slots;
    const dim3 grid(P.head_slots * (uint32_t)SH + ((tail + 7u) / 8u) * 8u * 2u), block(256);
    if (P.avol) {
        Params Q = P;
        Q.sx = P.asx;
        Q.sy = P.asy;
        Q.sz = P.asz;
        switch (method) {
        case 1: hipLaunchKernelGGL((k_march_seg_head<B, 1, SH, 2, 3>), grid, block, occupancy_lds(P), s, P.avol, Q); break;
        case 2: hipLaunchKernelGGL((k_march_seg_head<B, 2, SH, 2, 3>), grid, block, occupancy_lds(P), s, P.avol, Q); break;
        default: return hipErrorInvalidValue;
        }
    } else {
        switch (method) {
        case 1: hipLaunchKernelGGL((k_march_seg_head<B, 1, SH, 2>), grid, block, occupancy_lds(P), s, vol, P); break;
        case 2: hipLaunchKernelGGL((k_march_seg_head<B, 2, SH, 2>), grid, block, occupancy_lds(P), s, vol, P); break;
        default: return hipErrorInvalidValue;
        }
    }
    return hipGetLastError();
}

template <int B, int S, bool PIPE>
static hipError_t seg_launch(int method, const float *vol, const Params &P, uint32_t nslots,
                             hipStream_t s) {
    const dim3 grid(((nslots + 7u) / 8u) * 8u * S), block(256);
    switch (method) {
    case 0:  // baked statistics, one float per voxel (vr_stats.hip), 32-bit offsets
        if constexpr (B == 1) {
            // a plane's y- / z-rows copy (gather8 MODE 4 / 5)
            if (P.plane_axis == 1)
                hipLaunchKernelGGL((k_march_seg<1, 0, S, PIPE, 4>), grid, block, occupancy_lds(P), s, vol, P);
            else if (P.plane_axis == 2)
                hipLaunchKernelGGL((k_march_seg<1, 0, S, PIPE, 5>), grid, block, occupancy_lds(P), s, vol, P);
            else if (P.plane_axis == 3)  // the 8 x 2 x 2 brick copy (oblique views, MODE 6)
                hipLaunchKernelGGL((k_march_seg<1, 0, S, PIPE, 6>), grid, block, occupancy_lds(P), s, vol, P);
            else
                hipLaunchKernelGGL((k_march_seg<1, 0, S, PIPE>), grid, block, occupancy_lds(P), s, vol, P);
            break;
        }
        return hipErrorInvalidValue;
    case -1:  // baked, 64-bit offsets
        if constexpr (B == 1) {
            hipLaunchKernelGGL((k_march_seg<1, -1, S, PIPE>), grid, block, occupancy_lds(P), s, vol, P);
            break;
        }
        return hipErrorInvalidValue;
    case 1: hipLaunchKernelGGL((k_march_seg<B, 1, S, PIPE>), grid, block, occupancy_lds(P), s, vol, P); break;
    case 2: hipLaunchKernelGGL((k_march_seg<B, 2, S, PIPE>), grid, block, occupancy_lds(P), s, vol, P); break;
    case 3: hipLaunchKernelGGL((k_march_seg<B, 3, S, PIPE>), grid, block, occupancy_lds(P), s, vol, P); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// pipelined windows over an axis-rows copy (P.avol, strides P.asx / asy / asz):
// methods 1/2/3, the record march's arithmetic, gathers addressed in the copy
template <int B, int S>
static hipError_t seg_axis_launch(int method, const Params &P, uint32_t nslots, hipStream_t s) {
    const dim3 grid(((nslots + 7u) / 8u) * 8u * S), block(256);
    Params Q = P;
    Q.sx = P.asx;
    Q.sy = P.asy;
    Q.sz = P.asz;
    switch (method) {
    case 1: hipLaunchKernelGGL((k_march_seg<B, 1, S, true, 3>), grid, block, occupancy_lds(P), s, P.avol, Q); break;
    case 2: hipLaunchKernelGGL((k_march_seg<B, 2, S, true, 3>), grid, block, occupancy_lds(P), s, P.avol, Q); break;
    case 3: hipLaunchKernelGGL((k_march_seg<B, 3, S, true, 3>), grid, block, occupancy_lds(P), s, P.avol, Q); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int B>
static bool seg_b(int method, int S, const float *vol, const Params &P, uint32_t nslots,
                  hipStream_t s, hipError_t &err) {
    if (P.avol && method >= 1 && method <= 3) {  // axis views: pipelined windows only
        switch (S) {
        case -2: err = seg_axis_launch<B, 2>(method, P, nslots, s); return true;
        case -4: err = seg_axis_launch<B, 4>(method, P, nslots, s); return true;
        default: return false;
        }
    }
    // S > 0: plain windows; S < 0: pipelined windows of |S| lanes (the
    // dispatch uses 4, -2 and -4; 2 is kept as the plain counterpart of -2)
    switch (S) {
    case 2: err = seg_launch<B, 2, false>(method, vol, P, nslots, s); return true;
    case 4: err = seg_launch<B, 4, false>(method, vol, P, nslots, s); return true;
    case -2: err = seg_launch<B, 2, true>(method, vol, P, nslots, s); return true;
    case -4: err = seg_launch<B, 4, true>(method, vol, P, nslots, s); return true;
    default: return false;
    }
}

bool launch_march_seg(int nb, int method, int S, const float *vol, const Params &P,
                      uint32_t nslots, hipStream_t s, hipError_t &err) {
    if (method < (nb == 1 ? -1 : 1) || method > 3) return false;
    bool ok = false;
    if (nb == 8 && S == -2 && (method == 1 || method == 2) && P.head_slots > 0 &&
        P.head_slots < nslots && (P.head_slots & 7u) == 0 &&
        (P.head_lanes == -2 || P.head_lanes == -4 || P.head_lanes == -8)) {
        if (P.head_tail == 1)
            err = P.head_lanes == -2 ? pipe_head_launch<8, 2>(method, vol, P, nslots, s)
                : P.head_lanes == -4 ? pipe_head_launch<8, 4>(method, vol, P, nslots, s)
                                     : pipe_head_launch<8, 8>(method, vol, P, nslots, s);
        else
            err = P.head_lanes == -2 ? seg_head_launch<8, 2>(method, vol, P, nslots, s)
                : P.head_lanes == -4 ? seg_head_launch<8, 4>(method, vol, P, nslots, s)
                                     : seg_head_launch<8, 8>(method, vol, P, nslots, s);
        char kind[48];
        snprintf(kind, sizeof kind, "k_march_segp%d_head_%s%s", -P.head_lanes,
                 P.head_tail == 1 ? "pipe" : "segp2",
                 P.avol ? (P.asy == 1 ? "_yrows" : "_zrows") : "");
        note_kernel(kind, nb, method);
        return true;
    }
    switch (nb) {
    case 1: ok = seg_b<1>(method, S, vol, P, nslots, s, err); break;
    case 2: ok = seg_b<2>(method, S, vol, P, nslots, s, err); break;
    case 4: ok = seg_b<4>(method, S, vol, P, nslots, s, err); break;
    case 8: ok = seg_b<8>(method, S, vol, P, nslots, s, err); break;
    default: return false;
    }
    if (ok) {
        char kind[40];
        snprintf(kind, sizeof kind, S < 0 ? "k_march_segp%d%s" : "k_march_seg%d%s", S < 0 ? -S : S,
                 (P.avol && method >= 1 && method <= 3) ? (P.asy == 1 ? "_yrows" : "_zrows")
                 : (nb == 1 && method == 0 && P.plane_axis)
                     ? (P.plane_axis == 1 ? "_plane_yrows" : P.plane_axis == 2 ? "_plane_zrows" : "_plane8")
                 : "");
        note_kernel(kind, nb, method);
    }
    return ok;
}

}  // namespace vr
