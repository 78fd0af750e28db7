// vr_codec.hip -- methods 4/5/6 (K:195-222, 639-652, 775-871): the march over
// the fractal/template codec volume, each corner decoded from its codebook
// entry, template row and sparse errors at every step; the codec's footprint
// bytes, validation and synthetic volume.
//
//  k_march_codec       one lane per ray (any B of 1..32)
//  k_march_codec_quad  B = 8 oblique views: a quad decodes a ray's 8 corners
//
// K = volumeRender_kernel.cu of the reference.
#include "vr_device.h"
#include "vr_internal.h"
#include "vr_march.h"
#include "vr_quad.h"

#include <cstdlib>

namespace vr {

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
                         ~(size_t)31) + (method == 6 ? kLogTabN * sizeof(LogEnt) : 0);
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
}  // namespace vr
