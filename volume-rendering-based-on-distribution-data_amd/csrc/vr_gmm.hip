// vr_gmm.hip -- Gaussian-mixture (GMM) distribution volumes: BASELINE config 5
// (2048^3 x 16-component GMM, 3840x2160, 8 GPUs), DESIGN.md section 11.
//
// The reference stores histograms only (K:722-773); a GMM record is this
// build's extension, marched with the reference's own
// ray/step/transfer/composite semantics (K:282-717: the same make_ray,
// footprint, quantised trilinear blend, composite and early exit as methods
// 1/2), decoding the record statistic at every step:
//   mean     m = sum_k w_k mu_k                       (method 1, sample = m)
//   variance v = sum_k w_k (sigma_k^2 + mu_k^2) - m^2  (method 2, sample = 16 v)
// HBM layout: two planes, (w, mu) pairs [voxel][K][2] (8K bytes: 128 B = one
// cache line per voxel at K = 16) and sigma [voxel][K] (4K bytes), so the mean
// reads only the first plane.
//
// Decode across the wavefront: L = K/4 consecutive lanes share one ray (K = 16:
// 4 lanes, 16 rays per wave).  Lane s of the group loads 4 components of each
// corner record (32 bytes of (w, mu), 16 of sigma; the group reads the whole
// record), forms a partial sum, and log2(L) DPP steps complete it on every
// lane of the group.  Four components per lane balances the two costs of a
// ray-step: the record registers (8 corners x 8 floats) and the per-ray work
// every lane of a group repeats (footprint, corner addresses, blend, transfer
// function, composite), which made an 8-lane group VALU-issue-bound.  The
// canonical arithmetic the oracle restates (oracle/vr_oracle.c orc_gmm_*):
//   lane s partials over components k = 4s .. 4s + 3:
//     pm = w_k0 mu_k0;  pm = fma(w_k, mu_k, pm)
//     pq = w_k0 fma(s_k0, s_k0, mu_k0 mu_k0);  pq = fma(w_k, fma(s_k, s_k, mu_k mu_k), pq)
//   T(p) = p0 + p1                                           (L = 2, K = 8)
//        = (p0 + p1) + (p2 + p3)                             (L = 4, K = 16)
//        = ((p0 + p1) + (p2 + p3)) + ((p4 + p5) + (p6 + p7)) (L = 8, K = 32)
//   m = T(pm), v = T(pq) - m m.
//
// Active-ray refill: a wave owns 64 rays (a 64-pixel tile row, or 64 entries
// of an alive list) and marches 64/L at a time; when a group's ray ends (early
// exit, tfar, 500 steps, or leaving the slab) the wave ballots the free
// groups and hands them the next rays by prefix rank (mbcnt), so no lanes idle
// behind a long ray while work remains.
//
// Slabs (out-of-core / multi-GPU sort-last): only the slices
// [z_base, z_base + nzs) are resident; a launch takes the samples whose
// footprint z0 lies in [z_lo, z_hi) and hands every ray that leaves that range
// alive to the next slab as an exact state (sums, t, pos, samples taken), so a
// chain of slab launches in march order reproduces the whole-volume march bit
// for bit.
#include "vr_internal.h"
#include "vr_march.h"

namespace vr {

// alive-list entry: 36 bytes, 9 words -- the colour sums, t, the position and
// the pixel (23 bits: W*H <= 2^23, 3840x2160 fits) with the samples taken
// (9 bits: <= 500, K:381) in one word.  Every ray handed between ranks crosses
// xGMI as one entry, so its size is the chain's hand-off cost.
constexpr int kGmmRayWords = 9;
constexpr uint32_t kGmmPixBits = 23;
struct GmmRay {
    float sx, sy, sz, sw;
    float t, px, py, pz;
    uint32_t pix_n;               // pix | n << 23
};
static_assert(sizeof(GmmRay) == 4 * kGmmRayWords, "GmmRay is 9 words");

// ---- cross-lane sum over an L-lane group, T(p) above ----
template <int CTRL>
__device__ __forceinline__ float dppc(float v) {
    return __int_as_float(
        __builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int L>
__device__ __forceinline__ float group_sum(float p) {
    float s = p + dppc<0xB1>(p);                 // quad_perm [1,0,3,2]: lane ^ 1
    if constexpr (L >= 4) s = s + dppc<0x4E>(s);  // quad_perm [2,3,0,1]: lane ^ 2
    if constexpr (L >= 8) s = s + dppc<0x141>(s); // row_half_mirror: the other quad's sum
    return s;
}

// this lane's 4 components of one corner record
template <int M>
struct GmmPart {
    float4 wm[2];                 // (w, mu) of components 4s .. 4s + 3
    float4 sg[1];                 // sigma of the same components (method 2 only)
};

// statistic of one corner (whole group participates)
template <int L, int M>
__device__ __forceinline__ float gmm_stat(const GmmPart<M> &r) {
    const float4 a = r.wm[0], b = r.wm[1];
    float pm = a.x * a.y;
    pm = __builtin_fmaf(a.z, a.w, pm);
    pm = __builtin_fmaf(b.x, b.y, pm);
    pm = __builtin_fmaf(b.z, b.w, pm);
    const float m = group_sum<L>(pm);
    if constexpr (M == 1) {
        return m;
    } else {
        const float4 c = r.sg[0];
        float pq = a.x * __builtin_fmaf(c.x, c.x, a.y * a.y);
        pq = __builtin_fmaf(a.z, __builtin_fmaf(c.y, c.y, a.w * a.w), pq);
        pq = __builtin_fmaf(b.x, __builtin_fmaf(c.z, c.z, b.y * b.y), pq);
        pq = __builtin_fmaf(b.z, __builtin_fmaf(c.w, c.w, b.w * b.w), pq);
        const float q = group_sum<L>(pq);
        const float mm = m * m;
        return (q - mm) * 16.0f;
    }
}

// ray state of one group (identical on its L lanes)
struct GmmState {
    Ray r;
    float t, px, py, pz, stx, sty, stz;
    float sx, sy, sz, sw;
    uint32_t pix;
    int n;
};

// Sets up the ray of entry e (frame mode: pixel e of the wave's tile row;
// list mode: alive-list entry e).  Returns false if the entry holds no ray
// (outside the image or the list, or a miss -- written as the reference does).
__device__ __forceinline__ bool gmm_begin(const Params &P, uint32_t wave_base, uint32_t e,
                                          uint32_t row_x0, uint32_t row_y, bool write,
                                          GmmState &s) {
    uint32_t x, y;
    const GmmRay *in = nullptr;
    if (P.rays_in) {
        const uint32_t k = wave_base + e;
        if (k >= P.n_rays_in) return false;
        in = reinterpret_cast<const GmmRay *>(P.rays_in) + k;
        s.pix = in->pix_n & ((1u << kGmmPixBits) - 1u);
        x = s.pix % P.W;
        y = s.pix / P.W;
    } else {
        x = row_x0 + e;
        y = row_y;
        if (x >= P.CW || y >= P.CH) return false;
        s.pix = y * P.W + x;
    }
    if (!make_ray(P, x, y, s.r)) {
        if (write) write_miss(P, s.pix);
        return false;
    }
    s.stx = s.r.dx * kTStep;
    s.sty = s.r.dy * kTStep;
    s.stz = s.r.dz * kTStep;
    if (in) {
        s.sx = in->sx; s.sy = in->sy; s.sz = in->sz; s.sw = in->sw;
        s.t = in->t; s.px = in->px; s.py = in->py; s.pz = in->pz;
        s.n = (int)(in->pix_n >> kGmmPixBits);
    } else {
        s.sx = s.sy = s.sz = s.sw = 0.0f;
        s.t = s.r.tnear;
        s.px = s.r.ox + s.r.dx * s.r.tnear;
        s.py = s.r.oy + s.r.dy * s.r.tnear;
        s.pz = s.r.oz + s.r.dz * s.r.tnear;
        s.n = 0;
    }
    return true;
}

// linear voxel index of (x, y, z) in the resident slices
__device__ __forceinline__ uint64_t gmm_vox(const Params &P, int x, int y, int z) {
    return ((uint64_t)(z - P.z_base) * (uint64_t)P.ny + (uint64_t)y) * (uint64_t)P.nx + (uint64_t)x;
}

// the 8 corner records' 4-component chunks of lane `sub`: one 64-bit base
// address, the other corners by 32-bit offsets (x pair 0/1 record, y pair
// 0/1 row, z pair 0/1 slice; a slice is < 2^32 bytes for nx*ny <= 2^26 / K).
// z is clamped to the resident slices (a slab's discarded last look-ahead).
template <int K, int M>
__device__ __forceinline__ void gmm_gather(const Params &P, const Foot &f, uint32_t sub,
                                           GmmPart<M> (&r)[8]) {
    const int zl = P.z_base, zh = P.z_base + P.nzs - 1;
    const int z0 = min(max(f.z0, zl), zh), z1 = min(max(f.z1, zl), zh);
    const uint64_t v = gmm_vox(P, f.x0, f.y0, z0);
    const uint32_t ox = (uint32_t)(f.x1 - f.x0);
    const uint32_t oy = (uint32_t)(f.y1 - f.y0) * (uint32_t)P.nx;
    const uint32_t oz = (uint32_t)(z1 - z0) * (uint32_t)P.nx * (uint32_t)P.ny;
    const uint32_t off[8] = {0u, ox, oy, ox + oy, oz, oz + ox, oz + oy, oz + oy + ox};
    const float4 *a = reinterpret_cast<const float4 *>(P.gwm + v * (2u * K)) + sub * 2u;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const float4 *q = a + (size_t)off[j] * (K / 2);
        r[j].wm[0] = q[0];
        r[j].wm[1] = q[1];
    }
    if constexpr (M == 2) {
        const float4 *b = reinterpret_cast<const float4 *>(P.gsg + v * K) + sub;
#pragma unroll
        for (int j = 0; j < 8; j++) r[j].sg[0] = b[(size_t)off[j] * (K / 4)];
    }
}

// appends the group's ray to the alive list (groups of the wave that leave
// together share one atomic)
template <int L>
__device__ __forceinline__ void gmm_emit(const Params &P, const GmmState &s, uint32_t lane,
                                         uint32_t sub) {
    const uint64_t out = __ballot(sub == 0);
    uint32_t base = 0;
    if (lane == (uint32_t)__builtin_ctzll(out))
        base = atomicAdd(P.n_rays_out, (uint32_t)__popcll(out));
    base = __shfl(base, __builtin_ctzll(out), 64);
    const uint32_t k = base + (uint32_t)__popcll(out & ((1ull << (lane & ~(uint32_t)(L - 1))) - 1ull));
    // the list's capacity (include/vr.h): no slab emits more rays than enter
    // it and the library zeroes the counter before the launch, so this is a
    // second guard -- entries past it are dropped, never written past the end
    const uint64_t cap = P.rays_in ? (uint64_t)P.n_rays_in : (uint64_t)P.W * P.H;
    if ((uint64_t)k < cap) {
        // the group's L lanes share the 9 words: lane sub writes words sub,
        // sub + L, ... (K = 8: two lanes, five and four words)
        const uint32_t w[kGmmRayWords] = {
            __float_as_uint(s.sx), __float_as_uint(s.sy), __float_as_uint(s.sz),
            __float_as_uint(s.sw), __float_as_uint(s.t), __float_as_uint(s.px),
            __float_as_uint(s.py), __float_as_uint(s.pz),
            s.pix | ((uint32_t)s.n << kGmmPixBits)};
        uint32_t *dst = P.rays_out + (uint64_t)k * kGmmRayWords;
#pragma unroll
        for (int j = 0; j < kGmmRayWords; j++)
            if ((uint32_t)(j % L) == sub) dst[j] = w[j];
    }
}

#ifndef VR_GMM_WAVES
#define VR_GMM_WAVES 1
#endif
template <int K, int M, bool COUNT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VR_GMM_WAVES, 8))) void k_march_gmm(Params P) {
    constexpr int L = K / 4;              // lanes per ray
    constexpr uint32_t R = 64u / L;       // rays in flight per wave
    static_assert(L == 2 || L == 4 || L == 8, "K = 8, 16 or 32");
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t g = lane / L, sub = lane % L;
    uint32_t wave_base = 0, row_x0 = 0, row_y = 0;
    if (P.rays_in) {
        wave_base = (blockIdx.x * 4u + wave) * 64u;
        if (wave_base >= P.n_rays_in) return;
    } else {
        const uint32_t slot = launch_slot(P);
        const uint32_t tile = tile_of(P, slot);
        if (tile == kPad) return;
        row_x0 = (tile % P.tiles_x) * kTileW;
        row_y = (tile / P.tiles_x) * kTileH + wave;
    }
    GmmState s;
    uint32_t next = R;          // wave-uniform: entries handed out so far
    bool act = gmm_begin(P, wave_base, g, row_x0, row_y, sub == 0, s);
    const uint64_t below = (1ull << (lane & ~(uint32_t)(L - 1))) - 1ull;  // lanes of earlier groups
    while (true) {
        // refill groups without a ray (ballot over the groups' first lanes,
        // prefix rank among them)
        // P.path == 1 (VR_GMM_LOCKSTEP): a new batch only when the whole wave is
        // idle, so the wave's rays stay adjacent and at the same step
        while (!(P.path == 1 && __ballot(act) != 0)) {
            const uint64_t idle = __ballot(!act && sub == 0);
            if (idle == 0 || next >= 64) break;
            const uint32_t e = next + (uint32_t)__popcll(idle & below);
            if (!act && e < 64) act = gmm_begin(P, wave_base, e, row_x0, row_y, sub == 0, s);
            next += __popcll(idle);
        }
        if (__ballot(act) == 0) break;
        if (act) {
            const Foot f = footprint(P, s.px, s.py, s.pz);
            if (P.rays_out && (f.z0 < P.z_lo || f.z0 >= P.z_hi)) {
                gmm_emit<L>(P, s, lane, sub);  // leaves the slab alive: exact state onwards
                act = false;
            } else {
                if constexpr (COUNT) {
                    if (sub == 0) {
                        mark_voxel(P.mark, gmm_vox(P, f.x0, f.y0, f.z0)); mark_voxel(P.mark, gmm_vox(P, f.x1, f.y0, f.z0));
                        mark_voxel(P.mark, gmm_vox(P, f.x0, f.y1, f.z0)); mark_voxel(P.mark, gmm_vox(P, f.x1, f.y1, f.z0));
                        mark_voxel(P.mark, gmm_vox(P, f.x0, f.y0, f.z1)); mark_voxel(P.mark, gmm_vox(P, f.x1, f.y0, f.z1));
                        mark_voxel(P.mark, gmm_vox(P, f.x0, f.y1, f.z1)); mark_voxel(P.mark, gmm_vox(P, f.x1, f.y1, f.z1));
                    }
                }
                GmmPart<M> rc[8];
                gmm_gather<K, M>(P, f, sub, rc);
                float sv[8];
#pragma unroll
                for (int j = 0; j < 8; j++) sv[j] = gmm_stat<L, M>(rc[j]);
                s.n = s.n + 1;
                bool end = composite(P, blend8(sv, f), s.sx, s.sy, s.sz, s.sw);  // K:698
                if (!end) {
                    s.t = s.t + kTStep;                                          // K:701
                    end = s.t > s.r.tfar || s.n >= kMaxSteps;                    // K:703, K:381
                    s.px = s.px + s.stx;                                         // K:706
                    s.py = s.py + s.sty;
                    s.pz = s.pz + s.stz;
                }
                if (end) {
                    if (!COUNT && sub == 0)
                        write_pixel(P, s.pix, s.n, s.sx * P.brightness, s.sy * P.brightness,
                                    s.sz * P.brightness, s.sw * P.brightness);
                    act = false;
                }
            }
        }
    }
}

template <int K, int M, bool COUNT>
static void launch_gmm_km(const Params &P, uint32_t nblocks, hipStream_t s) {
    hipLaunchKernelGGL((k_march_gmm<K, M, COUNT>), dim3(nblocks), dim3(256), occupancy_lds(P), s, P);
}

template <int K>
static hipError_t launch_gmm_k(int method, const Params &P, uint32_t nblocks, bool count,
                               hipStream_t s) {
    if (count) {  // the samples (and so the footprints) depend on the statistic
        if (method == 1) launch_gmm_km<K, 1, true>(P, nblocks, s);
        else if (method == 2) launch_gmm_km<K, 2, true>(P, nblocks, s);
        else return hipErrorInvalidValue;
    } else if (method == 1) {
        note_kernel("k_march_gmm", K, 1);
        launch_gmm_km<K, 1, false>(P, nblocks, s);
    } else if (method == 2) {
        note_kernel("k_march_gmm", K, 2);
        launch_gmm_km<K, 2, false>(P, nblocks, s);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_march_gmm(int K, int method, const Params &P, uint32_t nblocks, bool count,
                            hipStream_t s) {
    if (nblocks == 0) return hipSuccess;
    switch (K) {
    case 8: return launch_gmm_k<8>(method, P, nblocks, count, s);
    case 16: return launch_gmm_k<16>(method, P, nblocks, count, s);
    case 32: return launch_gmm_k<32>(method, P, nblocks, count, s);
    default: return hipErrorInvalidValue;
    }
}

// ---- synthetic GMM volume ----
// The section-5 blob field f places the mixture: per component k of voxel v
// (global index x + nx*(y + ny*z)), h = splitmix64(seed ^ 0x6A09E667F3BCC909 ^
// (v*K + k)), a = (h >> 40) 2^-24, r = 0.05 + ((h >> 16) & 0xFFFFFF) 2^-24,
// mu = clamp((0.8 f + 0.1) + 0.2 (a - 0.5), 0, 1),
// sigma = ((h & 0xFFFF) 2^-16) 0.05 + 0.005, w = r / sum_k r (float, in order).
__device__ __forceinline__ uint64_t gmm_hash(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_synth_gmm(float *__restrict__ wm, float *__restrict__ sg,
                                                   SynthArgs a, int K, int z_base, int nzs) {
    const uint64_t nvox = (uint64_t)a.nx * a.ny * (uint64_t)nzs;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t lv = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; lv < nvox; lv += stride) {
        const uint32_t x = (uint32_t)(lv % (uint64_t)a.nx);
        const uint64_t yz = lv / (uint64_t)a.nx;
        const uint32_t y = (uint32_t)(yz % (uint64_t)a.ny);
        const uint32_t z = (uint32_t)(yz / (uint64_t)a.ny) + (uint32_t)z_base;
        float f = 0.0f;
#pragma unroll
        for (int k = 0; k < kSynthBlobs; k++)
            f = f + ((a.amp[k] * a.gx[k * a.nx + x]) * a.gy[k * a.ny + y]) * a.gz[k * a.nz + z];
        if (f > 1.0f) f = 1.0f;
        const uint64_t v = ((uint64_t)z * a.ny + y) * a.nx + x;
        float sum = 0.0f;
        for (int k = 0; k < K; k++) {
            const uint64_t h = gmm_hash(a.seed ^ 0x6A09E667F3BCC909ull ^ (v * (uint64_t)K + (uint64_t)k));
            const float r = 0.05f + (float)((h >> 16) & 0xFFFFFFull) * 0x1p-24f;
            sum = sum + r;
        }
        for (int k = 0; k < K; k++) {
            const uint64_t h = gmm_hash(a.seed ^ 0x6A09E667F3BCC909ull ^ (v * (uint64_t)K + (uint64_t)k));
            const float u = (float)(h >> 40) * 0x1p-24f;
            const float r = 0.05f + (float)((h >> 16) & 0xFFFFFFull) * 0x1p-24f;
            float mu = (f * 0.8f + 0.1f) + (u - 0.5f) * 0.2f;
            mu = fminf(fmaxf(mu, 0.0f), 1.0f);
            const float sig = ((float)(h & 0xFFFFull) * 0x1p-16f) * 0.05f + 0.005f;
            wm[(lv * K + k) * 2u] = r / sum;
            wm[(lv * K + k) * 2u + 1u] = mu;
            sg[lv * K + k] = sig;
        }
    }
}

hipError_t launch_synth_gmm(float *wm, float *sg, const SynthArgs &a, int K, int z_base, int nzs,
                            hipStream_t s) {
    const uint64_t nvox = (uint64_t)a.nx * a.ny * (uint64_t)nzs;
    uint64_t blocks = (nvox + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_synth_gmm, dim3((uint32_t)blocks), dim3(256), 0, s, wm, sg, a, K, z_base,
                       nzs);
    return hipGetLastError();
}

}  // namespace vr
