// vr_internal.h -- declarations shared by the kernels (vr_kernels.hip) and the
// host-side library state / C-ABI (vr_api.cpp).  Not a public header.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vr_device.h"

namespace vr {

constexpr int kSynthBlobs = 8;   // Gaussian blobs of the scalar field
constexpr int kSynthG = 16;      // spread levels
constexpr int kSynthQ = 4096;    // quantised field levels

struct SynthArgs {
    float amp[kSynthBlobs];
    const float *gx, *gy, *gz;   // [k][n] separable blob factors
    const float *table;          // [g][q][nb] normalised histograms
    int nx, ny, nz, nb;
    uint64_t sy, sz;             // record pitch of a row / slice
    uint64_t seed;
};

// the synthetic volumes' hash: k_synth, k_synth_codec
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// records an error for vr_last_error() (vr_api.cpp); returns status
int record_error(int status, const char *msg);

hipError_t launch_march(int nb, int method, const float *vol, const Params &P,
                        uint32_t nslots, bool count, hipStream_t s);
// method 7 (vr_m7.hip; -7: over the baked corner means); launch_march routes to it
hipError_t launch_march_m7(int nb, int method, const float *vol, const Params &P,
                           uint32_t nslots, hipStream_t s);
// name of the march kernel the last non-counting launch_march() chose
const char *last_march_kernel();
void note_kernel(const char *kind, int B, int method);
// ray-segmented march (vr_seg.hip): S lanes per ray; false if (B, S) has no
// specialisation
bool launch_march_seg(int nb, int method, int S, const float *vol, const Params &P,
                      uint32_t nslots, hipStream_t s, hipError_t &err);
// tuning knob `key` set through vr_set_tuning (nullptr if unset); a -DVR_TUNING
// build falls back to the environment.  The default build never reads it.
const char *tuning(const char *key);
hipError_t launch_march_codec(int nb, int method, const Params &P, uint32_t nslots, bool count,
                              hipStream_t s);
hipError_t launch_codec_bytes(const unsigned long long *bits, uint64_t nvox, const int4 *cb,
                              unsigned long long *total, hipStream_t s);
hipError_t launch_codec_check(const int4 *cb, uint64_t n, int ntpl, int nb, int slots,
                              unsigned long long *bad, hipStream_t s);
hipError_t launch_synth_codec(int4 *cb, float2 *err, const SynthArgs &a, int ntpl, int slots,
                              hipStream_t s);
// ---- flexible blocks (methods 8/9/0, vr_flex.hip) ----
// span key: six coordinates of 10 bits, low x/y/z then high x/y/z
__host__ __device__ inline uint64_t span_key(int lx, int ly, int lz, int hx, int hy, int hz) {
    return (uint64_t)lx | (uint64_t)ly << 10 | (uint64_t)lz << 20 | (uint64_t)hx << 30 |
           (uint64_t)hy << 40 | (uint64_t)hz << 50;
}
constexpr int kFlexMaxBins = 64;     // flexNBin (K:97)
constexpr int kFlexMaxDim = 126;     // dyadic split of K:1248-1282 stays within 6 spans per axis
struct FlexTables {                  // device arrays
    int dim, nb;
    const uint64_t *fkeys;           // fractal spans: sorted keys -> chosen entry
    const int32_t *fidx;
    int nfk;
    const int4 *fcode;               // template id, shift, flip, NE
    const float2 *ferr;              // nb (bin, value) pairs per entry
    const uint64_t *skeys;           // simple spans (0-based keys)
    const int32_t *sidx;
    int nsk;
    const int32_t *scount;
    const float2 *shist;             // nb (bin, freq) pairs per entry
    const float *tpl;                // [ntpl][nb]
};
hipError_t launch_flex_corners(const FlexTables &t, int block, int nblk, float *corner_hist,
                               unsigned int *missing, hipStream_t s);
hipError_t launch_flex_blocks(int nb, int nblk, const float *corner_hist, float4 *blocks,
                              hipStream_t s);
hipError_t launch_march_flex(int method, const Params &P, uint32_t nslots, hipStream_t s);
// ---- GMM volumes (config 5, vr_gmm.hip) ----
hipError_t launch_march_gmm(int K, int method, const Params &P, uint32_t nblocks, bool count,
                            hipStream_t s);
hipError_t launch_synth_gmm(float *wm, float *sg, const SynthArgs &a, int K, int z_base, int nzs,
                            hipStream_t s);
// ---- baked statistics (basicDataProcessing, vr_stats.hip): planes of `plane`
// floats each in 16 x 2 x 1 bricks of plane pitches psy / psz (plane_index),
// statistic k+1 (raw) / C = k (codec)
hipError_t launch_bake_raw(const float *vol, const Params &P, float *out, uint64_t plane,
                           uint64_t psy, uint64_t psz, hipStream_t s);
hipError_t launch_bake_codec(const Params &P, float *out, uint64_t plane, uint64_t psy,
                             uint64_t psz, hipStream_t s);
// 2x2 (x, y) micro-brick copy of an 8-bin volume (oblique views, vr_stats.hip):
// pitches bsy (records per brick row) and bsz (records per slice), brick_index
hipError_t launch_brick8(const float *vol, const Params &P, float *out, uint64_t bsy,
                         uint64_t bsz, hipStream_t s);
// axis-rows copy of a B <= 8 volume (views along y / z, vr_stats.hip) with the
// record strides of axis_copy_strides
hipError_t launch_axis_copy(const float *vol, const Params &P, float *out, uint64_t asx,
                            uint64_t asy, uint64_t asz, hipStream_t s);
// axis copy of one baked plane (views along y / z, vr_stats.hip k_plane_axis):
// axis 1 y rows, 2 z rows, into plane_pitches(fast, pair) = (dsy, dsz) bricks
// 8 x 2 x 2 brick copy of one baked plane (oblique views, vr_stats.hip k_plane8)
// into plane8_pitches(nx, ny) = (dsy, dsz) bricks
hipError_t launch_plane8(const float *src, uint64_t ssy, uint64_t ssz, float *out, uint64_t dsy,
                         uint64_t dsz, int nx, int ny, int nz, hipStream_t s);
hipError_t launch_plane_axis(const float *src, uint64_t ssy, uint64_t ssz, float *out,
                             uint64_t dsy, uint64_t dsz, int nx, int ny, int nz, int axis,
                             hipStream_t s);
// streaming read of bytes (a multiple of 16, 16-B aligned) by nblocks workgroups
// of 256 threads; one xor word per workgroup into out (bench read ceiling)
hipError_t launch_stream_read(const void *buf, uint64_t bytes, uint32_t *out, uint32_t nblocks,
                              hipStream_t s);
hipError_t launch_logcheck(unsigned long long *cnt, hipStream_t s);
hipError_t launch_synth(float *vol, const SynthArgs &a, hipStream_t s);
hipError_t launch_unscatter(const uint32_t *packed, const uint32_t *lists, uint32_t ntiles,
                            uint32_t tiles_x, uint32_t *frame, uint32_t W, uint32_t H,
                            hipStream_t s);
hipError_t launch_popcount(const unsigned long long *bits, uint64_t nwords,
                           unsigned long long *total, hipStream_t s);

}  // namespace vr
