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

// records an error for vr_last_error() (vr_api.cpp); returns status
int record_error(int status, const char *msg);

hipError_t launch_march(int nb, int method, const float *vol, const Params &P,
                        uint32_t nslots, bool count, hipStream_t s);
// name of the march kernel the last non-counting launch_march() chose
const char *last_march_kernel();
void note_kernel(const char *kind, int B, int method);
// ray-segmented march (vr_seg.hip): S lanes per ray; false if (B, S) has no
// specialisation
bool launch_march_seg(int nb, int method, int S, const float *vol, const Params &P,
                      uint32_t nslots, hipStream_t s, hipError_t &err);
#ifdef VR_WG_PROF
hipError_t wg_prof_read(unsigned long long *host);   // tooling build only
#endif
hipError_t launch_march_codec(int nb, int method, const Params &P, uint32_t nslots, bool count,
                              hipStream_t s);
hipError_t launch_codec_bytes(const unsigned long long *bits, uint64_t nvox, const int4 *cb,
                              unsigned long long *total, hipStream_t s);
hipError_t launch_codec_check(const int4 *cb, uint64_t n, int ntpl, int nb, int slots,
                              unsigned long long *bad, hipStream_t s);
hipError_t launch_synth_codec(int4 *cb, float2 *err, const SynthArgs &a, int ntpl, int slots,
                              hipStream_t s);
hipError_t launch_logcheck(unsigned long long *cnt, hipStream_t s);
hipError_t launch_synth(float *vol, const SynthArgs &a, hipStream_t s);
hipError_t launch_unscatter(const uint32_t *packed, const uint32_t *lists, uint32_t ntiles,
                            uint32_t tiles_x, uint32_t *frame, uint32_t W, uint32_t H,
                            hipStream_t s);
hipError_t launch_popcount(const unsigned long long *bits, uint64_t nwords,
                           unsigned long long *total, hipStream_t s);

}  // namespace vr
