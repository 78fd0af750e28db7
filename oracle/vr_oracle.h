/*
 * vr_oracle.h -- CPU restatement of the reference d_render path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libvr.so, the Python
 * package) includes, links or calls this code.  Only tests/, the smoke() check
 * in __graft_entry__.py and bench.py's cpu_baseline leg load it, and only as
 * the checker / the reported CPU baseline.
 *
 * Parity status: the reference (CUDA 5.0 + texture hardware) cannot be built or
 * run here and ships no golden image.  This restatement is
 * pinned by analytic known-answer tests (tests/test_oracle.py) and by the
 * committed fixtures in tests/golden/; against real NVIDIA output it is
 * "parity unpinned" (see DESIGN.md section 3).
 */
#ifndef VR_ORACLE_H
#define VR_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int   width, height;          /* imageW, imageH (K:272-274)                 */
    float inv_view[12];           /* c_invViewMatrix, 3 rows of float4 (K:116) */
    float density, brightness;    /* C:130-131                                  */
    float transfer_offset;        /* C:132                                      */
    float transfer_scale;         /* C:133                                      */
    int   query_method;           /* 1 mean, 2 variance, 3 entropy, 7 interp   */
    int   m7_dims[3];             /* render_kernel's volumeSize (K:2399)        */
} orc_render_params;

/* Fractal/template codec (methods 4/5/6), the initCuda arrays of K:1893-1900:
 * codebook: 4 int32 per voxel (template id, shift, flip, NE), voxel order
 *           x + X*(y + Y*z) (C:620, K:777);
 * templates: ntemplates x nbins floats (C:657-675, K:792-793);
 * errors: err_slots (bin id, value) float pairs per voxel, NE used (C:626-641,
 *         K:805-807). */
typedef struct {
    const int32_t *codebook;
    const float *templates;
    int ntemplates;
    const float *errors;
    int err_slots;
} orc_codec;

/* decoded, error-corrected, normalised histogram of voxel vidx (K:775-835) */
void orc_codec_decode(const orc_codec *c, int nbins, size_t vidx, float *dec);
/* its mean / variance / entropy as the fractal pre-pass computes them (K:837-868) */
void orc_codec_stats(const orc_codec *c, int nbins, size_t vidx, float out[3]);

/* orc_render for methods 4/5/6 from a codec-encoded volume */
int64_t orc_render_codec(const orc_codec *codec, int nx, int ny, int nz, int nbins,
                         const orc_render_params *p, uint32_t *out, float *out_f,
                         int32_t *out_n, int row_start, int row_stride, int nthreads);

/* statistic of one B-bin record: d_basicDataProcessing K:736-773 */
void orc_record_stats(const float *rec, int nbins, float out[3]);

/* un-normalised corner mean used by the method-7 path, K:355-366 */
float orc_corner_mean(const float *rec, int nbins);

/* transfer-function lookup (normalised, linear, clamp), K:683-684, 2322-2344 */
void orc_transfer(float x, float out[4]);

/* rgbaFloatToInt, K:186-193 */
uint32_t orc_pack(const float rgba[4]);

/*
 * Render rows row_start, row_start+row_stride, ... of the frame.
 * vol:      AoS fp32 records, vol[((z*ny + y)*nx + x)*nbins + b]  (K:2024-2031)
 * out:      W*H packed RGBA8; miss pixels are left untouched (K:302-303)
 * out_f:    optional W*H*4 floats: the saturated float RGBA that is packed
 * out_n:    optional W*H int32: samples taken per pixel (-1 for a miss)
 * nthreads: OpenMP threads (<=0: library default)
 * returns total samples taken
 */
int64_t orc_render(const float *vol, int nx, int ny, int nz, int nbins,
                   const orc_render_params *p, uint32_t *out, float *out_f,
                   int32_t *out_n, int row_start, int row_stride, int nthreads);

/*
 * U = number of distinct voxel records in the union of all 2x2x2 trilinear
 * footprints of the samples actually taken (methods 1/2/3, early termination
 * honoured).  The algorithmic-bytes figure of SURVEY.md 8(d).
 */
int64_t orc_count_footprint(const float *vol, int nx, int ny, int nz, int nbins,
                            const orc_render_params *p, int nthreads);

/* ---- synthetic distribution volume ---- */
void orc_synth_codec(int nx, int ny, int nz, int nbins, int ntpl, int slots, uint64_t seed,
                     int32_t *codebook, float *templates, float *errors);
uint64_t orc_splitmix64(uint64_t x);
void orc_synth_fill(int nx, int ny, int nz, int nbins, uint64_t seed, float *vol,
                    int nthreads);

#ifdef __cplusplus
}
#endif
#endif
