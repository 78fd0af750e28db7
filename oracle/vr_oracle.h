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

/* Flexible blocks (methods 8/9/0): the integral-histogram span tables of
 * initCuda's arguments 10-18 (K:1893-1900, loaders C:709-997) and the
 * dataProcessing pre-pass (K:1735-1796).
 *   fractal spans: low/high 4 int32 (x, y, z, 0), 1-based inclusive; code 4
 *     int32 (template id, shift, flip, NE); err nbins (bin id, value) float
 *     pairs per entry (C:773-877);
 *   simple spans: low/high 0-based; count int32; hist nbins (bin id, freq)
 *     float pairs per entry (C:879-949);
 *   templates: ntemplates x nbins floats (C:951-997).
 * Table entry i sits at (i % 64, (i / 64) % 64, i / 4096) of the reference's
 * 64x64x32 lookup textures (K:1352-1370). */
typedef struct {
    int dim;            /* cubic raw volume edge (rawVolumeDim, K:106)          */
    int block;          /* block edge (dataProcessing's blockSize, K:1737)      */
    int nbins;          /* flexNBin (K:97)                                      */
    int n_fractal;
    const int32_t *fractal_low, *fractal_high, *fractal_code;
    const float *fractal_err;
    int n_simple;
    const int32_t *simple_low, *simple_high, *simple_count;
    const float *simple_hist;
    const float *templates;
    int ntemplates;
} orc_flex;

/* histogram sum of the integral-histogram corner (x, y, z) (1-based), K:1142-1544;
 * returns the number of sub-spans, or -1 - k when sub-span k has no table entry */
int orc_flex_corner(const orc_flex *f, int x, int y, int z, float *hist);
/* dataProcessing: per block (mean, variance, entropy, 0) in blocks[nblk^3 * 4],
 * block n = (z * nblk + y) * nblk + x (K:1013-1031, 1033-1126); returns nblk, or
 * a negative value when a sub-span is missing from the tables */
int orc_flex_process(const orc_flex *f, float *blocks);
/* orc_render for methods 8 (entropy), 9 (mean) and 0 (variance) from the block
 * statistics (flexBlockTex, K:654-680, bound K:1691-1714) */
int64_t orc_render_flex(const float *blocks, int nblk, const orc_render_params *p,
                        uint32_t *out, float *out_f, int32_t *out_n, int row_start,
                        int row_stride, int nthreads);

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
int orc_max_threads(void);
/* parity-margin study only: alternative readings of the texture weights, rsqrtf
 * and logf (vr_oracle.c g_w_trunc / g_rsqrt_ulps / g_log_ulps); (0, 0, 0) =
 * the canonical reading.  Not thread-safe: set it before a render. */
void orc_set_reading(int w_trunc, int rsqrt_ulps, int log_ulps);
void orc_synth_fill(int nx, int ny, int nz, int nbins, uint64_t seed, float *vol,
                    int nthreads);

/* ---- GMM distribution volumes (config 5) ----
 * Restates vr_gmm.hip (this build's extension; the reference has no GMM).
 * wm: (w, mu) pairs [voxel][K][2]; sg: sigma [voxel][K]; voxel order
 * x + nx*(y + ny*(z - z_base)) over the resident slices [z_base, z_base + nzs). */
typedef struct {                  /* march state of one ray                     */
    float sum[4];
    float t, pos[3];
    uint32_t pix, n;
} orc_gmm_ray;

/* alive-list entry (vr_gmm.hip GmmRay): 9 uint32 words -- sum[4], t, pos[3]
 * as float bits, then pix | n << 23 (pixel < 2^23, samples <= 500) */
#define ORC_GMM_RAY_WORDS 9

typedef struct {
    const float *wm, *sg;
    int nx, ny, nz, K, z_base, nzs;
} orc_gmm;

/* statistic of one mixture record in the canonical order (vr_gmm.hip header):
 * method 1 mean, 2 variance x 16 */
float orc_gmm_stat(const float *wm_rec, const float *sg_rec, int K, int method);

/* slices [z_base, z_base + nzs) of the synthetic GMM volume */
void orc_synth_gmm(int nx, int ny, int nz, int K, uint64_t seed, int z_base, int nzs, float *wm,
                   float *sg, int nthreads);

/* Render with a GMM volume.  z_lo/z_hi: the slab (samples whose footprint z0
 * lies in [z_lo, z_hi)); whole volume: 0, nz with rays_out == NULL.  rays_in ==
 * NULL: camera rays of the whole frame; else n_in alive-list entries
 * (ORC_GMM_RAY_WORDS words each).  Rays leaving the slab alive are appended to
 * rays_out (in input / raster order),
 * their count stored in *n_out.  out / out_f / out_n as orc_render (pixel
 * y*width + x).  mark: optional footprint bitset over nx*ny*nz voxels.
 * Returns the samples taken. */
int64_t orc_render_gmm(const orc_gmm *v, const orc_render_params *p, int z_lo, int z_hi,
                       const uint32_t *rays_in, uint32_t n_in, uint32_t *rays_out,
                       uint32_t *n_out, uint32_t *out, float *out_f, int32_t *out_n,
                       uint64_t *mark);

/* The synthetic GMM volume as a procedural source: each record computed from
 * its voxel index when a sample reads it (orc_synth_gmm fills its slices through
 * the same function), for frames whose volume no host holds (config 5: 2048^3 x
 * 16 = 1.65 TB). */
typedef struct orc_gmm_proc orc_gmm_proc;
orc_gmm_proc *orc_gmm_proc_new(int nx, int ny, int nz, int K, uint64_t seed);
void orc_gmm_proc_free(orc_gmm_proc *g);

/* whole-volume render of the given rows (any order) of the frame from the
 * procedural source: out / out_n [nrows][width] (out_n -1 = ray misses the box,
 * out 0 there); returns the samples taken, -1 on a bad K (4..32) */
int64_t orc_render_gmm_rows_proc(const orc_gmm_proc *g, const orc_render_params *p,
                                 const int32_t *rows, int nrows, uint32_t *out, int32_t *out_n,
                                 int nthreads);

/* CPU baseline: camera rays of rows [row_lo, row_hi), whole resident volume,
 * OpenMP over rows; returns the samples taken */
int64_t orc_render_gmm_rows(const orc_gmm *v, const orc_render_params *p, int row_lo, int row_hi,
                            uint32_t *out, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
