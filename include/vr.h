/*
 * vr.h -- C-ABI of libvr.so, the MI355X (gfx950) drop-in for the d_render path
 * of ykou/Volume-Rendering-Based-on-Distribution-Data.
 *
 * Citations: K = volumeRender_kernel.cu, C = volumeRender.cpp (reference).
 *
 * Part 1 -- the reference's own extern "C" entry points (declared C:156-170),
 * same names, argument order and meaning.  vr_dim3 / vr_extent are
 * layout-identical to dim3 (3 x uint32) and cudaExtent/hipExtent (3 x size_t),
 * so a caller written against the reference header links unchanged.
 *
 * Part 2 -- extensions (vr_*): explicit-parameter render with tile lists for
 * the multi-GPU image split, on-device synthetic volumes, the footprint counter
 * used for the roofline, and error reporting.  The library never calls exit():
 * failures are recorded for vr_last_error() (the reference's checkCudaErrors
 * printed and exited, C:201-216).
 *
 * Threading: like the reference, all state is module-global and the entry
 * points are not thread-safe (K:22-88, 116).  One process drives one GPU.
 */
#ifndef VR_H
#define VR_H

#include <stddef.h>
#include <stdint.h>
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { uint32_t x, y, z; } vr_dim3;                /* == dim3       */
typedef struct { size_t width, height, depth; } vr_extent;   /* == cudaExtent */
typedef struct { int32_t x, y, z, w; } vr_int4;               /* == int4       */
typedef struct { float x, y; } vr_float2;                     /* == float2     */

/* ---------------- Part 1: reference entry points ------------------------- */

/* Replaces render_kernel, K:2387-2401.  Launches the per-ray march into the
 * caller-owned device buffer d_output (imageW*imageH packed RGBA8, row-major,
 * A<<24|B<<16|G<<8|R).  Miss pixels are not written (caller zeroes, C:208).
 * gridSize/blockSize keep their meaning -- pixels with x < gridSize.x*blockSize.x
 * and y < gridSize.y*blockSize.y are rendered (K:282-286), the rest of the
 * image is left untouched; an empty grid/block or more than 1024 threads per
 * block is an invalid launch (VR_ERR_ARG, nothing rendered) -- but not their
 * geometry: the library picks its own gfx950 launch (64x4-pixel tiles, one
 * 64-pixel row per wave).
 * volumeSize is used exactly where the reference uses it: the method-7 corner
 * grid (K:322-352).  queryMethod: 1 mean, 2 variance, 3 entropy,
 * 7 software-interpolated mean, 4/5/6 fractal-codec mean / variance / entropy
 * (needs the codec arrays of initCuda or vr_init_codec), 8/9/0 flexible-block
 * entropy / mean / variance (needs dataProcessing or vr_flex_process after the
 * span tables of initCuda or vr_init_flex).  Asynchronous on the library stream (default: null stream),
 * like the reference's default-stream launch. */
void render_kernel(vr_dim3 gridSize, vr_dim3 blockSize, uint32_t *d_output,
                   uint32_t imageW, uint32_t imageH, float density, float brightness,
                   float transferOffset, float transferScale, int queryMethod,
                   vr_extent volumeSize);

/* Replaces copyInvViewMatrix, K:2403-2406: 3 rows of float4 (48 bytes). */
void copyInvViewMatrix(float *invViewMatrix, size_t sizeofMatrix);

/* Replaces initCuda, K:1893-2358 (declared C:157-163 with arg 1 as void*).
 * h_histogram: fp32 records, record r = bins [r*B, r*B+B) where
 * B = histogramSize.width and r = x + X*(y + Y*z) -- the reference's layered
 * layout (bin, r % height, r / height) is exactly this AoS order (K:363-364).
 * histogramSize.height*depth must equal volumeSize.width*height*depth.
 * Args 4-9 (codebook, templates, errorsbook and their sizes) make the codec
 * volume of methods 4/5/6 resident when all three arrays are non-null (see
 * vr_init_codec); the flexible-block span tables (args 10-18) are made
 * resident when all nine are non-null, with the reference's fixed sizes
 * (64x64x32 fractal and simple entries, 64 bins, 469 templates, 64^3 raw
 * volume, K:93-106; see vr_init_flex). */
void initCuda(void *h_histogram, vr_extent volumeSize, vr_extent histogramSize,
              vr_int4 *h_codebook, vr_extent codebookSize, float *h_templates,
              vr_extent templatesSize, vr_float2 *h_errorsbook, vr_extent errorsbookSize,
              vr_int4 *h_codebookSpanLow, vr_int4 *h_codebookSpanHigh,
              vr_int4 *h_flexibleCodebook, vr_float2 *h_flexibleErrorsbook,
              vr_int4 *h_simpleLow, vr_int4 *h_simpleHigh, int *h_simpleCount,
              vr_float2 *h_simpleHistogram, float *h_flexibleTemplates);

/* Replaces freeCudaBuffers, K:2360-2385. */
void freeCudaBuffers(void);

/* Replaces setTextureFilterMode, K:1889-1891.  In the reference it switches the
 * filter of the integer index volume `tex`, which methods 1/2/3 never sample;
 * the flag is stored and has no effect on any supported method. */
void setTextureFilterMode(bool bLinearFilter);

/* Replaces basicDataProcessing, K:1798-1887.  The reference pre-bakes per-voxel
 * mean/variance/entropy of the raw volume (originalQueryTex, K:722-773) and of
 * the codec volume (fractalQueryTex, K:775-871) into float4 textures.  Here the
 * same statistics are baked once into three float planes per resident volume
 * (vr_bake_stats); frames of methods 1-7 then read the planes instead of
 * decoding the corner records at every step -- bit-identical output, 4 bytes
 * per corner voxel read instead of a whole record.  Without it (or after
 * vr_release_stats) the march decodes the records per step.  Errors (no
 * volume, out of memory) go to vr_last_error(); the per-step decode stays. */
void basicDataProcessing(void);

/* Replaces dataProcessing, K:1735-1796: the flexible-block pre-pass of
 * methods 8/9/0 with the reference's block edge of 6 voxels (K:1737), i.e.
 * vr_flex_process(6). */
void dataProcessing(void);

/* ---------------- Part 2: extensions ------------------------------------- */

#define VR_OK 0
#define VR_ERR_ARG -1
#define VR_ERR_STATE -2
#define VR_ERR_HIP -3
#define VR_ERR_UNSUPPORTED -4

/* Baked statistics (basicDataProcessing).  vr_bake_stats bakes the planes of
 * the resident raw and codec volumes that are not baked yet: 4 planes for the
 * raw volume (mean, variance, entropy and method 7's undivided corner mean)
 * and 3 for the codec volume (methods 4/5/6).  A plane is laid out in
 * 16 x 2 x 1 bricks whose x runs overlap by one voxel: with
 * sy = ((X - 1) / 15 + 1) * 32 and sz = ((Y + 1) / 2) * sy floats, voxel
 * (x, y, z) sits at z * sz + (y / 2) * sy + (y % 2) * 16 + (x / 15) * 32 +
 * x % 15 (and, for x = 15 k > 0, also at offset 15 of brick k - 1); a plane
 * holds sz * Z floats.  Re-uploading or releasing a volume drops its planes; a volume
 * modified in place through vr_volume_info's pointer must be re-baked
 * (vr_release_stats, then vr_bake_stats).  vr_stats_info: device pointers
 * (nullptr = not baked) and plane lengths in floats.
 * Layout copy: the first oblique-view frame of a library-owned 8-bin volume
 * makes a second, 2x2 (x, y) micro-brick copy of its records (DESIGN.md 2;
 * as many bytes as the volume, made synchronously, only while HBM keeps
 * max(4 GiB, 5 %) free after it).  Views whose screen x runs along the volume's
 * z or y axis (|M[8]| or |M[4]| >= 0.95) of an owned volume with 1, 2, 4 or 8
 * bins get an axis-rows copy (that axis contiguous) on the same terms, one
 * axis (both a y and a z copy when they fit; one is dropped for the other only
 * when that makes room).  vr_release_stats drops the copies with the planes, so
 * after an in-place modification the next frame that needs one rebuilds it. */
int vr_bake_stats(void);
int vr_release_stats(void);
int vr_stats_info(const float **d_raw, uint64_t *raw_plane, const float **d_codec,
                  uint64_t *codec_plane);

/* Layout copies (the micro-brick and axis-rows copies above) are made only
 * within a byte budget: vr_set_layout_budget(bytes) caps their total HBM
 * (default UINT64_MAX = two record-volume copies plus three baked-plane
 * copies, 1/8 padding each, plus 64 MiB for small volumes' padding: one view
 * class and one change of view; a baked plane's copy is kept per (view axis,
 * method) while the budget holds it, so alternating methods builds each once;
 * 0 = never make
 * one, every view marches the records' x rows) and drops resident copies that
 * exceed a lowered budget.  vr_layout_info: bytes resident in copies, copies
 * made since load, and the time and size of the last one made (each is built
 * synchronously inside the first frame that needs it, so that frame costs
 * last_build_ms more). */
int vr_set_layout_budget(uint64_t bytes);
int vr_layout_info(uint64_t *resident_bytes, int *builds, float *last_build_ms,
                   uint64_t *last_build_bytes);

/* last error message ("" if none); vr_clear_error resets it */
const char *vr_last_error(void);
int vr_last_status(void);
void vr_clear_error(void);

/* Volume residency.  bins: fp32 AoS records as in initCuda.
 * where: 0 = host pointer (copied), 1 = device pointer (copied),
 *        2 = device pointer adopted (not freed by the library). */
int vr_init_distribution(const float *bins, vr_extent dims, int nbins, int where);

/* Generate the seeded synthetic distribution volume of DESIGN.md section 5
 * directly in HBM (library-owned). */
int vr_synthesize(vr_extent dims, int nbins, uint64_t seed);

/* Fractal/template codec volume for methods 4/5/6 (the initCuda arrays of
 * K:1893-1900, as the reference's loaders fill them, C:558-675):
 *   codebook  dims.width*height*depth x (template id, shift, flip, NE), voxel
 *             order x + X*(y + Y*z);
 *   templates ntemplates x nbins floats;
 *   errors    err_slots (bin id, value) pairs per voxel, the first NE used.
 * where: 0 = host arrays, 1 = device arrays (copied).  Entries are validated
 * (template id < ntemplates, 0 <= shift < nbins, 0 <= NE <= err_slots);
 * error bin ids outside [0, nbins) are skipped at decode.  nbins must be one
 * of 1, 2, 4, 8, 16, 32.  initCuda calls this when its codebook, templates and
 * errorsbook arguments are non-null. */
int vr_init_codec(const vr_int4 *codebook, vr_extent dims, const float *templates,
                  int ntemplates, const vr_float2 *errors, int err_slots, int nbins, int where);

/* Generate the seeded synthetic codec volume of DESIGN.md section 5 in HBM
 * (the section-5 scalar field encoded against ntemplates templates, `slots`
 * error pairs per voxel). */
int vr_synthesize_codec(vr_extent dims, int nbins, int ntemplates, int slots, uint64_t seed);

/* shape and device arrays of the resident codec volume (codebook int4 per
 * voxel, templates [ntemplates][nbins] fp32, errors [voxel][slots] float2) */
int vr_codec_info(vr_extent *dims, int *nbins, int *ntemplates, int *slots,
                  const void **codebook, const float **templates, const void **errors);

/* Flexible-block span tables (methods 8/9/0): an integral histogram of a cubic
 * dim^3 raw volume stored as dyadic spans, as the reference's loaders fill
 * initCuda's arguments 10-18 (C:709-997):
 *   fractal_*  spans of >= 8 voxels, 1-based inclusive low/high (x, y, z, -);
 *              code (template id, shift, flip, NE); errors nbins (bin id,
 *              value) pairs per entry, the first NE used (C:773-877);
 *   simple_*   spans of < 8 voxels, 0-based inclusive low/high; count and
 *              nbins (bin id, frequency) pairs per entry (C:879-949);
 *   templates  ntemplates x nbins floats (C:951-997).
 * Entry i of a table stands where the reference's 64x64x32 lookup texture
 * holds it (x = i % 64, y = i / 64 % 64, z = i / 4096); a span listed twice
 * resolves like the reference's scan (K:1352-1372: the last 64-entry row
 * holding it, first entry in that row).  Validated: 1 <= dim <= 126,
 * 1 <= nbins <= 64, template id < ntemplates, 0 <= shift < nbins,
 * 0 <= NE <= nbins, 0 <= count <= nbins.  Host arrays, copied. */
typedef struct {
    int dim;
    int nbins;
    int n_fractal;
    const vr_int4 *fractal_low, *fractal_high, *fractal_code;
    const vr_float2 *fractal_errors;
    int n_simple;
    const vr_int4 *simple_low, *simple_high;
    const int32_t *simple_count;
    const vr_float2 *simple_hist;
    const float *templates;
    int ntemplates;
} vr_flex_tables;

int vr_init_flex(const vr_flex_tables *tables);

/* The dataProcessing pre-pass (K:1735-1796) with blocks of `block` voxels per
 * axis (the last one cut at dim): per-block mean / variance / entropy of the
 * span-table histogram (K:1033-1126), resident for methods 8/9/0.  Returns the
 * blocks per axis, or a negative status (VR_ERR_ARG if some sub-span a block
 * corner needs has no table entry).  Synchronous. */
int vr_flex_process(int block);

/* blocks per axis, bins and device array (blocks^3 x float4 (mean, variance,
 * entropy, 0), block (x, y, z) at x + n*(y + n*z)) of the resident statistics */
int vr_flex_info(int *nblk, int *nbins, const float **d_blocks);

/* dims, bin count and device pointer of the resident volume */
int vr_volume_info(vr_extent *dims, int *nbins, const float **d_bins);

/* Record pitch of a voxel row and of a slice of the resident volume in HBM
 * (record (x,y,z) starts at d_bins + (z*slice_pitch + y*row_pitch + x)*nbins). */
int vr_volume_layout(size_t *row_pitch, size_t *slice_pitch);

/* Stream for all subsequent launches (hipStream_t; NULL = null stream). */
int vr_set_stream(void *stream);

/* Tuning knobs (tests and tools): kernel-path overrides ("VR_PATH" 0 quad,
 * 1 LDS-box, 2 per-ray pipelined, 4 wave-staged, 7 ray-segmented; "VR_SEG"
 * lanes per ray 2/4, pipelined -2/-4), occupancy caps ("VR_WG_PER_CU"),
 * layout experiments ("VR_PAD", "VR_BRICK", ...).
 * value NULL removes a knob; vr_clear_tuning removes all.  Every knob only
 * changes which kernel computes a frame, never its pixels.  The library reads
 * no environment variables (a build with -DVR_TUNING also takes unset knobs
 * from the environment, for tooling). */
int vr_set_tuning(const char *key, const char *value);
void vr_clear_tuning(void);

/* Explicit-parameter render.  With d_tile_list == NULL the whole frame is
 * rendered into d_output[y*width + x].  Otherwise the n_tiles 64x4-pixel
 * tiles named by d_tile_list (tile id = ty*ceil(width/64) + tx, device array)
 * are rendered into a packed buffer: tile slot s occupies
 * d_output[s*256 .. s*256+255] in row-major 64x4 order.  Entries of
 * 0xFFFFFFFF in the tile list are padding and are skipped.  Entry s is
 * rendered by workgroup s, which runs on XCD s % 8 (each XCD has its own L2):
 * order the list so every 8th entry forms an equally loaded, spatially
 * compact set (tiles.py tile_lists does).  Full frames use the library's own
 * XCD-balanced order.
 * In tile-list mode miss pixels are written as 0, so packed buffers need no
 * clearing between frames (full frames keep the reference's behaviour: misses
 * untouched).
 * d_output_f (optional) receives the saturated float RGBA of every written
 * pixel, d_steps (optional) the samples taken (-1 for a miss; written for
 * every pixel inside the image). */
typedef struct {
    uint32_t *d_output;
    float *d_output_f;
    int32_t *d_steps;
    uint32_t width, height;
    float inv_view[12];
    float density, brightness, transfer_offset, transfer_scale;
    int query_method;
    vr_extent volume_size;          /* method-7 grid (render_kernel's volumeSize) */
    const uint32_t *d_tile_list;
    uint32_t n_tiles;
} vr_render_desc;

int vr_render(const vr_render_desc *desc);

/* U of SURVEY.md 8(d): distinct voxel records in the union of the trilinear
 * footprints of all samples taken (methods 1/2/3).  Synchronous; allocates a
 * bitset of voxels/8 bytes.  Returns U, or a negative status. */
int64_t vr_count_footprint(const vr_render_desc *desc);

/* Algorithmic bytes of one launch's volume reads: methods
 * 1/2/3: U * nbins * 4; methods 4/5/6: 16 bytes of codebook and 8 bytes per
 * used error pair for every distinct voxel the footprints touch, plus the
 * template table once.  Synchronous.  Returns bytes or a negative status. */
int64_t vr_footprint_bytes(const vr_render_desc *desc);

/* Rank-0 assembly of the multi-GPU frame: d_packed holds n_ranks x n_slots
 * tiles (each 256 uint32) gathered from the ranks, d_tile_lists the matching
 * n_ranks x n_slots tile ids (0xFFFFFFFF = padding); every listed tile is
 * copied into d_frame (width x height, pixels outside the image dropped). */
int vr_unscatter_tiles(const uint32_t *d_packed, const uint32_t *d_tile_lists,
                       uint32_t n_ranks, uint32_t n_slots, uint32_t *d_frame,
                       uint32_t width, uint32_t height);

/* tiles (64 wide, 4 high) across / down a width x height frame */
uint32_t vr_tiles_x(uint32_t width);
uint32_t vr_tiles_y(uint32_t height);

/* name and template arguments of the march kernel the last vr_render /
 * render_kernel call launched (e.g. "k_march_quad<B=8,M=1>"), "" before any */
const char *vr_last_kernel(void);

/* Tooling: while d_buf is non-null, every launch of the per-ray pipelined,
 * quad and ray-segmented marches overwrites 3 uint64 per wave (no zeroing
 * needed, nothing accumulates): wall clock at the
 * wave's start and end (100 MHz) and __smid() (CU id, XCC id in the high
 * bits), at d_buf[(slot*4 + wave)*3] (pipelined, quad), d_buf[(slot*8 +
 * half*4 + wave)*3] (k_march_quad2) or d_buf[(slot*16 + part*4 + wave)*3]
 * (segmented).  d_buf must hold 48 * n_slots values.  nullptr turns it off. */
int vr_debug_wave_clock(uint64_t *d_buf);

/* Tooling: d_buf = 6 x uint64 of device memory, zeroed by this call on the
 * library's stream (vr_set_stream); while it is non-null, every launch of the
 * staged marches (k_march, k_march_duo) of a library built with -DVR_BOX_CHECK
 * accumulates into it: d_buf[0] = reads whose box index or footprint falls
 * outside the wave's box (each such read is skipped), d_buf[1] = the largest
 * box index + 1 - box voxels seen, d_buf[2] = box voxels of a box whose far
 * corner lies outside the volume; and the decode work: d_buf[3] = box voxels
 * decoded, d_buf[4] = lane slots spent on them (64 per group); d_buf[5] is
 * unused.  Returns 1 for a checking build, 0 for the default build (which
 * counts nothing). */
int vr_debug_box_check(uint64_t *d_buf);

/* Device self-test: compares the entropy decode's fast float logarithms (the
 * series form and the table form, vr_device.h) with (float)log((double)x) for
 * every positive finite float (synchronous, a few seconds).  counts[0] =
 * mismatches of either (must be 0), counts[1] = inputs either form left to the
 * double-log fallback (summed). */
int vr_selftest_logf(uint64_t counts[2]);

/* Measured read ceiling of this device (bench.py reports the
 * march's traffic against it beside the 8 TB/s peak): the resident record
 * volume (all B * 4 bytes of every record, pitches included, rounded down to
 * 16 B) is streamed once untimed and then reps times by a coalesced 16-B-per-
 * lane read kernel on the library's stream.  ms[0] = fastest pass, ms[1] =
 * mean; *bytes (optional) = bytes per pass.  Synchronous. */
int vr_stream_read(int reps, float ms[2], uint64_t *bytes);

/* ---- the reference's input files ---- */

/* Parse a codebook file (loadCodebook's format, C:558-642): int nSteps,
 * int nBlocks, per block int spanId, int templateId, int shift, 1-byte flip,
 * int NE, NE int bin ids, NE double errors.  Writes min(nBlocks, max_blocks)
 * entries: codebook 4 x int32 per block, errors nbins (bin, value) float pairs
 * per block (unused pairs 0).  Either output may be NULL.  Returns nBlocks,
 * -1 if unreadable/truncated, -2 if a block has NE > nbins. */
long long vr_parse_codebook(const char *path, int nbins, long long max_blocks, int32_t *codebook,
                            float *errors);

/* Parse a templates file (loadTemplates' format, C:645-675): int nTemplates,
 * per template 6 doubles (ignored) + nbins doubles.  Writes
 * min(nTemplates, max_templates) x nbins floats (may be NULL).  Returns
 * nTemplates or -1. */
long long vr_parse_templates(const char *path, int nbins, long long max_templates,
                             float *templates);

/* Load the reference's input files and make them resident, as its main()
 * does (C:1156-1203): the raw fp32 histogram volume (nBlocks x nbins), and
 * optionally the codebook + templates files for methods 4/5/6.
 * histogram_path may be NULL; codebook/templates both NULL or both given. */
int vr_load_reference_files(const char *histogram_path, const char *codebook_path,
                            const char *templates_path, vr_extent dims, int nbins);

/* Flexible-block input files (methods 8/9/0), the formats of loadSpanList,
 * loadFractalHistogram, loadSimpleHistogram and loadFlexibleTemplates
 * (C:709-997; layouts in vr_io.cpp).  Each parser writes min(count, max)
 * entries (outputs may be NULL) and returns the file's entry count, -1 if
 * unreadable or truncated, -2 if an entry is rejected the way the reference's
 * loader rejects it, -3 (fractal) if a spanId lies past the span list.
 *   span list: low/high int4 (x, y, z, 0);
 *   fractal spans: low/high = the span list's entry spanId, code int4
 *     (template id, shift, flip, NE), errors nbins (bin, value) float pairs;
 *   simple spans: low/high int4, count, hist nbins (bin, freq) float pairs. */
long long vr_parse_span_list(const char *path, long long max, int32_t *low, int32_t *high);
long long vr_parse_fractal_histogram(const char *path, const int32_t *span_low,
                                     const int32_t *span_high, long long nspans, int nbins,
                                     long long max, int32_t *low, int32_t *high, int32_t *code,
                                     float *errors);
long long vr_parse_simple_histogram(const char *count_path, const char *binid_path,
                                    const char *binfreq_path, int nbins, long long max,
                                    int32_t *low, int32_t *high, int32_t *count, float *hist);

/* Parse all six flexible-block files (flexible templates in the templates
 * format, values in [0, 1]) and make the span tables resident (vr_init_flex)
 * for a dim^3 raw volume, as main() does (C:1170-1203). */
int vr_load_flex_files(const char *span_list_path, const char *fractal_path,
                       const char *simple_count_path, const char *simple_binid_path,
                       const char *simple_binfreq_path, const char *templates_path, int dim,
                       int nbins);

/* ---- GMM distribution volumes (BASELINE config 5) ----
 * An extension: the reference holds histograms only.  Each voxel is a K-component
 * Gaussian mixture in two planes:
 *   wm     (w_k, mu_k) float pairs, [voxel][K][2]  (8K bytes per voxel)
 *   sigma  sigma_k floats,          [voxel][K]     (4K bytes per voxel)
 * voxel order x + X*(y + Y*(z - z_base)) over the resident slices
 * [z_base, z_base + nslices) of an X x Y x Z volume (dims).  K: 8, 16 or 32.
 * The march is the reference's (K:282-717) with the per-step statistic decoded
 * from the 8 corner mixtures: queryMethod 1 samples the mean sum w mu,
 * queryMethod 2 samples 16 x the variance sum w (sigma^2 + mu^2) - mean^2
 * (canonical evaluation order in vr_gmm.hip).  where: 0 host, 1 device (copied),
 * 2 device (adopted, not freed).  A new GMM volume replaces the previous one. */
int vr_init_gmm(const float *wm, const float *sigma, vr_extent dims, int ncomp, int z_base,
                int nslices, int where);

/* Generate slices [z_base, z_base + nslices) of the seeded synthetic GMM volume
 * of DESIGN.md 11.1 (a dims-sized volume) directly in HBM. */
int vr_synthesize_gmm(vr_extent dims, int ncomp, uint64_t seed, int z_base, int nslices);

int vr_gmm_info(vr_extent *dims, int *ncomp, int *z_base, int *nslices, const float **d_wm,
                const float **d_sigma);
int vr_free_gmm(void);
/* Two GMM volumes may be resident, in slots 0 and 1 (a rank of a two-segment
 * slab chain holds a front and a back z-range): every vr_*gmm*
 * call acts on the selected slot (0 until changed); vr_free_gmm frees only it,
 * freeCudaBuffers both. */
int vr_gmm_select(int slot);

/* Slab of a slab-chained render (out-of-core and multi-GPU sort-last, DESIGN.md
 * 11.2).  The launch takes the samples whose trilinear footprint starts in
 * slices [z_lo, z_hi) (it reads slices z_lo .. min(z_hi, Z-1), which must be
 * resident).  Rays come from the camera (d_rays_in == NULL: whole frame) or
 * from the alive list of the previous slab (n_rays_in entries of 36 bytes:
 * float sum[4], t, pos[3]; uint32 pixel | samples taken << 23; slab launches
 * need width*height <= 2^23).  Rays that end in
 * the slab are written to the frame (d_output etc., pixel y*width + x); rays that
 * leave it alive are appended to d_rays_out (capacity: n_rays_in, or
 * width*height) and counted in *d_n_rays_out (device memory; the call sets it
 * to 0 on the library's stream before its launch, so the caller reads it
 * after synchronising with that stream; entries past the capacity would be
 * dropped, never written).
 * Slabs must be rendered in the order the view's rays cross them (every ray of
 * the frame must step the same way in z, else VR_ERR_UNSUPPORTED); the chain
 * then reproduces the whole-volume render bit for bit. */
typedef struct {
    int z_lo, z_hi;
    const void *d_rays_in;
    uint32_t n_rays_in;
    void *d_rays_out;
    uint32_t *d_n_rays_out;
} vr_gmm_slab;

/* Render the resident GMM volume: slab == NULL renders the whole frame (all
 * slices must be resident); otherwise one slab of a chain.  desc: as for
 * vr_render (d_tile_list must be NULL). */
int vr_render_gmm(const vr_render_desc *desc, const vr_gmm_slab *slab);

/* U for a whole-volume GMM render: distinct voxels in the union of the
 * footprints of all samples taken (algorithmic bytes = U * 8K for the mean,
 * U * 12K for the variance).  Synchronous. */
int64_t vr_gmm_count_footprint(const vr_render_desc *desc);
/* U of one slab of a chain (slab as for vr_render_gmm: the samples whose
 * footprint starts in the slab, from its camera rays or its alive list in).
 * The counting launch also writes the slab's alive list out (as a render
 * would) but no pixels.  Synchronous. */
int64_t vr_gmm_count_footprint_slab(const vr_render_desc *desc, const vr_gmm_slab *slab);

/* library version string */
const char *vr_version(void);

#ifdef __cplusplus
}
#endif
#endif /* VR_H */
