// vr_io.cpp -- readers for the reference's on-disk inputs
// and the one-call loader that makes them resident, so the reference's own
// files go through this library unchanged.  Host code only.
//
//   histogram volume  raw fp32, nBlocks x nBins records (loadRawFile, C:538-555)
//   codebook          int nSteps, int nBlocks, then per block: int spanId,
//                     int templateId, int shift, bool flip (1 byte), int NE,
//                     NE x int binId, NE x double error (loadCodebook, C:558-642)
//   templates         int nTemplates, then per template 6 doubles (ignored) and
//                     nBins doubles (loadTemplates, C:645-675)
// Flexible blocks (methods 8/9/0):
//   span list         int nSpan, per span int lowX, highX, lowY, highY, lowZ,
//                     highZ (loadSpanList, C:709-771)
//   fractal spans     int nTimeSteps, int nHistogram, per entry int spanId,
//                     int templateId, int shift, bool flip (1 byte), int NE,
//                     NE x int binId, NE x double error (loadFractalHistogram,
//                     C:773-875)
//   simple spans      counts file: int nHistogram, per entry 6 ints (low x, y,
//                     z, high x, y, z) and int count; bin-id file: the counts'
//                     ints back to back; frequency file: doubles likewise
//                     (loadSimpleHistogram, C:877-949)
//   flexible templates  as templates, every value in [0, 1] (C:951-997)
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/vr.h"
#include "vr_internal.h"

namespace {

struct File {
    FILE *f = nullptr;
    explicit File(const char *path) : f(path ? std::fopen(path, "rb") : nullptr) {}
    ~File() {
        if (f) std::fclose(f);
    }
    template <class T>
    bool get(T *dst, size_t n) {
        return n == 0 || std::fread(dst, sizeof(T), n, f) == n;
    }
};

}  // namespace

extern "C" {

// Parses a codebook file.  Writes min(nBlocks, max_blocks) entries: codebook
// as 4 int32 (template id, shift, flip, NE) and errors as nbins (bin, value)
// float pairs per block (unused pairs zero), as loadCodebook fills its arrays.
// Returns nBlocks, or -1 (unreadable / truncated), -2 (NE > nbins: the
// reference's loader rejects the file, C:611-614).
long long vr_parse_codebook(const char *path, int nbins, long long max_blocks, int32_t *codebook,
                            float *errors) {
    File in(path);
    if (!in.f || nbins <= 0) return -1;
    int nsteps = 0, nblocks = 0;
    if (!in.get(&nsteps, 1) || !in.get(&nblocks, 1) || nblocks < 0) return -1;
    std::vector<int> bins(nbins);
    std::vector<double> vals(nbins);
    for (long long i = 0; i < nblocks; i++) {
        int span = 0, tid = 0, shift = 0, ne = 0;
        unsigned char flip = 0;
        if (!in.get(&span, 1) || !in.get(&tid, 1) || !in.get(&shift, 1) || !in.get(&flip, 1) ||
            !in.get(&ne, 1))
            return -1;
        if (ne > nbins || ne < 0) return -2;
        if (!in.get(bins.data(), (size_t)ne) || !in.get(vals.data(), (size_t)ne)) return -1;
        if (i >= max_blocks) continue;
        if (codebook) {
            int32_t *c = codebook + 4 * i;
            c[0] = tid;
            c[1] = shift;
            c[2] = flip ? 1 : 0;
            c[3] = ne;
        }
        if (errors) {
            float *e = errors + 2 * (size_t)i * (size_t)nbins;
            std::memset(e, 0, sizeof(float) * 2 * (size_t)nbins);
            for (int j = 0; j < ne; j++) {
                e[2 * j] = (float)bins[j];
                e[2 * j + 1] = (float)vals[j];
            }
        }
    }
    return nblocks;
}

// Parses a templates file into min(nTemplates, max_templates) x nbins floats.
// Returns nTemplates or -1.
long long vr_parse_templates(const char *path, int nbins, long long max_templates,
                             float *templates) {
    File in(path);
    if (!in.f || nbins <= 0) return -1;
    int nt = 0;
    if (!in.get(&nt, 1) || nt < 0) return -1;
    std::vector<double> limits(6), freq(nbins);
    for (long long t = 0; t < nt; t++) {
        if (!in.get(limits.data(), 6) || !in.get(freq.data(), (size_t)nbins)) return -1;
        if (t < max_templates && templates)
            for (int b = 0; b < nbins; b++) templates[(size_t)t * nbins + b] = (float)freq[b];
    }
    return nt;
}

// Span list: min(nSpan, max) spans as int4 low/high (x, y, z, 0).  Returns
// nSpan, -1 (unreadable / truncated) or -2 (a span fails checkSpanLimit, C:693-699).
long long vr_parse_span_list(const char *path, long long max, int32_t *low, int32_t *high) {
    File in(path);
    if (!in.f) return -1;
    int n = 0;
    if (!in.get(&n, 1) || n < 0) return -1;
    for (long long i = 0; i < n; i++) {
        int v[6];  // lowX, highX, lowY, highY, lowZ, highZ (C:728-733)
        if (!in.get(v, 6)) return -1;
        const int lo[3] = {v[0], v[2], v[4]}, hi[3] = {v[1], v[3], v[5]};
        for (int a = 0; a < 3; a++)
            if (lo[a] > hi[a] || lo[a] < 0 || hi[a] < 0) return -2;
        if (i >= max) continue;
        if (low) {
            int32_t *o = low + 4 * i;
            o[0] = lo[0]; o[1] = lo[1]; o[2] = lo[2]; o[3] = 0;
        }
        if (high) {
            int32_t *o = high + 4 * i;
            o[0] = hi[0]; o[1] = hi[1]; o[2] = hi[2]; o[3] = 0;
        }
    }
    return n;
}

// Fractal-coded spans: entry i gets the span of its spanId from the span list
// (codebookSpanLow/High[i] = spanLow/High[spanId], C:833-834), its code
// (template id, shift, flip, NE) and nbins (bin id, error) pairs (unused zero).
// Returns nHistogram, -1 (unreadable / truncated), -2 (rejected as the
// reference's loader rejects: spanId outside [0, 2 nHistogram], template id < 0,
// NE outside [0, nbins], C:800-825) or -3 (spanId past the span list).
long long vr_parse_fractal_histogram(const char *path, const int32_t *span_low,
                                     const int32_t *span_high, long long nspans, int nbins,
                                     long long max, int32_t *low, int32_t *high, int32_t *code,
                                     float *errors) {
    File in(path);
    if (!in.f || nbins <= 0) return -1;
    int nsteps = 0, n = 0;
    if (!in.get(&nsteps, 1) || !in.get(&n, 1) || n < 0) return -1;
    std::vector<int> bins(nbins);
    std::vector<double> vals(nbins);
    for (long long i = 0; i < n; i++) {
        int span = 0, tid = 0, shift = 0, ne = 0;
        unsigned char flip = 0;
        if (!in.get(&span, 1) || !in.get(&tid, 1) || !in.get(&shift, 1) || !in.get(&flip, 1) ||
            !in.get(&ne, 1))
            return -1;
        if (span < 0 || span > 2 * (long long)n || tid < 0 || ne < 0 || ne > nbins) return -2;
        if (span >= nspans) return -3;
        if (!in.get(bins.data(), (size_t)ne) || !in.get(vals.data(), (size_t)ne)) return -1;
        if (i >= max) continue;
        if (low) std::memcpy(low + 4 * i, span_low + 4 * (size_t)span, 16);
        if (high) std::memcpy(high + 4 * i, span_high + 4 * (size_t)span, 16);
        if (code) {
            int32_t *c = code + 4 * i;
            c[0] = tid; c[1] = shift; c[2] = flip ? 1 : 0; c[3] = ne;
        }
        if (errors) {
            float *e = errors + 2 * (size_t)i * (size_t)nbins;
            std::memset(e, 0, sizeof(float) * 2 * (size_t)nbins);
            for (int j = 0; j < ne; j++) {
                e[2 * j] = (float)bins[j];
                e[2 * j + 1] = (float)vals[j];
            }
        }
    }
    return n;
}

// Simple spans from the three files.  Returns nHistogram, -1 (unreadable /
// truncated) or -2 (rejected like C:906-937: low span negative, count < 0 or
// > nbins, a bin id or frequency outside [0, nbins] x [0, 1]).
long long vr_parse_simple_histogram(const char *count_path, const char *binid_path,
                                    const char *binfreq_path, int nbins, long long max,
                                    int32_t *low, int32_t *high, int32_t *count, float *hist) {
    File fc(count_path), fi(binid_path), ff(binfreq_path);
    if (!fc.f || !fi.f || !ff.f || nbins <= 0) return -1;
    int n = 0;
    if (!fc.get(&n, 1) || n < 0) return -1;
    std::vector<int> bins(nbins);
    std::vector<double> freq(nbins);
    for (long long i = 0; i < n; i++) {
        int v[6], c = 0;
        if (!fc.get(v, 6) || !fc.get(&c, 1)) return -1;
        // checkSpanLimit(simpleLow, simpleLow) (sic, C:916): only the low corner's sign
        if (v[0] < 0 || v[1] < 0 || v[2] < 0) return -2;
        if (c < 0 || c > nbins) return -2;
        if (!fi.get(bins.data(), (size_t)c) || !ff.get(freq.data(), (size_t)c)) return -1;
        for (int j = 0; j < c; j++)
            if (bins[j] < 0 || freq[j] < 0 || bins[j] > nbins || freq[j] > 1.0) return -2;
        if (i >= max) continue;
        if (low) {
            int32_t *o = low + 4 * i;
            o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; o[3] = 0;
        }
        if (high) {
            int32_t *o = high + 4 * i;
            o[0] = v[3]; o[1] = v[4]; o[2] = v[5]; o[3] = 0;
        }
        if (count) count[i] = c;
        if (hist) {
            float *h = hist + 2 * (size_t)i * (size_t)nbins;
            std::memset(h, 0, sizeof(float) * 2 * (size_t)nbins);
            for (int j = 0; j < c; j++) {
                h[2 * j] = (float)bins[j];
                h[2 * j + 1] = (float)freq[j];
            }
        }
    }
    return n;
}

// Loads the flexible-block files and makes the span tables resident
// (vr_init_flex), as main() does with loadSpanList, loadFractalHistogram,
// loadSimpleHistogram, loadFlexibleTemplates and initCuda (C:1170-1203);
// then dataProcessing / vr_flex_process computes the block statistics.
int vr_load_flex_files(const char *span_list_path, const char *fractal_path,
                       const char *simple_count_path, const char *simple_binid_path,
                       const char *simple_binfreq_path, const char *templates_path, int dim,
                       int nbins) {
    using vr::record_error;
    if (nbins <= 0) return record_error(VR_ERR_ARG, "vr_load_flex_files: bad nbins");
    const long long nsp = vr_parse_span_list(span_list_path, 0, nullptr, nullptr);
    if (nsp < 0)
        return record_error(VR_ERR_ARG, nsp == -2 ? "span list: a span fails checkSpanLimit"
                                                  : "span list unreadable or truncated");
    std::vector<int32_t> sl(4 * (size_t)nsp), sh(4 * (size_t)nsp);
    vr_parse_span_list(span_list_path, nsp, sl.data(), sh.data());
    const long long nf = vr_parse_fractal_histogram(fractal_path, sl.data(), sh.data(), nsp,
                                                    nbins, 0, nullptr, nullptr, nullptr, nullptr);
    if (nf < 0)
        return record_error(VR_ERR_ARG, nf == -2 ? "fractal spans: entry rejected (C:800-825)"
                                        : nf == -3 ? "fractal spans: spanId past the span list"
                                                   : "fractal span file unreadable or truncated");
    std::vector<int32_t> fl(4 * (size_t)nf), fh(4 * (size_t)nf), fc(4 * (size_t)nf);
    std::vector<float> fe(2 * (size_t)nf * nbins);
    vr_parse_fractal_histogram(fractal_path, sl.data(), sh.data(), nsp, nbins, nf, fl.data(),
                               fh.data(), fc.data(), fe.data());
    const long long ns = vr_parse_simple_histogram(simple_count_path, simple_binid_path,
                                                   simple_binfreq_path, nbins, 0, nullptr,
                                                   nullptr, nullptr, nullptr);
    if (ns < 0)
        return record_error(VR_ERR_ARG, ns == -2 ? "simple spans: entry rejected (C:906-937)"
                                                 : "simple span files unreadable or truncated");
    std::vector<int32_t> ql(4 * (size_t)ns), qh(4 * (size_t)ns), qc((size_t)ns);
    std::vector<float> qe(2 * (size_t)ns * nbins);
    vr_parse_simple_histogram(simple_count_path, simple_binid_path, simple_binfreq_path, nbins,
                              ns, ql.data(), qh.data(), qc.data(), qe.data());
    const long long nt = vr_parse_templates(templates_path, nbins, 0, nullptr);
    if (nt <= 0) return record_error(VR_ERR_ARG, "flexible templates unreadable or empty");
    std::vector<float> tpl((size_t)nt * nbins);
    vr_parse_templates(templates_path, nbins, nt, tpl.data());
    for (float v : tpl)  // C:985-990
        if (!(v >= 0.0f && v <= 1.0f))
            return record_error(VR_ERR_ARG, "flexible templates: a frequency outside [0, 1]");
    vr_flex_tables t;
    t.dim = dim;
    t.nbins = nbins;
    t.n_fractal = (int)nf;
    t.fractal_low = reinterpret_cast<const vr_int4 *>(fl.data());
    t.fractal_high = reinterpret_cast<const vr_int4 *>(fh.data());
    t.fractal_code = reinterpret_cast<const vr_int4 *>(fc.data());
    t.fractal_errors = reinterpret_cast<const vr_float2 *>(fe.data());
    t.n_simple = (int)ns;
    t.simple_low = reinterpret_cast<const vr_int4 *>(ql.data());
    t.simple_high = reinterpret_cast<const vr_int4 *>(qh.data());
    t.simple_count = qc.data();
    t.simple_hist = reinterpret_cast<const vr_float2 *>(qe.data());
    t.templates = tpl.data();
    t.ntemplates = (int)nt;
    return vr_init_flex(&t);
}

// Loads the reference's input files and makes them resident, as main() does
// with loadRawFile / loadCodebook / loadTemplates and initCuda (C:1156-1203).
// histogram_path may be NULL (codec only); codebook_path and templates_path
// may both be NULL (histograms only).  dims = volume size in voxels (blocks).
int vr_load_reference_files(const char *histogram_path, const char *codebook_path,
                            const char *templates_path, vr_extent dims, int nbins) {
    using vr::record_error;
    const size_t nvox = dims.width * dims.height * dims.depth;
    if (nvox == 0 || nbins <= 0) return record_error(VR_ERR_ARG, "vr_load_reference_files: bad sizes");
    if (histogram_path) {
        std::vector<float> h(nvox * (size_t)nbins);
        File in(histogram_path);
        if (!in.f || !in.get(h.data(), h.size()))
            return record_error(VR_ERR_ARG, "histogram file missing or shorter than nBlocks x nBins floats");
        int rc = vr_init_distribution(h.data(), dims, nbins, 0);
        if (rc != VR_OK) return rc;
    }
    if (codebook_path || templates_path) {
        if (!codebook_path || !templates_path)
            return record_error(VR_ERR_ARG, "the codec needs both a codebook and a templates file");
        const long long nt = vr_parse_templates(templates_path, nbins, 0, nullptr);
        if (nt <= 0) return record_error(VR_ERR_ARG, "templates file unreadable or empty");
        std::vector<float> tpl((size_t)nt * nbins);
        vr_parse_templates(templates_path, nbins, nt, tpl.data());
        std::vector<int32_t> cb(4 * nvox);
        std::vector<float> err(2 * nvox * (size_t)nbins);
        const long long nb = vr_parse_codebook(codebook_path, nbins, (long long)nvox, cb.data(),
                                               err.data());
        if (nb == -2) return record_error(VR_ERR_ARG, "codebook: NE > nBins (rejected, C:611-614)");
        if (nb != (long long)nvox)
            return record_error(VR_ERR_ARG, "codebook unreadable or its block count != voxels");
        return vr_init_codec(reinterpret_cast<const vr_int4 *>(cb.data()), dims, tpl.data(),
                             (int)nt, reinterpret_cast<const vr_float2 *>(err.data()), nbins,
                             nbins, 0);
    }
    return VR_OK;
}

}  // extern "C"
