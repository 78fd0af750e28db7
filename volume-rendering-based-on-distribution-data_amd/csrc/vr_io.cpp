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
