// vr_single_test -- headless verify/bench run mirroring the reference's
// runSingleTest (C:1016-1084) on top of libvr.so.
//
// Loads the reference's input files (or generates the synthetic volume), sets
// the runSingleTest camera (eye at z = 4, C:1024-1043), renders 1 + iters
// frames through the reference entry points, prints the reference's
// throughput line, writes the frame as a binary PPM and, with --ref, compares
// it like sdkComparePPM(MAX_EPSILON_ERROR = 5, THRESHOLD = 0.30) (C:57-58,
// 1077): a byte differs when |ref - out| > 5; the test passes when fewer than
// 30 % of the bytes differ.  Exit status 0 on pass, 1 on failure.
//
//   vr_single_test [--file=hist.bin] [--codebook=cb.bin --templates=tpl.bin]
//                  [--synthetic] [--xsize=50 --ysize=50 --zsize=10] [--bins=32]
//                  [--method=1] [--width=512 --height=512] [--iters=10]
//                  [--density=0.05] [--brightness=1] [--offset=0] [--scale=1]
//                  [--out=volume.ppm] [--ref=ref_volume.ppm]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/vr.h"

namespace {

const char *arg(int argc, char **argv, const char *name) {
    const size_t n = std::strlen(name);
    for (int i = 1; i < argc; i++)
        if (std::strncmp(argv[i], "--", 2) == 0 && std::strncmp(argv[i] + 2, name, n) == 0) {
            const char *v = argv[i] + 2 + n;
            if (*v == '=') return v + 1;
            if (*v == 0) return "";
        }
    return nullptr;
}

long iarg(int argc, char **argv, const char *name, long def) {
    const char *v = arg(argc, argv, name);
    return v && *v ? std::strtol(v, nullptr, 10) : def;
}

float farg(int argc, char **argv, const char *name, float def) {
    const char *v = arg(argc, argv, name);
    return v && *v ? std::strtof(v, nullptr) : def;
}

bool check(const char *what) {
    if (vr_last_status() == VR_OK) return true;
    std::fprintf(stderr, "%s: %s\n", what, vr_last_error());
    return false;
}

// sdkSavePPM4ub: RGBA8 -> binary RGB PPM
bool save_ppm(const char *path, const std::vector<uint32_t> &px, int w, int h) {
    FILE *f = std::fopen(path, "wb");
    if (!f) return false;
    std::fprintf(f, "P6\n%d %d\n255\n", w, h);
    std::vector<unsigned char> rgb((size_t)w * h * 3);
    for (size_t i = 0; i < (size_t)w * h; i++) {
        rgb[3 * i] = (unsigned char)(px[i] & 0xFF);
        rgb[3 * i + 1] = (unsigned char)((px[i] >> 8) & 0xFF);
        rgb[3 * i + 2] = (unsigned char)((px[i] >> 16) & 0xFF);
    }
    const bool ok = std::fwrite(rgb.data(), 1, rgb.size(), f) == rgb.size();
    std::fclose(f);
    return ok;
}

bool load_ppm(const char *path, std::vector<unsigned char> &rgb, int &w, int &h) {
    FILE *f = std::fopen(path, "rb");
    if (!f) return false;
    char magic[3] = {0};
    int maxv = 0;
    bool ok = std::fscanf(f, "%2s %d %d %d", magic, &w, &h, &maxv) == 4 &&
              std::strcmp(magic, "P6") == 0 && maxv == 255 && w > 0 && h > 0;
    if (ok) {
        std::fgetc(f);  // the single whitespace after the header
        rgb.resize((size_t)w * h * 3);
        ok = std::fread(rgb.data(), 1, rgb.size(), f) == rgb.size();
    }
    std::fclose(f);
    return ok;
}

}  // namespace

int main(int argc, char **argv) {
    const vr_extent dims = {(size_t)iarg(argc, argv, "xsize", 50), (size_t)iarg(argc, argv, "ysize", 50),
                            (size_t)iarg(argc, argv, "zsize", 10)};
    const int bins = (int)iarg(argc, argv, "bins", 32);
    const int method = (int)iarg(argc, argv, "method", 1);
    const uint32_t width = (uint32_t)iarg(argc, argv, "width", 512);
    const uint32_t height = (uint32_t)iarg(argc, argv, "height", 512);
    const int iters = (int)iarg(argc, argv, "iters", 10);
    const float density = farg(argc, argv, "density", 0.05f);
    const float brightness = farg(argc, argv, "brightness", 1.0f);
    const float offset = farg(argc, argv, "offset", 0.0f);
    const float scale = farg(argc, argv, "scale", 1.0f);
    const char *out_path = arg(argc, argv, "out");
    if (!out_path || !*out_path) out_path = "volume.ppm";
    const char *ref = arg(argc, argv, "ref");

    if (arg(argc, argv, "synthetic")) {
        vr_synthesize(dims, bins, 20261015ull);
        if (!check("vr_synthesize")) return 1;
        if (method >= 4 && method <= 6) {
            vr_synthesize_codec(dims, bins, 64, bins < 4 ? bins : 4, 20261015ull);
            if (!check("vr_synthesize_codec")) return 1;
        }
    } else {
        vr_load_reference_files(arg(argc, argv, "file"), arg(argc, argv, "codebook"),
                                arg(argc, argv, "templates"), dims, bins);
        if (!check("loading the input files")) return 1;
    }
    basicDataProcessing();
    if (!check("basicDataProcessing")) return 1;

    uint32_t *d_output = nullptr;
    if (hipMalloc(&d_output, (size_t)width * height * 4) != hipSuccess ||
        hipMemset(d_output, 0, (size_t)width * height * 4) != hipSuccess) {
        std::fprintf(stderr, "device allocation failed\n");
        return 1;
    }
    // runSingleTest's modelView (C:1024-1043), transposed into 3 rows
    float inv_view[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 4};
    copyInvViewMatrix(inv_view, sizeof inv_view);
    const vr_dim3 block = {16, 16, 1};
    const vr_dim3 grid = {(width + 15) / 16, (height + 15) / 16, 1};
    auto t0 = std::chrono::steady_clock::now();
    for (int i = -1; i < iters; i++) {
        if (i == 0) {
            (void)hipDeviceSynchronize();
            t0 = std::chrono::steady_clock::now();
        }
        render_kernel(grid, block, d_output, width, height, density, brightness, offset, scale,
                      method, dims);
    }
    (void)hipDeviceSynchronize();
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() /
                     (iters > 0 ? iters : 1);
    if (!check("render_kernel")) return 1;
    std::printf("volumeRender, Throughput = %.4f MTexels/s, Time = %.5f s, Size = %u Texels, "
                "NumDevsUsed = %u, Workgroup = %u\n",
                1.0e-6 * width * height / t, t, width * height, 1u, block.x * block.y);

    std::vector<uint32_t> px((size_t)width * height);
    (void)hipMemcpy(px.data(), d_output, px.size() * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d_output);
    freeCudaBuffers();
    if (!save_ppm(out_path, px, (int)width, (int)height)) {
        std::fprintf(stderr, "cannot write %s\n", out_path);
        return 1;
    }
    if (!ref) return 0;
    std::vector<unsigned char> a, b;
    int wa = 0, ha = 0, wb = 0, hb = 0;
    if (!load_ppm(out_path, a, wa, ha) || !load_ppm(ref, b, wb, hb) || wa != wb || ha != hb) {
        std::fprintf(stderr, "cannot compare %s with %s\n", out_path, ref);
        return 1;
    }
    // sdkComparePPM compares the 4-channel images (alpha 0 in both)
    const size_t len = (size_t)wa * ha * 4;
    size_t bad = 0;
    for (size_t i = 0; i < a.size(); i++) {
        const float d = (float)b[i] - (float)a[i];
        bad += !(d <= 5.0f && d >= -5.0f);
    }
    if (bad) std::printf("%4.2f(%%) of bytes mismatched (count=%zu)\n", bad * 100.0 / len, bad);
    const bool pass = (double)len * 0.30 > (double)bad;
    std::printf("%s\n", pass ? "PASSED" : "FAILED");
    return pass ? 0 : 1;
}
