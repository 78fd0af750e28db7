/* footprint_sim.c -- distinct 128-B lines of the march's footprints under
 * different sharing scopes (tooling).  Rays are marched with the kernels' float
 * arithmetic for the samples-per-pixel a GPU run recorded (tools/dump_steps.py),
 * so early termination is honoured.  1024^3 x 8-bin volume (32-B records,
 * 4 per line), 1920x1080.
 *
 *   gcc -O3 -fopenmp -ffp-contract=off tools/footprint_sim.c -o tools/build/footprint_sim -lm
 *   tools/build/footprint_sim gpurun_out/steps_C0.npy C0
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifndef N
#define N 1024
#endif
#define W 1920
#define H 1080

static float M[12];
static int PF = 0;
static int ALIGN = 0; /* 1: per-step scopes count a ray's sample s at iteration s + its depth
                         offset round((tnear - tnear_min of the tile) / 0.01) */
static int RING = 0;  /* > 1: per-tile ring of the last RING steps' lines (an LDS cache of
                         recent steps): a tile-step counts only lines not in the previous
                         RING - 1 steps of the same tile */
static int LAYOUT = 0; /* 0: x-rows (4 records along x per line), 1: 2x2 (x,y) micro-bricks,
                          2: 2x1x2 (x,z) micro-bricks, 3: 1x2x2 (y,z) micro-bricks */

/* LAYOUT=10: baked statistics planes, 4-B voxels, 32 per line, bricks of
   BX x BY x BZ voxels (BX*BY*BZ = 32; default 32x1x1 = x-rows) */
static uint32_t BX = 32, BY = 1, BZ = 1;
static uint32_t line_of(uint32_t x, uint32_t y, uint32_t z) {
    if (LAYOUT == 10)
        return (uint32_t)(((uint64_t)(z / BZ) * (N / BY) + y / BY) * (N / BX) + x / BX);
    if (LAYOUT == 1)
        return (uint32_t)(((uint64_t)z * (N / 2) + (y >> 1)) * (N / 2) + (x >> 1));
    if (LAYOUT == 2)
        return (uint32_t)(((uint64_t)(z >> 1) * N + y) * (N / 2) + (x >> 1));
    if (LAYOUT == 3)  /* 1x2x2 (y,z) micro-bricks: a line = 2 y x 2 z records at one x */
        return (uint32_t)(((uint64_t)(z >> 1) * (N / 2) + (y >> 1)) * N + x);
    return (uint32_t)((((uint64_t)z * N + y) * N + x) >> 2);
}

static void lin_axis(float u, int n, int *i0, int *i1) {
    u = fminf(fmaxf(u, 0.0f), 1.0f);
    float xb = u * (float)n - 0.5f;
    int i = (int)floorf(xb);
    *i0 = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
    *i1 = i + 1 < 0 ? 0 : (i + 1 > n - 1 ? n - 1 : i + 1);
}

/* the 4 line ids (one per (y,z) combo; x0/x1 records share or straddle) */
static float g_tn;  /* tnear of the last ray_lines call (per thread below) */
#pragma omp threadprivate(g_tn)
static int ray_lines(int x, int y, int nsteps, uint32_t *out /* 8 per step */) {
    float u = ((float)x / (float)W) * 2.0f - 1.0f, v = ((float)y / (float)H) * 2.0f - 1.0f;
    float ox = M[3], oy = M[7], oz = M[11];
    float inv = 1.0f / sqrtf(u * u + v * v + 4.0f);
    float ax = u * inv, ay = v * inv, az = -2.0f * inv;
    float dx = ax * M[0] + ay * M[1] + az * M[2];
    float dy = ax * M[4] + ay * M[5] + az * M[6];
    float dz = ax * M[8] + ay * M[9] + az * M[10];
    float ix = 1.0f / dx, iy = 1.0f / dy, iz = 1.0f / dz;
    float bx = ix * (-1.0f - ox), by = iy * (-1.0f - oy), bz = iz * (-1.0f - oz);
    float tx = ix * (1.0f - ox), ty = iy * (1.0f - oy), tz = iz * (1.0f - oz);
    float tn = fmaxf(fmaxf(fminf(tx, bx), fminf(ty, by)), fmaxf(fminf(tx, bx), fminf(tz, bz)));
    float tf = fminf(fminf(fmaxf(tx, bx), fmaxf(ty, by)), fminf(fmaxf(tx, bx), fmaxf(tz, bz)));
    if (tn < 0) tn = 0;
    g_tn = tn;
    /* PF=1: also the step the pipelined kernels prefetch after an early exit */
    if (PF && nsteps < 500) {
        float t = tn;
        for (int i = 0; i < nsteps - 1; i++) t += 0.01f;
        if (!(t + 0.01f > tf)) nsteps++;
    }
    float px = ox + dx * tn, py = oy + dy * tn, pz = oz + dz * tn;
    float sx = dx * 0.01f, sy = dy * 0.01f, sz = dz * 0.01f;
    int k = 0;
    for (int i = 0; i < nsteps; i++) {
        int x0, x1, y0, y1, z0, z1;
        lin_axis(px * 0.5f + 0.5f, N, &x0, &x1);
        lin_axis(py * 0.5f + 0.5f, N, &y0, &y1);
        lin_axis(pz * 0.5f + 0.5f, N, &z0, &z1);
        int ys[2] = {y0, y1}, zs[2] = {z0, z1};
        if (LAYOUT == 11 || LAYOUT == 12) {
            /* baked planes as gather8 reads them, 4-B voxels, 32 per line.
               11: y-pair rows -- element (x, y0, z) holds (v[z][y0][x], v[z][y0+1][x]),
                   16 x per line, runs of 15 x + one apron voxel: a footprint is
                   two 16-B loads (z0, z1), one line each.
               12: 8x2x2 bricks, runs of 7 x + apron (k_plane8): four 8-B loads. */
            for (int c = 0; c < 4; c++) {
                uint32_t l;
                if (LAYOUT == 11)
                    l = (uint32_t)(((uint64_t)zs[c >> 1] * N + y0) * (N / 15 + 1) + x0 / 15);
                else
                    l = (uint32_t)(((uint64_t)(zs[c >> 1] >> 1) * (N / 2) + (ys[c & 1] >> 1)) *
                                   (N / 7 + 1) + x0 / 7);
                out[k++] = l;
                out[k++] = l;
            }
            px += sx; py += sy; pz += sz;
            continue;
        }
        for (int c = 0; c < 4; c++) {
            out[k++] = line_of(x0, ys[c & 1], zs[c >> 1]);
            out[k++] = line_of(x1, ys[c & 1], zs[c >> 1]);
        }
        px += sx; py += sy; pz += sz;
    }
    return k;
}

static int cmp_u32(const void *a, const void *b) {
    uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return x < y ? -1 : x > y;
}

static uint64_t uniq(uint32_t *v, size_t n) {
    if (!n) return 0;
    qsort(v, n, 4, cmp_u32);
    uint64_t u = 1;
    for (size_t i = 1; i < n; i++) u += v[i] != v[i - 1];
    return u;
}

int main(int argc, char **argv) {
    if (argc < 3) return 1;
    const float c0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 4};
    const float c1[12] = {0.70710677f, 0.0f, -0.70710677f, -2.828427f, 0.35355338f, 0.8660254f,
                          0.35355338f, 1.4142135f, 0.61237246f, -0.5f, 0.61237246f, 2.4494898f};
    memcpy(M, strcmp(argv[2], "C0") == 0 ? c0 : c1, sizeof M);
    if (getenv("LAYOUT")) LAYOUT = atoi(getenv("LAYOUT"));
    if (getenv("PF")) PF = atoi(getenv("PF"));
    if (getenv("ALIGN")) ALIGN = atoi(getenv("ALIGN"));
    if (getenv("BRICK") && sscanf(getenv("BRICK"), "%ux%ux%u", &BX, &BY, &BZ) == 3 &&
        BX * BY * BZ != 32)
        return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 1;
    int32_t *steps = malloc(sizeof(int32_t) * W * H);
    fseek(f, 128, SEEK_SET); /* npy v1 header of this shape is 128 bytes */
    if (fread(steps, 4, W * H, f) != W * H) return 1;
    fclose(f);
    const size_t nlines = (size_t)N * N * N * 32 / 128 * ((LAYOUT == 11 || LAYOUT == 12) ? 2 : 1);
    uint8_t *bits = calloc(nlines / 8 + 1, 1);
    uint64_t samples = 0, per_tile = 0, per_wave_step = 0, per_tile_step = 0, per_wave = 0;
    uint64_t per_ring = 0, max_ring = 0, max_tile_step = 0;
    if (getenv("RING")) RING = atoi(getenv("RING"));
    uint64_t per_block4 = 0;
    const int TX = 120, TY = 68;
#pragma omp parallel for schedule(dynamic) reduction(+ : samples, per_tile, per_wave_step, per_tile_step, per_wave, per_ring) reduction(max : max_ring, max_tile_step)
    for (int t = 0; t < (argc >= 5 ? 0 : TX * TY); t++) {
        int tx = t % TX, ty = t / TX;
        uint32_t *buf = malloc(sizeof(uint32_t) * 256 * 500 * 8);
        uint32_t *tmp = malloc(sizeof(uint32_t) * 256 * 8);
        int lens[256], off[256];
        float tns[256];
        uint32_t *rl[256];
        size_t tot = 0;
        for (int i = 0; i < 256; i++) {
            int x = tx * 16 + (i & 15), y = ty * 16 + (i >> 4);
            lens[i] = 0;
            rl[i] = buf + tot;
            if (x >= W || y >= H) continue;
            int n = steps[(size_t)y * W + x];
            if (n <= 0) continue;
            lens[i] = ray_lines(x, y, n, rl[i]);
            tns[i] = g_tn;
            tot += lens[i];
            samples += n;
        }
        {
            float tmin = 1e30f;
            for (int i = 0; i < 256; i++) if (lens[i] && tns[i] < tmin) tmin = tns[i];
            for (int i = 0; i < 256; i++)
                off[i] = (ALIGN && lens[i]) ? (int)lrintf((tns[i] - tmin) / 0.01f) : 0;
        }
        for (size_t k = 0; k < tot; k++) {
            uint32_t l = buf[k];
#pragma omp atomic
            bits[l >> 3] |= (uint8_t)(1u << (l & 7));
        }
        /* per wave (16x4 rows) per step, and per tile per step */
        int maxs = 0;
        for (int i = 0; i < 256; i++) if (lens[i] / 8 + off[i] > maxs) maxs = lens[i] / 8 + off[i];
        for (int k = 0; k < maxs; k++) {
            size_t nt = 0;
            for (int w = 0; w < 4; w++) {
                size_t nw = 0;
                for (int i = w * 64; i < w * 64 + 64; i++) {
                    const int s = k - off[i];
                    if (s >= 0 && lens[i] / 8 > s)
                        for (int c = 0; c < 8; c++) tmp[nw++] = rl[i][s * 8 + c];
                }
                uint32_t *cp = malloc(sizeof(uint32_t) * (nw + 1));
                memcpy(cp, tmp, nw * 4);
                per_wave_step += uniq(cp, nw);
                free(cp);
            }
            for (int i = 0; i < 256; i++) {
                const int s = k - off[i];
                if (s >= 0 && lens[i] / 8 > s)
                    for (int c = 0; c < 8; c++) tmp[nt++] = rl[i][s * 8 + c];
            }
            const uint64_t u = uniq(tmp, nt);
            per_tile_step += u;
            if (u > max_tile_step) max_tile_step = u;
            if (RING > 1) {
                /* lines of steps k - RING + 1 .. k - 1 of this tile, sorted */
                size_t np = 0;
                uint32_t *prev = malloc(sizeof(uint32_t) * 256 * 8 * RING + 4);
                for (int j = k - RING + 1; j < k; j++)
                    for (int i = 0; i < 256; i++) {
                        const int s = j - off[i];
                        if (j >= 0 && s >= 0 && lens[i] / 8 > s)
                            for (int c = 0; c < 8; c++) prev[np++] = rl[i][s * 8 + c];
                    }
                qsort(prev, np, 4, cmp_u32);
                /* tmp holds step k's lines sorted (uniq sorted it): count the new ones */
                uint64_t fresh = 0, ring = 0;
                for (size_t a = 0; a < nt; a++) {
                    if (a > 0 && tmp[a] == tmp[a - 1]) continue;
                    size_t lo = 0, hi = np;
                    while (lo < hi) { size_t mid = (lo + hi) / 2; if (prev[mid] < tmp[a]) lo = mid + 1; else hi = mid; }
                    if (lo == np || prev[lo] != tmp[a]) fresh++;
                }
                for (size_t a = 0; a < np; a++) ring += (a == 0 || prev[a] != prev[a - 1]);
                per_ring += fresh;
                if (ring + fresh > max_ring) max_ring = ring + fresh;
                free(prev);
            }
        }
        for (int w = 0; w < 4; w++) {
            size_t nw = 0;
            for (int i = w * 64; i < w * 64 + 64; i++) nw += lens[i];
            uint32_t *cp = malloc(sizeof(uint32_t) * (nw + 1));
            size_t k = 0;
            for (int i = w * 64; i < w * 64 + 64; i++) { memcpy(cp + k, rl[i], lens[i] * 4); k += lens[i]; }
            per_wave += uniq(cp, nw);
            free(cp);
        }
        per_tile += uniq(buf, tot);
        free(buf);
        free(tmp);
    }
    /* per 4x4-tile block */
    if (argc >= 5) goto scope;
#pragma omp parallel for schedule(dynamic) reduction(+ : per_block4)
    for (int b = 0; b < 30 * 17; b++) {
        int bx = b % 30, by = b / 30;
        size_t cap = 16 * 256 * 500 * 8, tot = 0;
        uint32_t *buf = malloc(sizeof(uint32_t) * cap);
        for (int t = 0; t < 16; t++) {
            int tx = bx * 4 + (t & 3), ty = by * 4 + (t >> 2);
            if (tx >= TX || ty >= TY) continue;
            for (int i = 0; i < 256; i++) {
                int x = tx * 16 + (i & 15), y = ty * 16 + (i >> 4);
                if (x >= W || y >= H) continue;
                int n = steps[(size_t)y * W + x];
                if (n > 0) tot += ray_lines(x, y, n, buf + tot);
            }
        }
        per_block4 += uniq(buf, tot);
        free(buf);
    }
scope:
    /* generic scope: argv[3] x argv[4] pixels */
    if (argc >= 5) {
        const int SW = atoi(argv[3]), SH = atoi(argv[4]);
        const int nsx = (W + SW - 1) / SW, nsy = (H + SH - 1) / SH;
        uint64_t per_scope = 0;
#pragma omp parallel for schedule(dynamic) reduction(+ : per_scope)
        for (int b = 0; b < nsx * nsy; b++) {
            int sx0 = (b % nsx) * SW, sy0 = (b / nsx) * SH;
            size_t tot = 0, cap = (size_t)SW * SH * 500 * 8;
            uint32_t *buf = malloc(sizeof(uint32_t) * cap);
            for (int y = sy0; y < sy0 + SH && y < H; y++)
                for (int x = sx0; x < sx0 + SW && x < W; x++) {
                    int n = steps[(size_t)y * W + x];
                    if (n > 0) tot += ray_lines(x, y, n, buf + tot);
                }
            per_scope += uniq(buf, tot);
            free(buf);
        }
        printf("  sum per %dx%d scope %12llu  (%.3f GB)\n", SW, SH, (unsigned long long)per_scope,
               per_scope * 128e-9);
        return 0;
    }
    uint64_t global = 0;
    for (size_t i = 0; i < nlines / 8 + 1; i++) global += __builtin_popcount(bits[i]);
    printf("%s samples %llu\n", argv[2], (unsigned long long)samples);
    printf("  global unique lines     %12llu  (%.3f GB)\n", (unsigned long long)global, global * 128e-9);
    printf("  sum per 4x4-tile block  %12llu  (%.3f GB)\n", (unsigned long long)per_block4, per_block4 * 128e-9);
    printf("  sum per tile            %12llu  (%.3f GB)\n", (unsigned long long)per_tile, per_tile * 128e-9);
    printf("  sum per wave            %12llu  (%.3f GB)\n", (unsigned long long)per_wave, per_wave * 128e-9);
    printf("  sum per tile-step       %12llu  (%.3f GB)\n", (unsigned long long)per_tile_step, per_tile_step * 128e-9);
    printf("  sum per wave-step       %12llu  (%.3f GB)\n", (unsigned long long)per_wave_step, per_wave_step * 128e-9);
    printf("  max lines per tile-step %12llu\n", (unsigned long long)max_tile_step);
    if (RING > 1)
        printf("  sum per tile-step ring%d %12llu  (%.3f GB), max ring lines %llu\n", RING,
               (unsigned long long)per_ring, per_ring * 128e-9, (unsigned long long)max_ring);
    return 0;
}
