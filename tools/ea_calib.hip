// ea_calib.hip -- calibrate TCC_EA0_RDREQ / FETCH_SIZE against known byte counts
// for the march's own access shapes (tooling; MI355X_MICROARCH.md: "other access
// widths are uncalibrated").  4 GiB buffer (>> 256 MiB MALL), every 128-B line
// visited at most once per pattern in a scrambled order.  Run under
// rocprofv3 --pmc; prints lines touched and bytes requested per pattern.
//   0 stream   : contiguous float4 per lane (1 KiB / wave-instr)
//   1 lo64     : each 4-lane group reads the low 64 B of a scrambled line
//   2 lo64+hi64: same, then the high 64 B of the same line (next instruction)
//   3 line128  : each 8-lane group reads a full scrambled 128-B line
//   4 rec32    : each lane pair reads one 32-B record at a scrambled line (low 32 B)
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr uint64_t kBytes = 4ull << 30;
constexpr uint64_t kLines = kBytes / 128;

__device__ __forceinline__ uint64_t scramble(uint64_t i) {
    // bijection on [0, kLines): odd multiplier mod 2^25 (kLines = 2^25)
    return (i * 0x9E3779B1ull + 0x7F4A7C15ull) & (kLines - 1);
}

template <int PAT>
__global__ __launch_bounds__(256) void k_cal(const float4 *__restrict__ buf, uint64_t nunits,
                                             float *out) {
    const uint64_t lane = threadIdx.x & 63;
    const uint64_t wave = (blockIdx.x * 256ull + threadIdx.x) >> 6;
    const uint64_t nwaves = (gridDim.x * 256ull) >> 6;
    float acc = 0.f;
    for (uint64_t w = wave; w < nunits; w += nwaves) {
        float4 v = make_float4(0, 0, 0, 0), v2 = v;
        if constexpr (PAT == 0) {
            v = buf[w * 64 + lane];
        } else if constexpr (PAT == 1 || PAT == 2) {
            const uint64_t line = scramble(w * 16 + (lane >> 2));
            v = buf[line * 8 + (lane & 3)];
            if constexpr (PAT == 2) v2 = buf[line * 8 + 4 + (lane & 3)];
        } else if constexpr (PAT == 3) {
            const uint64_t line = scramble(w * 8 + (lane >> 3));
            v = buf[line * 8 + (lane & 7)];
        } else {
            const uint64_t line = scramble(w * 32 + (lane >> 1));
            v = buf[line * 8 + (lane & 1)];
        }
        acc += v.x + v.y + v.z + v.w + v2.x + v2.w;
    }
    if (acc == 12345.f) out[0] = acc;
}

int main() {
    float4 *buf;
    float *out;
    if (hipMalloc(&buf, kBytes) != hipSuccess) return 1;
    hipMemset(buf, 0, kBytes);
    hipMalloc(&out, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // units (one per wave iteration) and the lines / requested bytes they cover
    struct { const char *name; uint64_t units, lines, bytes; } pat[5] = {
        {"stream", kBytes / 1024, kLines, kBytes},
        {"lo64", kLines / 16, kLines, kLines * 64},
        {"lo64+hi64", kLines / 16, kLines, kLines * 128},
        {"line128", kLines / 8, kLines, kBytes},
        {"rec32", kLines / 32, kLines, kLines * 32},
    };
    for (int p = 0; p < 5; p++) {
        const dim3 g(8192), b(256);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        switch (p) {
        case 0: hipLaunchKernelGGL(k_cal<0>, g, b, 0, 0, buf, pat[p].units, out); break;
        case 1: hipLaunchKernelGGL(k_cal<1>, g, b, 0, 0, buf, pat[p].units, out); break;
        case 2: hipLaunchKernelGGL(k_cal<2>, g, b, 0, 0, buf, pat[p].units, out); break;
        case 3: hipLaunchKernelGGL(k_cal<3>, g, b, 0, 0, buf, pat[p].units, out); break;
        case 4: hipLaunchKernelGGL(k_cal<4>, g, b, 0, 0, buf, pat[p].units, out); break;
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("pattern %d %-10s lines %llu  requested bytes %llu  %.3f ms  %.1f GB/s requested, %.1f Glines/s\n",
               p, pat[p].name, (unsigned long long)pat[p].lines, (unsigned long long)pat[p].bytes, ms,
               pat[p].bytes / (ms * 1e-3) / 1e9, pat[p].lines / (ms * 1e-3) / 1e9);
    }
    return 0;
}
