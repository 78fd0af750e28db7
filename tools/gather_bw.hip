// gather_bw.hip -- achievable HBM bandwidth for runs of R contiguous bytes at
// random offsets of a 32 GiB buffer (tooling; sizes the march's memory floor).
// Each wave reads 1 KiB per instruction = 1024/R runs of R bytes (R = 64..1024),
// 16 instructions in flight per lane, grid-stride over 4 GiB of reads.
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}

template <int RUN>
__global__ __launch_bounds__(256) void k_gather(const float4 *__restrict__ buf, uint64_t nchunks16,
                                                uint64_t iters, float *out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    constexpr int per_run = RUN / 16;             // lanes per run
    float4 acc = make_float4(0, 0, 0, 0);
    for (uint64_t it = 0; it < iters; it++) {
        float4 v[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint64_t run = mix(wave * 1315423911ull + it * 16 + k) * 64 + lane / per_run;
            const uint64_t nruns = nchunks16 / per_run;
            const uint64_t c = (mix(run) % nruns) * per_run + lane % per_run;
            v[k] = buf[c];
        }
#pragma unroll
        for (int k = 0; k < 16; k++) {
            acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

int main() {
    const size_t bytes = 32ull << 30;
    float4 *buf;
    float *out;
    if (hipMalloc(&buf, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(buf, 0, bytes);
    const int blocks = 256 * 8;
    hipMalloc(&out, blocks * 256 * 4);
    const uint64_t n16 = bytes / 16;
    const uint64_t iters = 64;  // 2048 blocks * 4 waves * 64 it * 16 KiB = 8 GiB per launch
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](int r) {
        switch (r) {
        case 64: hipLaunchKernelGGL(k_gather<64>, dim3(blocks), dim3(256), 0, 0, buf, n16, iters, out); break;
        case 128: hipLaunchKernelGGL(k_gather<128>, dim3(blocks), dim3(256), 0, 0, buf, n16, iters, out); break;
        case 256: hipLaunchKernelGGL(k_gather<256>, dim3(blocks), dim3(256), 0, 0, buf, n16, iters, out); break;
        case 512: hipLaunchKernelGGL(k_gather<512>, dim3(blocks), dim3(256), 0, 0, buf, n16, iters, out); break;
        case 1024: hipLaunchKernelGGL(k_gather<1024>, dim3(blocks), dim3(256), 0, 0, buf, n16, iters, out); break;
        }
    };
    const int runs[] = {64, 128, 256, 512, 1024};
    for (int r : runs) {
        run(r);
        hipEventRecord(e0);
        run(r);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double gb = (double)blocks * 4 * iters * 16 * 1024 / 1e9;
        printf("run %5d B: %8.1f GB/s  (%.3f ms for %.2f GB)\n", r, gb / (ms * 1e-3), ms, gb);
    }
    return 0;
}
