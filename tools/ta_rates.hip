// ta_rates.hip -- per-CU cost of one global_load_dwordx4 wave-instruction by
// lane->address pattern (tooling).  Working set L1- or L2-resident so only the
// TA/TCP/TD path is measured.  Reports ns per wave-instruction per CU.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int PAT>
__device__ __forceinline__ uint32_t lane_off(uint32_t lane, uint32_t k) {
    // byte offsets; k varies the base per instruction
    if constexpr (PAT == 0) return lane * 16;                              // 1 KiB contiguous (8 lines)
    if constexpr (PAT == 1) return lane * 32;                              // every other 16 B (16 lines)
    if constexpr (PAT == 2) return (lane / 2) * 128 + (lane & 1) * 16;     // 2 lanes/line (32 lines)
    if constexpr (PAT == 3) return lane * 128;                             // 1 lane/line (64 lines)
    if constexpr (PAT == 4) return (lane >> 3) * 4096 + (lane & 7) * 32;   // 8 rows x 8 records of 32 B
    if constexpr (PAT == 5) return 0;                                      // broadcast (1 line)
    if constexpr (PAT == 6) return (lane & 3) * 16 + (lane >> 2) * 128;    // 4 lanes/line (16 lines)
    return 0;
}

template <int PAT>
__global__ __launch_bounds__(256) void k_ta(const char *__restrict__ buf, uint32_t span_mask,
                                            int iters, float *out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 7919u;
    float4 acc = make_float4(0, 0, 0, 0);
    for (int it = 0; it < iters; it++) {
        float4 v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t base = ((w + it * 8 + k) * 65536u) & span_mask;
            v[k] = *reinterpret_cast<const float4 *>(buf + base + lane_off<PAT>(lane, k));
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
            acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

int main() {
    char *buf;
    float *out;
    const size_t bytes = 64ull << 20;
    hipMalloc(&buf, bytes + (1 << 20));
    hipMemset(buf, 0, bytes + (1 << 20));
    hipMalloc(&out, 256 * 16 * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"1KiB contiguous (8 lines)", "32B stride (16 lines)",
                           "2 lanes/line (32 lines)", "1 lane/line (64 lines)",
                           "8 rows x 8 recs of 32B", "broadcast (1 line)", "4 lanes/line (16 lines)"};
    const int iters = 256;
    for (int span = 0; span < 2; span++) {
        // span 0: 64 KiB window (L1/L2 resident), span 1: 64 MiB (L2/MALL)
        const uint32_t mask = span == 0 ? 0xFFFFu & ~0xFFFu : (uint32_t)((bytes - 1) & ~0xFFFull);
        for (int pat = 0; pat < 7; pat++) {
            for (int wps = 1; wps <= 8; wps *= 8) {
                const int blocks = 256 * wps;  // wps waves per SIMD (256-thread blocks)
                auto launch = [&]() {
#define L(P) if (pat == P) hipLaunchKernelGGL(k_ta<P>, dim3(blocks), dim3(256), 0, 0, buf, mask, iters, out);
                    L(0) L(1) L(2) L(3) L(4) L(5) L(6)
                };
                launch();
                hipEventRecord(e0);
                launch();
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                const double instr_per_cu = (double)blocks * 4 * iters * 8 / 256.0;
                printf("%s %-28s %d waves/SIMD: %7.2f ns/instr/CU  (%6.1f GB/s/CU of lane bytes)\n",
                       span == 0 ? "64KiB" : "64MiB", names[pat], wps,
                       ms * 1e6 / instr_per_cu, instr_per_cu * 1024 / (ms * 1e-3) / 1e9);
            }
        }
    }
    return 0;
}
