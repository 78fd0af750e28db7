// op_rates.hip -- issue cost of the decode's instructions on gfx950 (tooling).
// Each kernel runs a long loop of independent (ILP 8) or dependent chains of one
// operation; cycles per wave-instruction are reported for 1 wave/SIMD and
// 8 waves/SIMD (all 256 CUs busy).
#include <hip/hip_runtime.h>

#include <cstdio>

#define N_IT 4096

template <int OP, int ILP>
__global__ void k_op(float *out, float seed, long long *cyc) {
    float f[ILP];
    double d[ILP];
#pragma unroll
    for (int i = 0; i < ILP; i++) {
        f[i] = seed + i + threadIdx.x;
        d[i] = (double)f[i];
    }
    long long t0 = clock64();
    for (int it = 0; it < N_IT; it++) {
#pragma unroll
        for (int i = 0; i < ILP; i++) {
            if constexpr (OP == 0) f[i] = f[i] + 1.0001f;                 // v_add_f32
            if constexpr (OP == 1) d[i] = d[i] + 1.0001;                  // v_add_f64
            if constexpr (OP == 2) d[i] = d[i] * 1.0001;                  // v_mul_f64
            if constexpr (OP == 3) d[i] = (double)(float)d[i];            // cvt pair
            if constexpr (OP == 4) {                                      // one decode bin step
                f[i] = (float)((double)f[i] + (double)seed * 0.00123456789);
            }
            if constexpr (OP == 5) d[i] = __builtin_fma(d[i], 1.0001, 0.5);  // v_fma_f64
            if constexpr (OP == 6) f[i] = (float)((double)f[i] / 0.0217);     // f64 divide
        }
    }
    long long t1 = clock64();
    float acc = 0;
#pragma unroll
    for (int i = 0; i < ILP; i++) acc += f[i] + (float)d[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
    float *out;
    long long *cyc;
    hipMalloc(&out, 256 * 8 * 256 * 4 * sizeof(float));
    hipMalloc(&cyc, 8);
    const char *names[] = {"add_f32", "add_f64", "mul_f64", "cvt f64->f32->f64",
                           "decode bin step", "fma_f64", "f64 divide+cvt"};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int op = 0; op < 7; op++) {
        for (int cfg = 0; cfg < 4; cfg++) {
            // cfg: (ILP 1 | ILP 8) x (1 wave/SIMD | 8 waves/SIMD)
            const bool ilp8 = cfg & 1, full = cfg & 2;
            const int blocks = 256 * (full ? 8 : 1), threads = 256;
            auto launch = [&]() {
#define L(O)                                                                              \
    if (op == O) {                                                                        \
        if (ilp8) hipLaunchKernelGGL((k_op<O, 8>), dim3(blocks), dim3(threads), 0, 0, out, 1.5f, cyc); \
        else hipLaunchKernelGGL((k_op<O, 1>), dim3(blocks), dim3(threads), 0, 0, out, 1.5f, cyc);      \
    }
                L(0) L(1) L(2) L(3) L(4) L(5) L(6)
            };
            launch();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            long long c;
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            const double ops = (double)N_IT * (ilp8 ? 8 : 1);
            // wave-instructions per SIMD: blocks*4 waves / 1024 SIMDs * ops
            const double wi_per_simd = (double)blocks * 4 / 1024.0 * ops;
            printf("%-20s ILP%d %s waves/SIMD: %7.2f cyc/op (wave0 clock64)  %7.3f ns/op/SIMD (wall)\n",
                   names[op], ilp8 ? 8 : 1, full ? "8" : "1", (double)c / ops,
                   ms * 1e6 / wi_per_simd);
        }
    }
    return 0;
}
