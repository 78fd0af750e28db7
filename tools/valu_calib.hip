// valu_calib.hip -- calibrates the VALU issue counters against kernels of known
// instruction counts (tooling): bench.py's roofline.compute block divides
// SQ_ACTIVE_INST_VALU by the chip's SIMD cycles, so this fixes what one unit of
// that counter is on gfx950 for f32 and f64 instructions.
//
//   hipcc --offload-arch=gfx950 -O3 tools/valu_calib.hip -o tools/build/valu_calib
//   rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
//       --output-format csv -d OUT -- tools/build/valu_calib
//
// Each wave runs kIt x kIlp independent adds (f32 or f64): exactly
// kIt * kIlp VALU instructions of that type in the loop, all SIMDs busy with 4
// waves each; the program prints the measured time, the wave-instructions per
// SIMD-cycle (clock from s_memtime) and what the counter must read per
// instruction for each hypothesis.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIt = 8192, kIlp = 8;

template <typename T>
__global__ __launch_bounds__(256) void k_add(T *out, T seed, long long *cyc) {
    T v[kIlp];
#pragma unroll
    for (int i = 0; i < kIlp; i++) v[i] = seed + (T)(i + threadIdx.x);
    const long long t0 = clock64();
    for (int it = 0; it < kIt; it++) {
#pragma unroll
        for (int i = 0; i < kIlp; i++) {  // exactly one VALU instruction each (no packing)
            if constexpr (sizeof(T) == 4) asm volatile("v_add_f32 %0, 1.0, %0" : "+v"(v[i]));
            else asm volatile("v_add_f64 %0, 1.0, %0" : "+v"(v[i]));
        }
    }
    const long long t1 = clock64();
    T acc = 0;
#pragma unroll
    for (int i = 0; i < kIlp; i++) acc += v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <typename T>
static void run(const char *name) {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 4;  // 4 workgroups of 4 waves per CU: 4 waves per SIMD
    T *out = nullptr;
    long long *cyc = nullptr;
    hipMalloc(&out, sizeof(T) * blocks * 256);
    hipMalloc(&cyc, sizeof(long long));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k_add<T>, dim3(blocks), dim3(256), 0, 0, out, (T)1, cyc);
        hipEventRecord(b);
        hipEventSynchronize(b);
    }
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    long long c = 0;
    hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
    const double waves = (double)blocks * 4, instr = waves * kIt * kIlp;
    const double simds = cus * 4.0;
    // wave 0's loop: 4 waves share its SIMD, so cycles / (4 * kIt * kIlp) = cycles per
    // wave-instruction of SIMD issue
    printf("%s: %d CUs, %.0f waves, %.3e loop VALU instr, %.3f ms, wave-0 loop %lld cycles "
           "-> %.2f SIMD cycles per wave-instruction; counter per instruction if it counts "
           "cycles / quad-cycles: %.2f / %.2f\n",
           name, cus, waves, instr, ms, c, (double)c / (4.0 * kIt * kIlp),
           (double)c / (4.0 * kIt * kIlp), (double)c / (4.0 * kIt * kIlp) / 4.0);
    (void)simds;
    hipFree(out);
    hipFree(cyc);
}

int main() {
    run<float>("f32 v_add");
    run<double>("f64 v_add");
    return 0;
}
