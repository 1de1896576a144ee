// Microbenchmark (dev tool): f32 FMA throughput of v_fma_f32 vs v_pk_fma_f32
// on gfx950.  8 independent accumulator chains per lane, N iterations.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_scalar(float* out, float a, float b, int n) {
    float x[16];
    for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * 1e-3f + i;
    for (int it = 0; it < n; ++it)
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = __builtin_fmaf(x[i], a, b);
    float s = 0; for (int i = 0; i < 16; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_packed(float* out, float a, float b, int n) {
    f2 x[8];
    for (int i = 0; i < 8; ++i) x[i] = f2{threadIdx.x * 1e-3f + i, threadIdx.x * 2e-3f + i};
    const f2 A = {a, a}, B = {b, b};
    for (int it = 0; it < n; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], A, B);
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
    const int blocks = 256 * 8, n = 20000;
    float* d; hipMalloc(&d, blocks * 256 * 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
        for (int k = 0; k < 2; ++k) {
            hipEventRecord(e0);
            if (k == 0) hipLaunchKernelGGL(k_scalar, dim3(blocks), dim3(256), 0, 0, d, 0.999f, 1e-3f, n);
            else hipLaunchKernelGGL(k_packed, dim3(blocks), dim3(256), 0, 0, d, 0.999f, 1e-3f, n);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            const double flop = 2.0 * 16 * (double)n * blocks * 256;
            if (rep) printf("%s: %.3f ms  %.1f TFLOP/s\n", k ? "v_pk_fma_f32" : "v_fma_f32   ", ms, flop / ms / 1e9);
        }
    }
    return 0;
}
