// Microbenchmark (dev tool): issue rate of v_fma_mix_f32 (f16 src0, f32 src1 / src2)
// vs v_fma_f32 vs v_cvt_f32_ubyte0 + v_fma_f32 on gfx950: 16 independent chains per lane.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define CHAINS 16
template <int K>
__global__ __launch_bounds__(256) void k_probe(float* out, uint32_t w, float b, int n) {
    float x[CHAINS];
    for (int i = 0; i < CHAINS; ++i) x[i] = threadIdx.x * 1e-3f + i;
    const uint32_t hw = w + threadIdx.x;
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int i = 0; i < CHAINS; ++i) {
            if (K == 0) asm volatile("v_fma_f32 %0, %1, %0, %2" : "+v"(x[i]) : "v"(b), "v"(b));
            if (K == 1) asm volatile("v_fma_mix_f32 %0, %1, %0, %2 op_sel_hi:[1,0,0]" : "+v"(x[i]) : "v"(hw), "v"(b));
            if (K == 2) {
                float t;
                asm volatile("v_cvt_f32_ubyte0 %0, %1" : "=v"(t) : "v"(hw));
                asm volatile("v_fma_f32 %0, %1, %0, %2" : "+v"(x[i]) : "v"(t), "v"(b));
            }
        }
    }
    float s = 0;
    for (int i = 0; i < CHAINS; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
    const int blocks = 256 * 8, n = 20000;
    float* d;
    hipMalloc(&d, blocks * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[3] = {"v_fma_f32", "v_fma_mix_f32", "v_cvt_f32_ubyte0 + v_fma_f32"};
    for (int rep = 0; rep < 2; ++rep)
        for (int k = 0; k < 3; ++k) {
            hipEventRecord(e0);
            if (k == 0) hipLaunchKernelGGL(k_probe<0>, dim3(blocks), dim3(256), 0, 0, d, 0x3c00u, 1e-3f, n);
            if (k == 1) hipLaunchKernelGGL(k_probe<1>, dim3(blocks), dim3(256), 0, 0, d, 0x3c00u, 1e-3f, n);
            if (k == 2) hipLaunchKernelGGL(k_probe<2>, dim3(blocks), dim3(256), 0, 0, d, 0x3c00u, 1e-3f, n);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double fmas = (double)CHAINS * n * blocks * 256;
            if (rep) printf("%-30s %.3f ms  %.2f G fma-steps/s per CU\n", names[k], ms, fmas / ms / 1e6 / 256);
        }
    return 0;
}
