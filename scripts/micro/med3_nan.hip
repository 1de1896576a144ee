// Dev probe (GPU): v_med3_f32 (__builtin_amdgcn_fmed3f) and v_max_f32 with
// quiet-NaN inputs on gfx950 in IEEE mode — the semantics pt_path.h's fmax_q
// relies on (PT_FMAX_MED3: med3(a, b, FLT_MAX) == fmaxf(a, b) for the values
// the margins can take).  hipcc --offload-arch=gfx950 -O2 med3_nan.hip -o med3_nan
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
__global__ void k(const float* a, const float* b, float* med, float* mx, int n) {
    const int i = threadIdx.x;
    if (i >= n) return;
    med[i] = __builtin_amdgcn_fmed3f(a[i], b[i], 3.40282347e38f);
    float r;
    asm volatile("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a[i]), "v"(b[i]));
    mx[i] = r;
}
int main() {
    const float nan = std::nanf(""), inf = INFINITY;
    const float A[] = {nan, 1.0f, nan, -1.0f, inf, -inf, nan, 2.0f, -0.0f};
    const float B[] = {1.0f, nan, nan, -inf, 3.0f, nan, inf, 2.0f, 0.0f};
    const int n = sizeof(A) / sizeof(A[0]);
    float *da, *db, *dm, *dx, hm[16], hx[16];
    hipMalloc(&da, 64); hipMalloc(&db, 64); hipMalloc(&dm, 64); hipMalloc(&dx, 64);
    hipMemcpy(da, A, sizeof A, hipMemcpyHostToDevice);
    hipMemcpy(db, B, sizeof B, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dm, dx, n);
    hipMemcpy(hm, dm, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hx, dx, n * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; ++i) {
        const float want = fmaxf(A[i], B[i]);
        const float wantc = (want == inf) ? 3.40282347e38f : want;   // med3 clamps at FLT_MAX
        const bool ok = (std::isnan(wantc) ? std::isnan(hm[i]) : hm[i] == wantc) &&
                        (std::isnan(want) ? std::isnan(hx[i]) : hx[i] == want);
        bad += !ok;
        printf("a=%g b=%g  med3(a,b,FLT_MAX)=%g  v_max=%g  fmaxf=%g %s\n", A[i], B[i], hm[i], hx[i], want,
               ok ? "ok" : "DIFF");
    }
    printf("med3_nan: %d differences\n", bad);
    return 0;
}
