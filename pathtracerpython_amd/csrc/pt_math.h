// pt_math.h — f64 elementary functions for the render kernel, sized for the
// argument ranges the path tracer actually uses.  The general OCML routines
// (sincos with Payne-Hanek reduction for huge arguments, IEEE division and
// sqrt sequences) cost the kernel ~100 extra VGPRs; these reach ~1 ulp with a
// fraction of the registers.  Results differ from numpy's by an ulp or two,
// far inside the parity tolerance (tests compare at 1e-12).  Host builds (the
// test-only host check) use libm.
#pragma once
#include <math.h>

#ifndef PT_HD
#define PT_HD __host__ __device__ __forceinline__
#endif

namespace pt {

#if defined(__HIP_DEVICE_COMPILE__)
// 1/x: v_rcp_f64 seed + two Newton steps (quadratic: ~24 -> ~48 -> full bits)
PT_HD double rcp_d(double x) {
    double y = __builtin_amdgcn_rcp(x);
    double e = fma(-x, y, 1.0);
    y = fma(y, e, y);
    e = fma(-x, y, 1.0);
    return fma(y, e, y);
}
// 1/sqrt(x), x > 0 normal: v_rsq_f64 seed + two Newton steps
PT_HD double rsqrt_d(double x) {
    double y = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
    double r = fma(-h * y, y, 0.5);
    y = fma(y, r, y);
    r = fma(-h * y, y, 0.5);
    return fma(y, r, y);
}
#else
PT_HD double rcp_d(double x) { return 1.0 / x; }
PT_HD double rsqrt_d(double x) { return 1.0 / sqrt(x); }
#endif

// sqrt for x >= 0 (0 -> 0)
PT_HD double sqrt_d(double x) { return x > 0.0 ? x * rsqrt_d(x) : 0.0; }

#if defined(__HIP_DEVICE_COMPILE__)
// sin and cos of x in [0, 8): Cody-Waite reduction by pi/2 (k <= 5, the
// 33-bit leading part times k is exact), then the fdlibm kernel polynomials
// on |r| <= pi/4 (Sun Microsystems fdlibm k_sin.c / k_cos.c coefficients).
PT_HD void sincos_small(double x, double* s, double* c) {
    const double pio2_1 = 1.57079632673412561417e+00;   // first 33 bits of pi/2
    const double pio2_1t = 6.07710050650619224932e-11;  // pi/2 - pio2_1
    const double k = rint(x * 6.36619772367581382433e-01);   // 2/pi
    const double r = (x - k * pio2_1) - k * pio2_1t;
    const double z = r * r;
    const double ps = z * (8.33333333332248946124e-03 +
                      z * (-1.98412698298579493134e-04 +
                      z * (2.75573137070700676789e-06 +
                      z * (-2.50507602534068634195e-08 +
                      z * 1.58969099521155010221e-10))));
    const double sr = r + r * z * (-1.66666666666666324348e-01 + ps);
    const double pc = z * (4.16666666666666019037e-02 +
                      z * (-1.38888888888741095749e-03 +
                      z * (2.48015872894767294178e-05 +
                      z * (-2.75573143513906633035e-07 +
                      z * (2.08757232129817482790e-09 +
                      z * -1.13596475577881948265e-11)))));
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double cr = w + (((1.0 - w) - hz) + z * pc);
    const int n = ((int)k) & 3;
    const double sv = (n & 1) ? cr : sr;
    const double cv = (n & 1) ? sr : cr;
    *s = (n & 2) ? -sv : sv;
    *c = ((n + 1) & 2) ? -cv : cv;
}
#else
PT_HD void sincos_small(double x, double* s, double* c) {
    *s = sin(x);
    *c = cos(x);
}
#endif

}  // namespace pt
