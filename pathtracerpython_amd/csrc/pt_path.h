// pt_path.h — per-lane path logic of the render kernel (closest hit, direct
// light, bounce), written once for the gfx950 kernels (pt_hip.hip) and for
// the host-side check build used by tests (tests/hostcheck).
//
// Reference loop flattened (main.py:186-271): per (pixel, sample) the
// spp x bounce iteration of the reference becomes an iterative bounce loop in
// registers; the reference's per-bounce pool phases (main.py:197-231) become
// closest() and nee() calls.
#pragma once
#include "pt_core.h"

#if defined(__HIP_DEVICE_COMPILE__)
#define PT_WAVE_ALL(x) (__all(x) != 0)
#else
#define PT_WAVE_ALL(x) (x)
#endif

namespace pt {

struct Counters {
    uint32_t closest_tests, shadow_tests, ray_bounces, shading_points;
    uint32_t light_hits, escapes, fallbacks, rescans;
};

template <bool COUNT>
PT_HD void bump(Counters* c, uint32_t Counters::*f, uint32_t v) {
    if (COUNT) c->*f += v;
}

// ----------------------------------------------------------- closest hit --
// intersect_objects (main.py:83-122): the triangle whose intersection has the
// smallest squared distance > 1e-5 from the origin, objects first, light
// last, first minimum wins.  d need not be normalised (utils.py:110).
// Returns the triangle index (-1 = None) and the hit point P (f64).  ogrp: the
// coplanar group of the triangle the origin lies on (-1: none / unknown).
template <bool FORCE64, bool COUNT>
PT_HD int closest(const SceneK& S, D3 o, D3 d, int ogrp, D3* P, Counters* cnt) {
    const D3 dn = unit(d);
    int best = -1;
    bool decided = false;
    if (!FORCE64) {
        const F3 o32 = to_f3(o - ld3(S.center));
        const F3 d32 = to_f3(dn);
        float a1 = INFINITY, a2 = INFINITY, b1 = INFINITY;
        int i1 = -1;
        for (int t = 0; t < S.n_tri; ++t) {
            const TriF T = S.trif[t];
            const OriginF O = origin_f(T, o32);
            float at = 0.f, dt = 0.f;
            int st = classify(T, O, d32, INFINITY, INFINITY, &at, &dt);
            if (T.grp == ogrp) st = kMiss;
            float a = INFINITY, b = INFINITY;
            if (st == kCand) { a = at - dt; b = at + dt; }
            if (st == kAmb) {   // rare: decide this test in f64
                D3 Q; double sqd;
                bump<COUNT>(cnt, &Counters::fallbacks, 1);
                if (eval64(S.trid[t], o, dn, &Q, &sqd) && sqd > kZero) {
                    const float s = (float)sqrt(sqd);
                    a = s * (1.0f - 1e-6f);
                    b = s * (1.0f + 1e-6f);
                }
            }
            if (a < a1) { a2 = a1; a1 = a; b1 = b; i1 = t; }
            else { a2 = fminf(a2, a); }
        }
        // the candidate with the smallest lower bound is certainly the
        // closest when its interval ends before every other one starts
        decided = (i1 < 0) || (b1 < a2);
        best = i1;
    }
    if (!decided) {   // exact f64 scan (FORCE64, or overlapping intervals)
        if (!FORCE64) bump<COUNT>(cnt, &Counters::rescans, 1);
        best = -1;
        double bsq = 0.0;
        for (int t = 0; t < S.n_tri; ++t) {
            D3 Q; double sqd;
            if (eval64(S.trid[t], o, dn, &Q, &sqd) && sqd > kZero && (best < 0 || sqd < bsq)) {
                best = t;
                bsq = sqd;
            }
        }
    }
    if (best >= 0) {   // hit point exactly as the reference computes it
        double sqd;
        eval64(S.trid[best], o, dn, P, &sqd);
    }
    bump<COUNT>(cnt, &Counters::closest_tests, (uint32_t)S.n_tri);
    bump<COUNT>(cnt, &Counters::ray_bounces, 1);
    return best;
}

// ---------------------------------------------------------- direct light --
// compute_color (main.py:142-145) = compute_ambient_color (main.py:76-80) +
// compute_shadow_rays (main.py:23-73) at hit point P with normal n on object
// `obj`.  u: the 12 light-sampling uniforms (slots 0..11).  Occlusion: any
// OBJECT triangle hit with 1e-5 <= sqd < |P - L|^2 (main.py:42-55, line
// semantics); the colour factor is that of `obj` after the loop of the LAST
// shadow ray (main.py:70): its first occluding object, else the last object.
template <bool FORCE64, bool COUNT>
PT_HD D3 nee(const SceneK& S, D3 P, D3 n, int obj, int ogrp, const double u[12], Counters* cnt) {
    D3 dn[kLightSamples];
    double lsq[kLightSamples];
    float hlo[kLightSamples], hhi[kLightSamples];
    F3 d32[kLightSamples];
    bool occ[kLightSamples];
    int first[kLightSamples];
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) {
        const int li = pick_light(S, u[4 * k]);
        const D3 L = light_point(S.trid[S.light_tri[li]], u[4 * k + 1], u[4 * k + 2], u[4 * k + 3]);
        dn[k] = unit(L - P);
        lsq[k] = squared_dist(P, L);
        const double tl = sqrt(lsq[k]);
        hlo[k] = (float)(tl * (1.0 - 1e-6));
        hhi[k] = (float)(tl * (1.0 + 1e-6));
        d32[k] = to_f3(dn[k]);
        occ[k] = false;
        first[k] = S.n_obj_tri;
    }
    int leak = S.n_obj - 1;
    const F3 o32 = to_f3(P - ld3(S.center));
    for (int t = 0; t < S.n_obj_tri; ++t) {
        if (PT_WAVE_ALL(occ[0] && occ[1] && occ[2])) break;
        const TriF T = S.trif[t];
        const OriginF O = FORCE64 ? OriginF{0.f, 0.f, 0.f} : origin_f(T, o32);
        const bool coplanar = (T.grp == ogrp);
#pragma unroll
        for (int k = 0; k < kLightSamples; ++k) {
            if (occ[k]) continue;
            bool hit;
            int st = kAmb;
            if (!FORCE64) {
                float at, dt;
                st = classify(T, O, d32[k], hlo[k], hhi[k], &at, &dt);
                if (coplanar) st = kMiss;
            }
            if (st == kAmb) {
                D3 Q; double sqd;
                if (!FORCE64) bump<COUNT>(cnt, &Counters::fallbacks, 1);
                hit = eval64(S.trid[t], P, dn[k], &Q, &sqd) && !(sqd < kZero) && sqd < lsq[k];
            } else {
                hit = (st == kCand);
            }
            if (hit) {
                occ[k] = true;
                first[k] = t + 1;
                if (k == kLightSamples - 1) leak = S.tri_obj[t];
            }
        }
    }
    double dsum = 0.0;
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) {
        if (!occ[k]) dsum += dot(dn[k], n);
        bump<COUNT>(cnt, &Counters::shadow_tests, (uint32_t)first[k]);
    }
    dsum /= (double)kLightSamples;
    const Mat& m = S.mat[obj];
    const Mat& lm = S.mat[leak];
    bump<COUNT>(cnt, &Counters::shading_points, 1);
    return d3(m.rgb[0] * m.ka * S.ambient + S.light_rgb[0] * lm.rgb[0] * dsum,
              m.rgb[1] * m.ka * S.ambient + S.light_rgb[1] * lm.rgb[1] * dsum,
              m.rgb[2] * m.ka * S.ambient + S.light_rgb[2] * lm.rgb[2] * dsum);
}

// ---------------------------------------------------------------- bounce --
// Next-ray generation, main.py:236-268.  d_old is the incoming direction as
// the reference holds it (unnormalised for primary rays).  Returns the new
// direction and the throughput factor (accumulated_k update).
PT_HD D3 bounce(const SceneK& S, const TriS& R, const Mat& m, D3 P, D3 d_old,
                double u_sel, double u_phi, double u_theta, double* kf) {
    const D3 n = ld3(R.n);
    const double xi = 0.0 + (m.kdks - 0.0) * u_sel;
    if (xi <= m.kd) {   // diffuse: phi = arccos(sqrt(u)), theta = 6.28 u
        const double cphi = sqrt(u_phi);
        const double sphi = sqrt(1.0 - u_phi);   // sin(arccos(sqrt(u)))
        const double th = kTau * u_theta;
        double st, ct;
#if defined(__HIP_DEVICE_COMPILE__)
        sincos(th, &st, &ct);
#else
        st = sin(th);
        ct = cos(th);
#endif
        const D3 nd = rotate_y(R, d3(sphi * ct, sphi * st, cphi));
        *kf = m.kd * dot(nd, n);
        return nd;
    }
    // "specular": r = 2 (n.d) n - d, normalised, rotated; k *= ks (e.r)^n
    const double nd2 = dot(n, d_old) * 2;
    const D3 r = unit(d3(nd2 * n.x - d_old.x, nd2 * n.y - d_old.y, nd2 * n.z - d_old.z));
    const D3 e = unit(ld3(S.eye) - P);
    const D3 nd = rotate_y(R, r);
    *kf = m.ks * pow_ref(dot(e, nd), m);
    return nd;
}

PT_HD double linspace_at(double a, double b, int n, int i) {   // np.linspace
    if (n == 1) return a;
    if (i == n - 1) return b;
    const double step = (b - a) / (double)(n - 1);
    return (double)i * step + a;
}

// ------------------------------------------------------------ one lane --
struct LaneJob {
    uint64_t seed;
    uint32_t pixel;          // reference list index k = ix*H + iy
    int32_t sample0;         // first sample index
    int32_t sample_stride;
    int32_t n_samples;
    int32_t bounces;
    int32_t rr_depth;        // < 0: no Russian roulette
};

// All samples of one lane for one pixel; returns the SUM of sample colours.
// Paths are regenerated in place: when a path ends the lane starts its next
// sample from the cached primary hit (primary rays are identical for every
// sample, main.py:191), so a wave keeps tracing until all its lanes are out
// of samples.
template <bool FORCE64, bool COUNT>
PT_HD D3 render_lane(const SceneK& S, const LaneJob& J, D3 eye, D3 d0, int tri0, D3 P0,
                     Counters* cnt) {
    D3 acc = d3(0, 0, 0);
    if (J.n_samples <= 0 || J.bounces <= 0) return acc;   // main.py:192 never runs
    if (tri0 < 0 || tri0 >= S.n_obj_tri) {   // primary ray escapes or hits the light
        const D3 v = tri0 < 0 ? d3(0, 0, 0) : ld3(S.light_rgb);
        for (int i = 0; i < J.n_samples; ++i) {
            acc = acc + v;
            if (COUNT) {
                bump<COUNT>(cnt, &Counters::closest_tests, (uint32_t)S.n_tri);
                bump<COUNT>(cnt, &Counters::ray_bounces, 1);
                bump<COUNT>(cnt, &Counters::escapes, tri0 < 0 ? 1u : 0u);
                bump<COUNT>(cnt, &Counters::light_hits, tri0 < 0 ? 0u : 1u);
            }
        }
        return acc;
    }
    int si = 0;
    int b = 0;
    int tri = tri0;
    D3 P = P0, d = d0, rgb = d3(0, 0, 0);
    double k = 1.0;
    bool active = true;
    if (COUNT) {   // the cached primary trace, counted per sample
        bump<COUNT>(cnt, &Counters::closest_tests, (uint32_t)S.n_tri);
        bump<COUNT>(cnt, &Counters::ray_bounces, 1);
    }
    while (active) {
        const uint32_t sample = (uint32_t)(J.sample0 + si * J.sample_stride);
        const int obj = S.tri_obj[tri];
        const TriS R = S.tris[tri];
        const Mat& m = S.mat[obj];
        // direct light at this hit (slots 0..11)
        double u[12];
        uint32_t w[4];
#pragma unroll
        for (int blk = 0; blk < 3; ++blk) {
            rng_block(J.seed, J.pixel, sample, (uint32_t)b, (uint32_t)blk, w);
#pragma unroll
            for (int j = 0; j < 4; ++j) u[4 * blk + j] = u_of(w[j]);
        }
        const int ogrp = S.trif[tri].grp;
        const D3 col = nee<FORCE64, COUNT>(S, P, ld3(R.n), obj, ogrp, u, cnt);
        rgb = rgb + col * k;   // main.py:230-231
        // next ray (slots 12..15)
        rng_block(J.seed, J.pixel, sample, (uint32_t)b, 3u, w);
        double kf;
        const D3 nd = bounce(S, R, m, P, d, u_of(w[0]), u_of(w[1]), u_of(w[2]), &kf);
        k *= kf;
        bool done = (b + 1 >= J.bounces);
        if (!done && J.rr_depth >= 0 && b >= J.rr_depth) {   // build extension
            double q = fabs(k);
            q = q < 0.05 ? 0.05 : (q > 1.0 ? 1.0 : q);
            if (u_of(w[3]) >= q) done = true;
            else k /= q;
        }
        if (!done) {
            D3 Pn;
            const int tn = closest<FORCE64, COUNT>(S, P, nd, ogrp, &Pn, cnt);
            if (tn < 0) {
                bump<COUNT>(cnt, &Counters::escapes, 1);
                done = true;
            } else if (tn >= S.n_obj_tri) {   // light: main.py:214-215
                rgb = rgb + ld3(S.light_rgb) * k;
                bump<COUNT>(cnt, &Counters::light_hits, 1);
                done = true;
            } else {
                d = nd;
                P = Pn;
                tri = tn;
                ++b;
            }
        }
        if (done) {
            acc = acc + rgb;
            ++si;
            if (si >= J.n_samples) {
                active = false;
            } else {   // next sample from the cached primary hit
                b = 0;
                tri = tri0;
                P = P0;
                d = d0;
                k = 1.0;
                rgb = d3(0, 0, 0);
                if (COUNT) {
                    bump<COUNT>(cnt, &Counters::closest_tests, (uint32_t)S.n_tri);
                    bump<COUNT>(cnt, &Counters::ray_bounces, 1);
                }
            }
        }
    }
    (void)eye;
    return acc;
}

}  // namespace pt
