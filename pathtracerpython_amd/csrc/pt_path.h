// pt_path.h — per-lane path logic of the render kernel (closest hit, direct
// light, bounce), written once for the gfx950 kernels (pt_hip.hip) and for
// the host-side check build used by tests (tests/hostcheck).
//
// Reference loop flattened (main.py:186-271): per (pixel, sample) the
// spp x bounce iteration of the reference becomes an iterative bounce loop in
// registers.  Per bounce the reference runs two pool phases (closest hit
// main.py:197-205, colour main.py:208-231) and then samples the next ray
// (main.py:236-268).  The next ray does not depend on the colour phase, so a
// bounce here samples it first and runs ONE pass over the triangles that
// tests the 3 shadow rays (main.py:42-55) and the next ray's closest hit
// (main.py:94-109) together: the four lines share their origin, so the
// origin terms of each test are computed once.
#pragma once
#include "pt_core.h"
#include <assert.h>

#if defined(__HIP_DEVICE_COMPILE__)
#define PT_WAVE_ALL(x) (__all(x) != 0)
#define PT_WAVE_ANY(x) (__any(x) != 0)
#else
#define PT_WAVE_ALL(x) (x)
#define PT_WAVE_ANY(x) (x)
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

// Per-lane f64 scratch that the f32 test loops only touch on a fallback or
// once per bounce: a home in LDS on the device (structure-of-arrays,
// conflict-free) that the register allocator can reload from instead of
// keeping these values live across the loops.  (Not volatile: a volatile
// access counts as a possible clobber of global memory, which would stop the
// compiler from using scalar loads for the uniform triangle reads.)  Slots:
//   0..8  light sample points L_k       9..11  next-ray direction (as the
//   12..14 ray origin P                        reference holds it, unnormalised)
//   15..16 primary direction d0 (x, y; its z is -eye.z)
//   17..19 primary hit point P0
// The path's origin P and the cached primary hit P0 live here rather than in
// VGPRs across the bounce loop: 20 slots x 256 lanes = 40 KB per block, the
// 160 KB of a CU at 4 blocks (the register allocator otherwise spills them to
// scratch, which costs ~1.2 GB of HBM writes per K2 launch).
struct Spill {
    double* base;
    int stride;
    PT_HD double get(int i) const { return base[i * stride]; }
    PT_HD void put(int i, double v) const { base[i * stride] = v; }
    PT_HD D3 get3(int i) const { return d3(get(i), get(i + 1), get(i + 2)); }
    PT_HD void put3(int i, D3 v) const { put(i, v.x); put(i + 1, v.y); put(i + 2, v.z); }
};
constexpr int kSpillSlots = 20;
// PT_WF_LRNG: a wavefront path record (pt_wavefront.h WfPath) keeps no light
// points — shadow_setup_k<.., false> does not store them, and the rare f64
// blocks that need one draw it again from the slot's RNG key (wf_light; the
// record's light-point slots hold that key, WfPath::put_rkey).  Writing the
// points into the record's second line cost the shade step 10% (a
// partial-line write per slot and bounce).  The render kernel's LDS home is
// unchanged (a compile-time choice: the kernel's code stays as it was).
#ifndef PT_WF_LRNG
#define PT_WF_LRNG 1
#endif
#ifndef PT_SETUP_REUSE
#define PT_SETUP_REUSE 1
#endif
// P and Nd first: the wavefront path record (pt_wavefront.h WfPath) keeps them
// in the same 128-B line as the per-step fields; the light points and the
// primary hit follow in the other line
constexpr int kSpP = 0, kSpNd = 3, kSpL = 6, kSpD0 = 15, kSpP0 = 17;

// ----------------------------------------------------------- closest hit --
// intersect_objects (main.py:83-122): the triangle whose intersection has the
// smallest squared distance > 1e-5 from the origin, objects first, light
// last, first minimum wins.
struct ClosestAcc {   // f32 interval bookkeeping of the candidates
    float a1, a2, b1;
    int i1;
};
PT_HD ClosestAcc closest_init() { ClosestAcc c; c.a1 = c.a2 = c.b1 = INFINITY; c.i1 = -1; return c; }
PT_HD void closest_add(ClosestAcc* c, int t, float a, float b) {
    if (a < c->a1) { c->a2 = c->a1; c->a1 = a; c->b1 = b; c->i1 = t; }
    else { c->a2 = fminf(c->a2, a); }
}

// Origin terms of a unit (shared by every ray from the same origin): the
// plane distance and each triangle's barycentric forms at the origin.
struct OriginU { float h, bo0, co0, bo1, co1, eh = 0.f, eo = 0.f; };
PT_HD OriginU origin_u(const UnitF& U, F3 o) {
    OriginU r;
    r.eh = U.eh;
    r.eo = U.eo;
    r.h = aff3(U.n, U.cn, o);
    r.bo0 = aff3(U.tri[0].gb, U.tri[0].cb, o);
    r.co0 = aff3(U.tri[0].gc, U.tri[0].cc, o);
    r.bo1 = r.co1 = 0.f;
    if (U.count == 2) {   // wave-uniform
        r.bo1 = aff3(U.tri[1].gb, U.tri[1].cb, o);
        r.co1 = aff3(U.tri[1].gc, U.tri[1].cc, o);
    }
    return r;
}

template <bool COUNT>
PT_HD void closest_tri(const SceneK& S, const TriB& B, int t, const RayPlane& p, float bo, float co,
                       F3 d32, bool coplanar, const Spill& sp, int o_slot, int dn_slot,
                       ClosestAcc* acc, Counters* cnt) {
    const int st = coplanar ? kMiss : verdict_code(classify_tri(B, p, bo, co, d32));
    float a = (st == kCand) ? p.at - p.dt : INFINITY;
    float b = (st == kCand) ? p.at + p.dt : INFINITY;
    if (st == kAmb) {   // rare: decide this test in f64
        D3 Q;
        double sqd;
        bump<COUNT>(cnt, &Counters::fallbacks, 1);
        if (eval64(S.trid[t], sp.get3(o_slot), unit(sp.get3(dn_slot)), &Q, &sqd) && sqd > kZero) {
            const float sq = sqrtf((float)sqd);   // |t| to ~1e-7; brackets are 1e-6
            a = sq * (1.0f - 1e-6f);
            b = sq * (1.0f + 1e-6f);
        }
    }
    closest_add(acc, t, a, b);
}

// One closest-hit ray against one plane unit.
template <bool COUNT>
PT_HD void closest_unit(const SceneK& S, const UnitF& U, const OriginU& O, F3 d32, bool coplanar,
                        const Spill& sp, int o_slot, int dn_slot, ClosestAcc* acc,
                        Counters* cnt) {
    const RayPlane p = ray_plane(U, O.h, d32, INFINITY, INFINITY);
    closest_tri<COUNT>(S, U.tri[0], U.t[0], p, O.bo0, O.co0, d32, coplanar, sp, o_slot, dn_slot, acc, cnt);
    if (U.count == 2)
        closest_tri<COUNT>(S, U.tri[1], U.t[1], p, O.bo1, O.co1, d32, coplanar, sp, o_slot, dn_slot, acc, cnt);
}

// BVH helpers (the traversal itself, bvh_pass, follows fused_unit below)
PT_HD F3 rcp_dir(F3 d) {   // 1/d; a zero component gives +-1e30 (finite: no 0 * inf)
    F3 r;
    r.x = 1.0f / (d.x == 0.0f ? 1e-30f : d.x);
    r.y = 1.0f / (d.y == 0.0f ? 1e-30f : d.y);
    r.z = 1.0f / (d.z == 0.0f ? 1e-30f : d.z);
    return r;
}
// slab test of the line o + t d against a box given relative to o (lo - o,
// hi - o): some |t| <= R inside (the line is two-sided, utils.py:118-120)
PT_HD bool box_hit(F3 l, F3 h, F3 inv, float R) {
    const float ax = l.x * inv.x, bx = h.x * inv.x;
    const float ay = l.y * inv.y, by = h.y * inv.y;
    const float az = l.z * inv.z, bz = h.z * inv.z;
    const float tmin = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float tmax = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    return (tmin <= tmax) & (tmin <= R) & (tmax >= -R);
}

// f64 rescan of the BVH triangles within |t| <= R (an upper bound of the true
// closest distance): the reference's closest hit, ties to the lower index
PT_HD void bvh_rescan(const SceneK& S, D3 o, D3 dn, float R, int* best, double* bsq) {
    const F3 o32 = to_f3(o - ld3(S.center));
    const F3 inv = rcp_dir(to_f3(dn));
    int node = 0;
    while (node >= 0) {
        const BNode N = S.bnode[node];
        const F3 l = {N.lo[0] - o32.x, N.lo[1] - o32.y, N.lo[2] - o32.z};
        const F3 h = {N.hi[0] - o32.x, N.hi[1] - o32.y, N.hi[2] - o32.z};
        const bool hit = box_hit(l, h, inv, R);
        if (hit && N.leaf >= 0) {
            const int u0 = N.leaf >> 3, nu = N.leaf & 7;
            for (int i = 0; i < nu; ++i) {
                const UnitF& U = S.bunit[u0 + i];
                for (int m = 0; m < U.count; ++m) {
                    const int t = U.t[m];
                    D3 Q;
                    double sqd;
                    if (eval64(S.trid[t], o, dn, &Q, &sqd) && sqd > kZero &&
                        (*best < 0 || sqd < *bsq || (sqd == *bsq && t < *best))) {
                        *best = t;
                        *bsq = sqd;
                    }
                }
            }
        }
        node = (hit && N.leaf < 0) ? node + 1 : N.skip;
    }
}

// Finish a closest-hit query: the candidate with the smallest lower bound is
// certainly the closest when its interval ends before every other one
// starts; otherwise rescan exactly in f64.  Returns the triangle (-1 = None)
// and the hit point exactly as the reference computes it.
// P_home: when given, the hit point also goes to that spill slot (the
// render loop's next origin), written where it is computed so that it is not
// carried in VGPRs across the join.
template <bool FORCE64, bool COUNT, bool BVH = true>
PT_HD int closest_finish(const SceneK& S, const ClosestAcc& c, D3 o, D3 dn, D3* P,
                         Counters* cnt, const Spill* P_home = nullptr) {
    int best = c.i1;
    const bool decided = !FORCE64 && ((c.i1 < 0) || (c.b1 < c.a2));
    if (!decided) {
        if (!FORCE64) bump<COUNT>(cnt, &Counters::rescans, 1);
        best = -1;
        double bsq = 0.0;
        if (FORCE64 || !BVH || S.n_bnode == 0) {
            for (int t = 0; t < S.n_tri; ++t) {
                D3 Q; double sqd;
                if (eval64(S.trid[t], o, dn, &Q, &sqd) && sqd > kZero && (best < 0 || sqd < bsq)) {
                    best = t;
                    bsq = sqd;
                }
            }
        } else {   // the uniform units' triangles, then the BVH within |t| <= b1
            for (int u = 0; u < S.n_unit; ++u) {
                const UnitF& U = S.unit[u];
                for (int m = 0; m < U.count; ++m) {
                    const int t = U.t[m];
                    D3 Q; double sqd;
                    if (eval64(S.trid[t], o, dn, &Q, &sqd) && sqd > kZero &&
                        (best < 0 || sqd < bsq || (sqd == bsq && t < best))) {
                        best = t;
                        bsq = sqd;
                    }
                }
            }
            bvh_rescan(S, o, dn, c.b1, &best, &bsq);
        }
    }
    if (P_home) {   // branch-free (the winner passed eval64): a miss writes a point nobody reads
        *P = plane_point(S.trid[best >= 0 ? best : 0], o, dn);
        P_home->put3(kSpP, *P);
    } else if (best >= 0) {
        double sqd;
        eval64(S.trid[best], o, dn, P, &sqd);
    }
    bump<COUNT>(cnt, &Counters::closest_tests, (uint32_t)S.n_tri);
    bump<COUNT>(cnt, &Counters::ray_bounces, 1);
    return best;
}

// ---------------------------------------------------------- direct light --
// compute_color (main.py:142-145) = compute_ambient_color (main.py:76-80) +
// compute_shadow_rays (main.py:23-73).  Occlusion: any OBJECT triangle hit
// with 1e-5 <= sqd < |P - L|^2 (main.py:42-55, line semantics); the colour
// factor is that of `obj` after the loop of the LAST shadow ray (main.py:70):
// its first occluding object, else the last object.
struct ShadowSet {
    F3 d32[kLightSamples];
    float hlo[kLightSamples], hhi[kLightSamples];
    bool occ[kLightSamples];
    int first[kLightSamples];  // count mode: lowest occluding triangle (n_tri: none)
    // the last ray's first occluder (main.py:70): only its object matters for
    // the colour, and objects are contiguous in scene order, so outside count
    // mode the lowest occluding OBJECT is tracked (n_obj: none) — an occluded
    // ray then only looks at lower objects; count mode tracks the lowest
    // triangle (n_tri: none) for the reference's test counts
    int key2;
    double ln[kLightSamples];  // l_k . n of each light sample (main.py:66-68), from setup
    int leak;                  // its object (main.py:70), the last object when none
};

// Light sample k uses the uniforms of slots 4k..4k+3 (one Philox block: the
// triangle pick utils.py:30 and the three barycentric draws utils.py:23).
// The points go to the spill; f32 copies of the directions and distance
// brackets into sh, with l_k . n for the colour.  u: the 12 uniforms (the
// render loop draws them with rng_blocks4; the batched API passes them in).
// light sample k of shadow_setup (u: its 4 uniforms)
template <bool COUNT, bool STORE_L = true>
PT_HD void shadow_setup_k(const SceneK& S, D3 P, D3 n, int k, double u0, double u1, double u2,
                          double u3, ShadowSet* sh, const Spill& sp) {
    const int li = pick_light(S, u0);
    const D3 L = light_point(S.trid[S.light_tri[li]], u1, u2, u3);
    if (STORE_L) sp.put3(kSpL + 3 * k, L);
#if PT_SETUP_REUSE
    // |L - P|^2 once: squared_dist(P, L) sums the same squares in the same
    // order as unit()'s dot (dx = P - L only flips the signs the squares drop,
    // and 0 + x^2 is x^2), so both uses get the same bits
    const D3 a = L - P;
    const double s2 = dot(a, a);
    const D3 dn = a * rsqrt_d(s2);                // main.py:37-38 (unit())
    const float tl = sqrtf((float)s2);            // main.py:40, to ~2e-7
#else
    const D3 dn = unit(L - P);                    // main.py:37-38
    const float tl = sqrtf((float)squared_dist(P, L));   // main.py:40, to ~2e-7
#endif
    sh->hlo[k] = tl * (1.0f - 1e-6f);
    sh->hhi[k] = tl * (1.0f + 1e-6f);
    sh->d32[k] = to_f3(dn);
    sh->ln[k] = dot(dn, n);
    sh->occ[k] = false;
    sh->first[k] = S.n_tri;
}
template <bool COUNT>
PT_HD void shadow_setup(const SceneK& S, D3 P, D3 n, const double u[12], ShadowSet* sh,
                        const Spill& sp) {
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k)
        shadow_setup_k<COUNT>(S, P, n, k, u[4 * k], u[4 * k + 1], u[4 * k + 2], u[4 * k + 3], sh, sp);
    sh->key2 = COUNT ? S.n_tri : S.n_obj;
    sh->leak = S.n_obj - 1;
}
// light sample k of the path's current bounce drawn again from its RNG key,
// with shadow_setup_k's operations (bit for bit its L)
PT_HD D3 light_redraw(const SceneK& S, uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t b, int k) {
#if defined(__HIP_DEVICE_COMPILE__)
    // (the launch's seed, the same in every lane: rng_block keys from SGPRs)
    seed = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(seed >> 32)) << 32) |
           (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)seed);
#endif
    uint32_t c[4];
    rng_block(seed, pixel, sample, b, (uint32_t)k, c);
    const int li = pick_light(S, u_of(c[0]));
    return light_point(S.trid[S.light_tri[li]], u_of(c[1]), u_of(c[2]), u_of(c[3]));
}
// the wavefront record's RNG key in its light-point slots (written once per
// slot, k_wf_shade step 0): the seed, pixel | sample0 << 32, the sample stride;
// the sample index and the bounce are the record's si and sb, just below
// the home (offsets checked in pt_wavefront.h).  sp: a wavefront home only.
PT_HD D3 wf_light(const SceneK& S, const Spill& sp, int k) {
#if !defined(__HIP_DEVICE_COMPILE__)
    assert(sp.stride == 1 && "wf_light: a wavefront path record's home (stride 1) only");
#endif
    const double* base = sp.base;
    uint64_t w0, w1, w2;
    const double d0 = sp.get(kSpL), d1 = sp.get(kSpL + 1), d2 = sp.get(kSpL + 2);
    __builtin_memcpy(&w0, &d0, 8);
    __builtin_memcpy(&w1, &d1, 8);
    __builtin_memcpy(&w2, &d2, 8);
    const int32_t si = reinterpret_cast<const int32_t*>(base)[-2];
    const uint32_t sb = reinterpret_cast<const uint32_t*>(base)[-1];
    const uint32_t sample = (uint32_t)((int32_t)(w1 >> 32) + si * (int32_t)w2);
    return light_redraw(S, w0, (uint32_t)w1, sample, sb >> 3, k);
}

// Shadow rays of the uniform (scene-order) loop with the filter verdicts as
// float margins in VGPRs rather than lane masks: cand iff
// min(cm, m - del) > 0, ambiguous iff min3(nm, m + del, -cand) >= 0 (cm, nm:
// the plane part's candidate / not-miss margins), occlusion a running max
// (> 0: occluded).  Same verdicts as classify_tri (boundary cases lean to
// "ambiguous"), fewer SGPRs and scalar ops.  Render kernel only (not count
// mode, not forced f64); ambiguous tests go to the same f64 block.
#ifndef PT_MARGIN
#define PT_MARGIN 1
#endif
#ifndef PT_QUAD
#define PT_QUAD 1
#endif
// (Round 3's light-side cull and closest-skip experiments, both exact and
// both slower, and their skip counters are no longer in the product; the
// code is at commit 38ea783, DESIGN.md §11 has the measurements.)
#ifndef PT_RNG_PERBLOCK
#define PT_RNG_PERBLOCK 1
#endif
// The candidate margins propagate NaN (v_minimum: a NaN compare is "not a
// candidate" in classify_tri); the ambiguity margins drop it (fminf: a NaN
// compare is "not certainly out").
PT_HD float nan_min(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_elementwise_minimum(a, b);
#else
    return (a != a || b != b) ? NAN : fminf(a, b);
#endif
}
// plane part: cm > 0 iff the range test is certain (rcand), nm >= 0 unless
// it certainly fails (rmiss, boundary leaning to "not a miss"); cop = -1 for
// a coplanar unit (certain miss), else +inf
PT_HD void margin_plane(const UnitF& U, const RayPlane& p, float hi_lo, float hi_hi, float cop,
                        float* cm, float* nm) {
    const float lo = p.at - p.dt, hi = p.at + p.dt;
    *cm = nan_min(nan_min(fabsf(p.q) - U.qhi, lo - kTzHi), nan_min(hi_lo - hi, cop));
    *nm = fminf(fminf(hi - kTzLo, hi_hi - lo), cop);
}
// a test's margins from its weight minimum m
PT_HD void margin_m(float m, const RayPlane& p, float cm, float nm, float* c, float* a) {
    *c = nan_min(cm, m - p.del);
    *a = fminf(fminf(nm, m + p.del), -*c);
}
PT_HD void margin_tri(const TriB& B, const RayPlane& p, float bo, float co, F3 d, float cm,
                      float nm, float* c, float* a) {
    const float beta = fmaf(p.t, lin3(B.gb, d), bo);
    const float gam = fmaf(p.t, lin3(B.gc, d), co);
    margin_m(min3f(beta, gam, (1.0f - beta) - gam), p, cm, nm, c, a);
}

// The render loop's form of a uniform unit (pt_prepare.h: U.quad 1 a
// parallelogram pair, 0 a single triangle, -1 any other coplanar pair): the
// first member's weights (beta, gamma, 1 - s), s = beta + gamma, and for a
// parallelogram the second member's from the same forms, (s, 1 - gamma,
// -beta) — each one rounding of an exact combination of the computed beta
// and gamma, so the unit's del (twice a form's error bound, 16u absolute
// slack included) covers them.  A single triangle's second test is a certain
// miss (m1 = -inf: negative margins, never ambiguous); another pair uses the
// second member's own forms.  Parallelograms skip the second member's forms:
// its origin terms and 8 VALU per ray.
struct QuadM { float m0, m1; };
PT_HD QuadM quad_m(const UnitF& U, const RayPlane& p, const OriginU& O, F3 d) {
    const float beta = fmaf(p.t, lin3(U.tri[0].gb, d), O.bo0);
    const float gam = fmaf(p.t, lin3(U.tri[0].gc, d), O.co0);
    const float s = beta + gam;
    QuadM r;
    r.m0 = min3f(beta, gam, 1.0f - s);
    r.m1 = -INFINITY;
    if (U.quad > 0) {   // wave-uniform
        r.m1 = min3f(s, 1.0f - gam, -beta);
    } else if (U.quad < 0) {
        const float b1 = fmaf(p.t, lin3(U.tri[1].gb, d), O.bo1);
        const float g1 = fmaf(p.t, lin3(U.tri[1].gc, d), O.co1);
        r.m1 = min3f(b1, g1, (1.0f - b1) - g1);
    }
    return r;
}
#ifndef PT_MICRO
#define PT_MICRO 5
#endif
// origin terms of the render loop's unit form (the second member's only for
// a pair that is no parallelogram), and (PT_VCONST) VGPR copies of the
// record's eh and eo for ray_plane_e
#ifndef PT_VCONST
#define PT_VCONST 1
#endif
PT_HD OriginU origin_q(const UnitF& U, F3 o) {
    OriginU r;
    r.eh = U.eh;
    r.eo = U.eo;
#if PT_VCONST && defined(__HIP_DEVICE_COMPILE__)
    asm("" : "+v"(r.eh), "+v"(r.eo));   // (pure: once per unit, no side effects)
#endif
    r.h = aff3(U.n, U.cn, o);
    r.bo0 = aff3(U.tri[0].gb, U.tri[0].cb, o);
    r.co0 = aff3(U.tri[0].gc, U.tri[0].cc, o);
#if PT_MICRO >= 6 && defined(__HIP_DEVICE_COMPILE__)
    // (6) bo1 / co1 are read only under U.quad < 0 (quad_m), where they are
    // set: no zero default (two v_mov per unit for the phi)
    r.bo1 = r.bo0;   // (any value: unread unless overwritten below)
    r.co1 = r.co0;
#else
    r.bo1 = r.co1 = 0.f;
#endif
    if (U.quad < 0) {   // wave-uniform
#if PT_MICRO >= 2 && defined(__HIP_DEVICE_COMPILE__)
        // (3) an opaque copy of the origin: the compiler otherwise computes
        // these two forms for every unit (speculated out of the branch)
        F3 oo = o;
        asm("" : "+v"(oo.x), "+v"(oo.y), "+v"(oo.z));
        r.bo1 = aff3(U.tri[1].gb, U.tri[1].cb, oo);
        r.co1 = aff3(U.tri[1].gc, U.tri[1].cc, oo);
#else
        r.bo1 = aff3(U.tri[1].gb, U.tri[1].cb, o);
        r.co1 = aff3(U.tri[1].gc, U.tri[1].cc, o);
#endif
    }
    return r;
}
// PT_AMB_MAX: the shadow rays' ambiguity is kept as one running maximum per
// lane and unit (amax >= 0: some test needs f64) instead of per-test bits —
// one v_max3 per ray instead of six bit-packing instructions; the rare block
// rebuilds the bits (shadow_bits_m)
#ifndef PT_AMB_MAX
#define PT_AMB_MAX 1
#endif
// PT_MICRO: (1) cop canonicalised once per unit, so the margins built from
// it need no per-ray canonicalisation before fminf (IEEE mode), (2) the
// ambiguity maximum taken before the occlusion margin is overwritten (no
// register copy of the loop-carried margin), (3) origin_q above.  Same values.
PT_HD float pt_canon(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_canonicalizef(x);
#else
    return x;
#endif
}
// PT_MMERGE: a shadow ray's two member tests of a unit as ONE pair of margins.
// Both members share the plane part (cm, nm, del), and a shadow ray only asks
// whether the unit occludes it (both members are one object), so with
// M = max(m0, m1):
//   c = min(cm, M - del) > 0   iff some member is a certain occluder
//                              (c_i = min(cm, m_i - del) > 0 for M's member)
//   a = min(nm, M + del, -c)   >= 0 whenever some member's test is ambiguous
//                              and no member occludes for certain
// (margin_unit; if one member occludes for certain, the other's ambiguity
// decides nothing: rays 0, 1 are occluded, ray 2's object is this unit's).
// For rays 0, 1 the "not occluded before this unit" term folds in as
// -max(old, c), the new occlusion margin.  The rare block rebuilds the
// per-member bits as before (shadow_bits_m), so the f64 decisions are the
// same ones; hostcheck's filter self-test checks both claims test by test.
#ifndef PT_MMERGE
#define PT_MMERGE 1
#endif
#ifndef PT_CLOSEST_LEAN
#define PT_CLOSEST_LEAN 1
#endif
#ifndef PT_DEL_PRE
#define PT_DEL_PRE 1
#endif
#ifndef PT_VOTE_MIN3
#define PT_VOTE_MIN3 1
#endif
#ifndef PT_LIGHT_QUAD
#define PT_LIGHT_QUAD 1
#endif
#ifndef PT_CADD_BF
#define PT_CADD_BF 1
#endif
PT_HD void margin_unit(float cm, float nm, float M, float del, float* c, float* a) {
    *c = nan_min(cm, M - del);
    *a = fminf(fminf(nm, M + del), -*c);
}
// fmaxf of two quiet-NaN-or-number values without the canonicalising
// v_max_f32 x, x the compiler puts before an IEEE-mode v_max_f32 whose input
// comes through a phi: the instruction itself (IEEE maxNum: a quiet NaN
// operand returns the other one, as fmaxf does).  The values here come from
// arithmetic (quiet NaNs only).  (A v_med3_f32(a, b, FLT_MAX) form avoids the
// asm's s_nop but costs an SGPR: 0.5% slower)
PT_HD float fmax_q(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return fmaxf(a, b);
#endif
}
PT_HD float fmin_q(float a, float b) {   // fminf likewise (IEEE minNum of quiet NaNs or numbers)
#if defined(__HIP_DEVICE_COMPILE__)
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return fminf(a, b);
#endif
}
// nan_min(nan_min(a, b), c) as one v_minimum3_f32 (the compiler emits each
// two-input minimum as its own v_minimum3_f32 with a repeated operand)
PT_HD float nan_min3(float a, float b, float c) {
#if defined(__HIP_DEVICE_COMPILE__)
    float r;
    asm("v_minimum3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return nan_min(nan_min(a, b), c);
#endif
}
PT_HD void shadow_unit_m(const SceneK& S, const UnitF& U, const OriginU& O, bool coplanar,
                         ShadowSet* sh, float oc[kLightSamples], uint32_t* amb, float* amax = nullptr) {
    const float cop = PT_MICRO ? pt_canon(coplanar ? -1.0f : INFINITY) : (coplanar ? -1.0f : INFINITY);
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) {
        const F3 d = sh->d32[k];
#if PT_DEL_PRE && defined(__HIP_DEVICE_COMPILE__)
        const RayPlane p0 = ray_plane_e(U, O.h, d, sh->hlo[k], sh->hhi[k], O.eh, O.eo);
        const RayPlane& p = p0;
#else
        const RayPlane p = ray_plane_e(U, O.h, d, sh->hlo[k], sh->hhi[k], O.eh, O.eo);
#endif
        float cm, nm;
        margin_plane(U, p, sh->hlo[k], sh->hhi[k], cop, &cm, &nm);
        // nm < 0 (the plane part is a certain miss; nm is never NaN, cop is
        // not) implies cm < 0, so every margin of the ray's triangles is
        // negative or a dropped NaN: no occlusion, no ambiguous test.  The
        // triangle part only runs when some lane of the wave is not
        // certainly out of range (K2 6.49 -> 6.35 ms).
#if PT_QUAD && PT_MMERGE && PT_MICRO >= 5
        // (5) ray 0 comes first and *amax enters at -1, only its sign is
        // read: when the wave skips the ray every lane's nm is < 0 (never
        // NaN), so nm serves as the "nothing ambiguous" value — no -1.0
        // constant materialised for the skip edge
        if (k == 0 && PT_AMB_MAX && amax) *amax = nm;
#endif
#if PT_DEL_PRE && defined(__HIP_DEVICE_COMPILE__)
        // (dev) del's |t| ed + eo term before the vote, where |t| is a source
        // modifier (after the branch the compiler materialises |t| with a v_and)
        float ye = fmaf(p.at, U.ed, O.eo);
        asm("" : "+v"(ye));
#endif
        if (!PT_WAVE_ANY(!(nm < 0.0f))) continue;
#if PT_QUAD && PT_MMERGE
        if (PT_AMB_MAX && amax) {
#if PT_DEL_PRE && defined(__HIP_DEVICE_COMPILE__)
            RayPlane p = p0;
            p.del = fmaf(U.g, p.dt, ye);
#endif
            const QuadM m = quad_m(U, p, O, d);
            const float M = fmax_q(m.m0, m.m1);
            const float old = oc[k];
            // c = min(cm, M - del), cm's five terms in two v_minimum3
            const float c = nan_min3(nan_min3(fabsf(p.q) - U.qhi, (p.at - p.dt) - kTzHi,
                                              sh->hlo[k] - (p.at + p.dt)),
                                     cop, M - p.del);
            if (k == kLightSamples - 1) {
                const bool need = U.obj < sh->key2;
                if (c > 0.0f && need) {
                    sh->key2 = U.obj;
                    sh->leak = U.obj;
                }
                *amax = fmax_q(*amax, need ? fminf(fminf(nm, M + p.del), -c) : -1.0f);
                oc[k] = fmax_q(old, c);
            } else {   // only while not occluded before this unit: -max(old, c)
                const float occ = fmax_q(old, c);
                const float a = fminf(fminf(nm, M + p.del), -occ);   // (never NaN: nm is not)
                // ray 0 comes first and *amax enters at -1: only its sign is read
                *amax = k == 0 ? a : fmax_q(*amax, a);
                oc[k] = occ;
            }
            continue;
        }
#endif
#if PT_QUAD
        const QuadM m = quad_m(U, p, O, d);
        float c0, a0, c1, a1;
        margin_m(m.m0, p, cm, nm, &c0, &a0);
        margin_m(m.m1, p, cm, nm, &c1, &a1);
#else
        float c0, a0, c1 = -INFINITY, a1 = -INFINITY;
        margin_tri(U.tri[0], p, O.bo0, O.co0, d, cm, nm, &c0, &a0);
        if (U.count == 2) margin_tri(U.tri[1], p, O.bo1, O.co1, d, cm, nm, &c1, &a1);
#endif
        const float old = oc[k];
        const float c = fmaxf(c0, c1);
        if (!PT_MICRO) oc[k] = fmaxf(old, c);
        if (k == kLightSamples - 1) {
            const bool need = U.obj < sh->key2;
            if (c > 0.0f && need) {
                sh->key2 = U.obj;
                sh->leak = U.obj;
            }
            if (PT_AMB_MAX && amax) *amax = fmaxf(*amax, need ? fmaxf(a0, a1) : -1.0f);
            else if (need) *amb |= (a0 >= 0.0f ? 1u : 0u) << (2 * k) | (a1 >= 0.0f ? 2u : 0u) << (2 * k);
        } else if (PT_AMB_MAX && amax) {   // only while not occluded before this unit
            *amax = fmaxf(*amax, fmaxf(fminf(a0, -old), fminf(a1, -old)));
        } else {   // only while not occluded before this unit
            *amb |= (fminf(a0, -old) >= 0.0f ? 1u : 0u) << (2 * k) |
                    (fminf(a1, -old) >= 0.0f ? 2u : 0u) << (2 * k);
        }
        if (PT_MICRO) oc[k] = fmaxf(old, c);
    }
}
// The shadow bits of shadow_unit_m rebuilt after the unit (PT_AMB_MAX, the
// rare path; no vote).  oc and key2 are already updated by this unit: a ray it
// occluded for certain gets no bits here where shadow_unit_m set some, and the
// f64 block would skip those ("decided meanwhile"), so the decisions are the
// same.
PT_HD uint32_t shadow_bits_m(const SceneK& S, const UnitF& U, const OriginU& O, bool coplanar,
                             const ShadowSet* sh, const float oc[kLightSamples]) {
    const float cop = coplanar ? -1.0f : INFINITY;
    uint32_t amb = 0;
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) {
        const F3 d = sh->d32[k];
        const RayPlane p = ray_plane(U, O.h, d, sh->hlo[k], sh->hhi[k]);
        float cm, nm;
        margin_plane(U, p, sh->hlo[k], sh->hhi[k], cop, &cm, &nm);
        if (nm < 0.0f) continue;   // every margin negative: no ambiguous test
        const QuadM m = quad_m(U, p, O, d);
        float c0, a0, c1, a1;
        margin_m(m.m0, p, cm, nm, &c0, &a0);
        margin_m(m.m1, p, cm, nm, &c1, &a1);
        if (k == kLightSamples - 1) {
            if (U.obj < sh->key2) amb |= (a0 >= 0.0f ? 1u : 0u) << (2 * k) | (a1 >= 0.0f ? 2u : 0u) << (2 * k);
        } else {
            amb |= (fminf(a0, -oc[k]) >= 0.0f ? 1u : 0u) << (2 * k) |
                   (fminf(a1, -oc[k]) >= 0.0f ? 2u : 0u) << (2 * k);
        }
    }
    return amb;
}

// The f64 decisions of a unit's ambiguous tests (bits of amb, see
// fused_unit): one rare block per unit (an eval64 per bit), entered by few
// waves.
template <bool FORCE64, bool COUNT, bool MARGIN, int PARTS = 3, bool LRNG = false>
PT_HD void fused_fallback(const SceneK& S, const UnitF& U, uint32_t amb, ShadowSet* sh,
                          ClosestAcc* ca, const Spill& sp, Counters* cnt, float* oc) {
    const D3 P = sp.get3(kSpP);
    for (int k = 0; k < ((PARTS & 1) ? kLightSamples : 0); ++k) {
        for (int i = 0; i < 2; ++i) {
            if (!((amb >> (2 * k + i)) & 1u)) continue;
            const int t = U.t[i];
            // decided meanwhile (a lower occluder of this unit, or occlusion)?
            if (k == kLightSamples - 1 ? ((COUNT ? t : U.obj) >= sh->key2)
                                       : (COUNT ? (t >= sh->first[k])
                                                : (MARGIN ? oc[k] > 0.0f : sh->occ[k])))
                continue;
            D3 Q;
            double sqd;
            if (!FORCE64) bump<COUNT>(cnt, &Counters::fallbacks, 1);
            const D3 L = LRNG ? wf_light(S, sp, k) : sp.get3(kSpL + 3 * k);
            if (eval64(S.trid[t], P, unit(L - P), &Q, &sqd) && !(sqd < kZero) &&
                sqd < squared_dist(P, L)) {
                if (COUNT && t < sh->first[k]) sh->first[k] = t;
                if (k == kLightSamples - 1) {
                    sh->key2 = COUNT ? t : U.obj;
                    sh->leak = U.obj;
                }
                if (MARGIN) oc[k] = 1.0f;
                else sh->occ[k] = true;
            }
        }
    }
    for (int i = 0; i < ((PARTS & 2) ? 2 : 0); ++i) {
        if (!((amb >> (6 + i)) & 1u)) continue;
        const int t = U.t[i];
        D3 Q;
        double sqd;
        bump<COUNT>(cnt, &Counters::fallbacks, 1);
        float a = INFINITY, b = INFINITY;
        if (eval64(S.trid[t], P, unit(sp.get3(kSpNd)), &Q, &sqd) && sqd > kZero) {
            const float sq = sqrtf((float)sqd);   // |t| to ~1e-7; brackets are 1e-6
            a = sq * (1.0f - 1e-6f);
            b = sq * (1.0f + 1e-6f);
        }
        closest_add(ca, t, a, b);
    }
}

// The next ray's closest-hit test against a uniform unit in the render
// loop's unit form (quad_m): per-member verdicts as lane masks, the candidate
// into ca, the ambiguous members as bits 6 / 7 of *amb.
PT_HD void closest_unit_m(const UnitF& U, const OriginU& O, bool coplanar, F3 n32, ClosestAcc* ca,
                          uint32_t* amb) {
    RayPlane p = ray_plane_e(U, O.h, n32, INFINITY, INFINITY, O.eh, O.eo);
#if PT_CLOSEST_LEAN
    // the closest ray's range has no far end (hi_lo = hi_hi = inf): rcand's
    // "at + dt < inf" follows from |q| > qhi (>= 1e-5: |t| <= |h| 1e5 (1 + u),
    // dt finite, for the finite origins and records here), and rmiss's
    // "at - dt >= inf" only holds for |t| = inf (q exactly 0), which is then
    // ambiguous (del = inf) and decided in f64 — two compares less per unit,
    // the same certain verdicts
    p.rcand = (fabsf(p.q) > U.qhi) & (p.at - p.dt > kTzHi);
    p.rmiss = p.at + p.dt < kTzLo;
#endif
    const QuadM m = quad_m(U, p, O, n32);
    const Verdict v0 = verdict_m(m.m0, p), v1 = verdict_m(m.m1, p);
    const bool c0 = v0.cand & !coplanar, a0 = v0.amb & !coplanar;
    const bool c1 = v1.cand & !coplanar, a1 = v1.amb & !coplanar;
    // both candidates of one unit cannot happen (a point certainly inside
    // one triangle is certainly outside its coplanar neighbour)
    const bool c = c0 | c1;
#if PT_CADD_BF
    // closest_add branch-free, the running minimum as an asm v_min_f32 (no
    // canonicalising v_max x, x of its phi inputs; a and a2 are never NaN)
    const float a = c ? p.at - p.dt : INFINITY, b = c ? p.at + p.dt : INFINITY;
    const int tc = c0 ? U.t[0] : U.t[1];
    const bool lt = a < ca->a1;
    ca->a2 = lt ? ca->a1 : fmin_q(ca->a2, a);
    ca->a1 = lt ? a : ca->a1;
    ca->b1 = lt ? b : ca->b1;
    ca->i1 = lt ? tc : ca->i1;
#else
    closest_add(ca, c0 ? U.t[0] : U.t[1], c ? p.at - p.dt : INFINITY, c ? p.at + p.dt : INFINITY);
#endif
    *amb |= (a0 ? 64u : 0u) | (a1 ? 128u : 0u);
}

// One plane unit against the 3 shadow rays and the next ray's closest hit,
// all from the same origin (the fused per-bounce pass).  Every verdict is
// computed branch-free; ambiguous tests are only recorded as bits and
// decided in f64 in one (rare) block per unit, so the common path carries no
// per-test exec-mask juggling.  Scene order is kept where it matters: for
// each shadow ray the lowest occluding triangle index is tracked, so the
// leaked colour of main.py:70 (object of the first occluder in scene order)
// does not depend on the order units are visited in.
// PARTS: bit 0 the shadow rays, bit 1 the closest ray can be present at this
// call site (the walks' leaves test one kind only: the other kind's code,
// its f64 block included, is then not compiled in — the closest walk
// kernel ran 21% faster without the dead shadow block)
template <bool FORCE64, bool COUNT, bool MARGIN = false, int PARTS = 3, bool LRNG = false>
PT_HD void fused_unit(const SceneK& S, const UnitF& U, const OriginU& O, bool coplanar,
                      bool do_shadow, bool do_closest, ShadowSet* sh, F3 n32, ClosestAcc* ca,
                      const Spill& sp, Counters* cnt, uint32_t rays = 15u,
                      float* oc = nullptr) {
    if (!(PARTS & 1)) do_shadow = false;
    if (!(PARTS & 2)) do_closest = false;
    // rays: bit k = shadow ray k, bit 3 = the closest ray (the BVH passes the
    // lines that reached the leaf's box; a line that did not cannot hit)
    uint32_t amb = 0;   // bit 2k+i: shadow ray k / triangle i; bit 6+i: closest / triangle i
    const bool two = (U.count == 2);
    float amax = -1.0f;   // PT_AMB_MAX: >= 0 when some shadow test of the unit is ambiguous
    if (MARGIN) {   // the render loop's uniform units (oc: occlusion margins)
        if (do_shadow) shadow_unit_m(S, U, O, coplanar, sh, oc, &amb, PT_QUAD ? &amax : nullptr);
    } else if (do_shadow) {   // (sh is only touched here and for shadow bits: null without shadows)
        bool occ0[kLightSamples];
#pragma unroll
        for (int k = 0; k < kLightSamples; ++k) occ0[k] = sh->occ[k];
#pragma unroll
        for (int k = 0; k < kLightSamples; ++k) {
            if (!((rays >> k) & 1u)) continue;
            bool c0 = false, c1 = false, a0 = true, a1 = two;
            if (!FORCE64) {
                const RayPlane p = ray_plane(U, O.h, sh->d32[k], sh->hlo[k], sh->hhi[k]);
                const Verdict v0 = classify_tri(U.tri[0], p, O.bo0, O.co0, sh->d32[k]);
                c0 = v0.cand & !coplanar;
                a0 = v0.amb & !coplanar;
                a1 = false;
                if (two) {   // wave-uniform
                    const Verdict v1 = classify_tri(U.tri[1], p, O.bo1, O.co1, sh->d32[k]);
                    c1 = v1.cand & !coplanar;
                    a1 = v1.amb & !coplanar;
                }
            }
            // which ambiguous tests still matter: rays 0, 1 until occluded (count
            // mode: until their lowest occluder is known), the last ray until
            // its lowest occluder is known (the leaked colour).  Units may come
            // in any order (the BVH), so "first" is the lowest triangle index.
            const int t0 = U.t[0];
            const bool need = (k == kLightSamples - 1) ? ((COUNT ? t0 : U.obj) < sh->key2)
                              : (COUNT ? (t0 < sh->first[k]) : !occ0[k]);
            const bool c = c0 | c1;
            const int tc = c0 ? t0 : U.t[1];
            if (COUNT && c && tc < sh->first[k]) sh->first[k] = tc;
            if (k == kLightSamples - 1 && c && (COUNT ? tc : U.obj) < sh->key2) {
                sh->key2 = COUNT ? tc : U.obj;
                sh->leak = U.obj;
            }
            sh->occ[k] = occ0[k] | c;
            if (need) amb |= (a0 ? 1u : 0u) << (2 * k) | (a1 ? 2u : 0u) << (2 * k);
        }
    }
    if (!FORCE64 && do_closest && (rays & 8u)) {
        if (MARGIN && PT_QUAD) {   // the render loop's unit form (quad_m)
            closest_unit_m(U, O, coplanar, n32, ca, &amb);
        } else {
            const RayPlane p = ray_plane(U, O.h, n32, INFINITY, INFINITY);
            bool c1 = false, a1 = false;
            const Verdict v0 = classify_tri(U.tri[0], p, O.bo0, O.co0, n32);
            const bool c0 = v0.cand & !coplanar;
            const bool a0 = v0.amb & !coplanar;
            if (two) {
                const Verdict v1 = classify_tri(U.tri[1], p, O.bo1, O.co1, n32);
                c1 = v1.cand & !coplanar;
                a1 = v1.amb & !coplanar;
            }
            // both candidates of one unit cannot happen (a point certainly inside
            // one triangle is certainly outside its coplanar neighbour)
            const bool c = c0 | c1;
            closest_add(ca, c0 ? U.t[0] : U.t[1], c ? p.at - p.dt : INFINITY,
                        c ? p.at + p.dt : INFINITY);
            amb |= (a0 ? 64u : 0u) | (a1 ? 128u : 0u);
        }
    }
    if (PT_AMB_MAX && MARGIN && PT_QUAD && (PARTS & 1) && !(amax < 0.0f))   // rare: rebuild the bits
        amb |= shadow_bits_m(S, U, O, coplanar, sh, oc);
    amb &= ((PARTS & 1) ? 0x3fu : 0u) | ((PARTS & 2) ? 0xc0u : 0u);
    if (amb) fused_fallback<FORCE64, COUNT, MARGIN, PARTS, LRNG>(S, U, amb, sh, ca, sp, cnt, oc);   // rare (FORCE64: every shadow test) — decide in f64
}

template <bool COUNT>
PT_HD D3 shadow_color(const SceneK& S, int obj, const ShadowSet& sh, Counters* cnt) {
    double dsum = 0.0;
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) {
        if (!sh.occ[k]) dsum += sh.ln[k];   // main.py:66-68
        // the reference's loop stops at the first occluder (main.py:42-55)
        bump<COUNT>(cnt, &Counters::shadow_tests,
                    (uint32_t)(sh.first[k] < S.n_tri ? sh.first[k] + 1 : S.n_obj_tri));
    }
    dsum /= (double)kLightSamples;
    const Mat& m = S.mat[obj];
    const Mat& lm = S.mat[sh.leak];   // main.py:70
    bump<COUNT>(cnt, &Counters::shading_points, 1);
    // m.rgb * m.ka * S.ambient + S.light_rgb * lm.rgb * dsum, the two
    // products precomputed per object (Mat::amb, Mat::lrgb)
    return d3(m.amb[0] + lm.lrgb[0] * dsum, m.amb[1] + lm.lrgb[1] * dsum, m.amb[2] + lm.lrgb[2] * dsum);
}

// ------------------------------------------------------------------ BVH --
// Large meshes (SceneK::bnode/bunit, built in pt_prepare.h).  One stackless
// traversal per lane and bounce serves all four lines of the fused pass: a
// node is entered when one of them meets its box within its range (shadow
// ray k: |t| <= hhi[k]; the closest ray: |t| <= the current best's upper
// bound), and its leaf units go through fused_unit like the uniform ones.
// Shadow rays still open for the BVH: 0, 1 until occluded (count mode:
// until no BVH triangle can be their lowest occluder); the last ray until no
// BVH object can be its first occluder's.  Bit k: ray k.
template <bool COUNT>
PT_HD uint32_t shadow_open(const SceneK& S, const ShadowSet* sh) {
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) {
        const bool open = (k == kLightSamples - 1)
                              ? (sh->key2 > (COUNT ? S.bvh_min_tri : S.bvh_min_obj))
                              : (COUNT ? (sh->first[k] > S.bvh_min_tri) : !sh->occ[k]);
        m |= open ? 1u << k : 0u;
    }
    return m;
}

template <bool FORCE64, bool COUNT>
PT_HD void bvh_pass(const SceneK& S, F3 o32, int ogrp, bool do_shadow, bool do_closest,
                    ShadowSet* sh, F3 n32, ClosestAcc* ca, const Spill& sp, Counters* cnt) {
    F3 inv[kLightSamples];
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) inv[k] = rcp_dir(sh->d32[k]);
    const F3 invc = rcp_dir(n32);
    // "while-while": each lane walks internal nodes on its own until it finds
    // a leaf its lines reach, then the lanes test their leaves together
    int node = (do_shadow || do_closest) ? 0 : -1;
    BNode N = S.bnode[0];
    while (node >= 0) {
        int leaf = -1;
        uint32_t leaf_rays = 0;
        while (node >= 0) {
            // both possible successors are fetched while this node is tested,
            // so the walk waits on one load per step, overlapped with the test
            const int na = node + 1 < S.n_bnode ? node + 1 : node;
            const int nb = N.skip >= 0 ? N.skip : node;
            const BNode A = S.bnode[na];
            const BNode B = S.bnode[nb];
            const F3 l = {N.lo[0] - o32.x, N.lo[1] - o32.y, N.lo[2] - o32.z};
            const F3 h = {N.hi[0] - o32.x, N.hi[1] - o32.y, N.hi[2] - o32.z};
            uint32_t rays = 0;
            if (do_shadow) {
                const uint32_t open = shadow_open<COUNT>(S, sh);
#pragma unroll
                for (int k = 0; k < kLightSamples; ++k)
                    if (((open >> k) & 1u) && box_hit(l, h, inv[k], sh->hhi[k])) rays |= 1u << k;
            }
            if (do_closest && box_hit(l, h, invc, ca->b1)) rays |= 8u;
            if (rays && N.leaf >= 0) {
                leaf = N.leaf;
                leaf_rays = rays;
                node = N.skip;
                N = B;
                break;
            }
            const bool down = rays != 0;   // (a leaf's skip is node + 1: A == B)
            node = down ? node + 1 : N.skip;
            N = down ? A : B;
        }
        if (leaf >= 0) {
            const int u0 = leaf >> 3, nu = leaf & 7;
            for (int i = 0; i < nu; ++i) {
                const UnitF U = S.bunit[u0 + i];
                const OriginU O = FORCE64 ? OriginU{0.f, 0.f, 0.f, 0.f, 0.f} : origin_u(U, o32);
                fused_unit<FORCE64, COUNT>(S, U, O, U.grp == ogrp, do_shadow, do_closest, sh, n32,
                                           ca, sp, cnt, leaf_rays);
            }
        }
    }
}

// The closest ray alone, nearest box first (by the smallest |t| of the line
// inside it: the line is two-sided), with a per-lane stack of the farther
// children; a popped node is dropped when its distance exceeds the bound the
// candidates found meanwhile give (the best's upper |t|).
constexpr int kBvhStack = 48;
PT_HD float box_dist(F3 l, F3 h, F3 inv, float R) {   // INFINITY: not within |t| <= R
    const float ax = l.x * inv.x, bx = h.x * inv.x;
    const float ay = l.y * inv.y, by = h.y * inv.y;
    const float az = l.z * inv.z, bz = h.z * inv.z;
    const float tmin = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float tmax = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    // the smallest |t| in [tmin, tmax]; within |t| <= R exactly when <= R
    const float d = fmaxf(fmaxf(tmin, -tmax), 0.0f);
    return ((tmin <= tmax) & (d <= R)) ? d : INFINITY;
}
PT_HD float node_dist(const SceneK& S, int i, F3 o32, F3 inv, float R) {
    const BNode N = S.bnode[i];
    const F3 l = {N.lo[0] - o32.x, N.lo[1] - o32.y, N.lo[2] - o32.z};
    const F3 h = {N.hi[0] - o32.x, N.hi[1] - o32.y, N.hi[2] - o32.z};
    return box_dist(l, h, inv, R);
}
PT_HD float cbox_dist(const float* lo, const float* hi, F3 o32, F3 inv, float R) {
    const F3 l = {lo[0] - o32.x, lo[1] - o32.y, lo[2] - o32.z};
    const F3 h = {hi[0] - o32.x, hi[1] - o32.y, hi[2] - o32.z};
    return box_dist(l, h, inv, R);
}
// The ordered traversals are resumable: a traversal object holds the walk's
// state and step() runs one "while-while" round (walk internal nodes to the
// next leaf its lines reach, test that leaf, pop the next entry).  The
// single-kernel path runs a traversal to completion in place; the wavefront
// query kernels (pt_wavefront.h) keep one per lane and refill a lane with the
// next query as soon as its traversal ends.
//
// Per-lane stack (scratch) with its top entry cached in registers: a pop
// takes the cached entry and starts the refill load, whose result is only
// needed at the next pop.
struct ClosestTrav {
    F3 o32, d32, inv;
    int ogrp;
    int ref;                  // next node / leaf (<= -2: leaf code; kNoRef: done)
    int top;                  // entries in the scratch part
    int tref;                 // cached top (kNoRef: empty)
    float tdist;
};
// The stack arrays live outside the traversal object (a local array indexed
// at run time is scratch memory; inside the object it would drag the whole
// object — origin, inverse direction — to scratch with it).  ClosestStack is
// a strided view: a per-lane local array (ClosestStackLocal, stride 1) or a
// column of shared-memory arrays (stride = block size; k_wf_closest).
// Entry distances are kept as the upper 16 bits of the f32 (truncation of a
// non-negative float rounds down, so the pop check against the shrinking
// bound is conservative: it may visit a node the exact distance would skip,
// never the reverse).
// PT_LDS: the walk kernels' stacks live in shared memory.  Their views name
// that address space, so pushes and pops compile to LDS instructions: through
// generic pointers the compiler merged each LDS store with its rare global
// overflow store into one flat store on a selected address.
#if defined(__HIP_DEVICE_COMPILE__)
#define PT_LDS __attribute__((address_space(3)))
#else
#define PT_LDS
#endif
template <class R, class D>   // R: int* / PT_LDS int*, D: uint16_t* / PT_LDS uint16_t*
struct ClosestStackT {
    R ref;
    D dist;
    int stride;
    // the walk kernels keep the first nl entries in LDS (ref / dist, stride
    // `stride`) and the deeper ones, rarely touched, in global memory (gref /
    // gdist, stride gs)
    int* gref = nullptr;
    uint16_t* gdist = nullptr;
    int gs = 0;
    int nl = 1 << 30;
    PT_HD void set(int i, int r, uint16_t d) const {
        if (i < nl) { ref[i * stride] = r; dist[i * stride] = d; }
        else { gref[(i - nl) * gs] = r; gdist[(i - nl) * gs] = d; }
    }
    PT_HD int get_ref(int i) const { return i < nl ? ref[i * stride] : gref[(i - nl) * gs]; }
    PT_HD uint16_t get_dist(int i) const { return i < nl ? dist[i * stride] : gdist[(i - nl) * gs]; }
};
using ClosestStack = ClosestStackT<int*, uint16_t*>;
using ClosestStackLds = ClosestStackT<PT_LDS int*, PT_LDS uint16_t*>;
// (local stacks hold kBvhStack + 2 entries: push3's dead stores reach two
// entries above the deepest live one)
constexpr int kBvhStackLocal = kBvhStack + 2;
struct ClosestStackLocal {
    int ref[kBvhStackLocal];
    uint16_t dist[kBvhStackLocal];
    PT_HD ClosestStack view() { return ClosestStack{ref, dist, 1}; }
};
PT_HD uint16_t dist_down16(float d) {
    uint32_t b;
    memcpy(&b, &d, sizeof b);
    return (uint16_t)(b >> 16);
}
PT_HD float dist_up16(uint16_t h) {
    const uint32_t b = (uint32_t)h << 16;
    float d;
    memcpy(&d, &b, sizeof d);
    return d;
}
// The pushes of a 4-wide node visit (children 3, 2, 1 of the distance order,
// farthest first; v1 >= v2 >= v3 since misses sort last) onto a stack with
// its top entry cached in (tc, td): what ctrav_push does child by child, but
// when the three entries fit below nl as unconditional stores above the top,
// each advancing the top only when its entry is real — no branch per child.
// (Stores at or above the final top are dead entries.)
template <class KS>
PT_HD void push3(const KS& K, int& top, int& tc, float& td, bool v1, bool v2, bool v3, int r1, float d1,
                 int r2, float d2, int r3, float d3) {
    if (top + 3 <= K.nl) {
        int p = top;
        K.ref[p * K.stride] = tc;
        K.dist[p * K.stride] = dist_down16(td);
        p += (v1 && tc != kNoRef) ? 1 : 0;
        K.ref[p * K.stride] = r3;
        K.dist[p * K.stride] = dist_down16(d3);
        p += v3 ? 1 : 0;
        K.ref[p * K.stride] = r2;
        K.dist[p * K.stride] = dist_down16(d2);
        p += v2 ? 1 : 0;
        top = p;
    } else {
        if (v1 && tc != kNoRef) K.set(top++, tc, dist_down16(td));
        if (v3) K.set(top++, r3, dist_down16(d3));
        if (v2) K.set(top++, r2, dist_down16(d2));
    }
    tc = v1 ? r1 : tc;
    td = v1 ? d1 : td;
}
template <class KS>
PT_HD void ctrav_push(ClosestTrav& T, const KS& K, int r, float d) {
    if (T.tref != kNoRef) {
        K.set(T.top, T.tref, dist_down16(T.tdist));
        ++T.top;
    }
    T.tref = r;
    T.tdist = d;
}
template <class KS>
PT_HD int ctrav_pop(ClosestTrav& T, const KS& K, float bound) {   // next node within the bound, or kNoRef
    while (T.tref != kNoRef) {
        const int r = T.tref;
        const float d = T.tdist;
        if (T.top > 0) {
            --T.top;
            T.tref = K.get_ref(T.top);
            T.tdist = dist_up16(K.get_dist(T.top));
        } else {
            T.tref = kNoRef;
        }
        if (d <= bound) return r;
    }
    return kNoRef;
}
// root: S.bvh_root (two-child walk) or S.qroot (4-wide walk)
PT_HD void ctrav_init(ClosestTrav& T, const SceneK& S, F3 o32, int ogrp, F3 d32, float bound,
                      int root) {
    T.o32 = o32;
    T.d32 = d32;
    T.inv = rcp_dir(d32);
    T.ogrp = ogrp;
    T.top = 0;
    T.tref = kNoRef;
    T.tdist = INFINITY;
    T.ref = node_dist(S, 0, o32, T.inv, bound) < INFINITY ? root : kNoRef;
}
// one internal node (T.ref >= 0): nearer child next, the farther stacked
PT_HD void ctrav_node(ClosestTrav& T, const ClosestStack& K, const SceneK& S, const ClosestAcc* ca) {
    const CNode C = S.cnode[T.ref];
    const float d0 = cbox_dist(C.lo0, C.hi0, T.o32, T.inv, ca->b1);
    const float d1 = cbox_dist(C.lo1, C.hi1, T.o32, T.inv, ca->b1);
    const bool near0 = d0 <= d1;
    const float dn = near0 ? d0 : d1, df = near0 ? d1 : d0;
    const int rn = near0 ? C.c0 : C.c1, rf = near0 ? C.c1 : C.c0;
    if (df < INFINITY) ctrav_push(T, K, rf, df);
    T.ref = dn < INFINITY ? rn : ctrav_pop(T, K, ca->b1);
}
// the units of leaf `ref` (<= -2: leaf codes have a unit count >= 1)
// BVH unit i as the walks test it: UC = from the 64-B form (the caller
// checked S.bunitc; a compile-time choice, so only one record is loaded)
PT_HD UnitF unitc_f(const SceneK& S, const UnitC& C) {
    UnitF U;
    U.n[0] = C.n[0]; U.n[1] = C.n[1]; U.n[2] = C.n[2];
    U.cn = C.cn;
    U.eh = bf16_hi(C.eoeh);
    U.eq = S.bvh_eq;
    U.qhi = S.bvh_qhi;
    U.eo = bf16_lo(C.eoeh);
    U.ed = C.g * kEdPerG;
    U.g = C.g;
    U.grp = C.grp;
    U.count = 1;
    U.obj = S.bvh_obj1 >= 0 ? S.bvh_obj1 : S.tri_obj[C.t];
    U.t[0] = U.t[1] = C.t;
    U.quad = 0;   // a single triangle
    U.tri[0] = C.tri;
    U.tri[1] = TriB{};
    return U;
}
template <bool UC>
PT_HD UnitF bvh_unit(const SceneK& S, int i) {
    if (!UC) return S.bunit[i];
    return unitc_f(S, S.bunitc[i]);
}
template <bool COUNT, bool UC = false>
PT_HD void ctrav_units(const ClosestTrav& T, const SceneK& S, ClosestAcc* ca, const Spill& sp,
                       Counters* cnt, int ref) {
    const int code = ~ref, u0 = code >> 3, nu = code & 7;
    for (int i = 0; i < nu; ++i) {
        const UnitF U = bvh_unit<UC>(S, u0 + i);
        fused_unit<false, COUNT, false, 2>(S, U, origin_u(U, T.o32), U.grp == T.ogrp, false, true, nullptr,
                                 T.d32, ca, sp, cnt, 8u);
    }
}
// the leaf T.ref, then the next entry
template <bool COUNT, bool UC = false, class KS = ClosestStack>
PT_HD void ctrav_leaf(ClosestTrav& T, const KS& K, const SceneK& S, ClosestAcc* ca,
                      const Spill& sp, Counters* cnt) {
    ctrav_units<COUNT, UC>(T, S, ca, sp, cnt, T.ref);
    T.ref = ctrav_pop(T, K, ca->b1);
}
// one "while-while" round: walk internal nodes to the next leaf, test it;
// returns true when the traversal has ended
template <bool COUNT>
PT_HD bool ctrav_step(ClosestTrav& T, const ClosestStack& K, const SceneK& S, ClosestAcc* ca,
                      const Spill& sp, Counters* cnt) {
    while (T.ref >= 0) ctrav_node(T, K, S, ca);
    if (T.ref != kNoRef) ctrav_leaf<COUNT>(T, K, S, ca, sp, cnt);
    return T.ref == kNoRef;
}
template <bool COUNT>
PT_HD void bvh_closest(const SceneK& S, F3 o32, int ogrp, F3 d32, ClosestAcc* ca, const Spill& sp,
                       Counters* cnt) {
    ClosestTrav T;
    ClosestStackLocal L;
    const ClosestStack K = L.view();
    ctrav_init(T, S, o32, ogrp, d32, ca->b1, S.bvh_root);
    while (!ctrav_step<COUNT>(T, K, S, ca, sp, cnt)) {
    }
}

// The shadow rays of a bounce, nearest box first (the rays share their
// origin; a box's distance is the smallest |t| of any of its rays in it):
// an occluder near the shading point closes a ray early.  Stack entries are
// (reference << 3 | rays that entered the box); rays closed meanwhile are
// dropped on pop.  Ends when every ray is closed.
struct ShadowTrav {
    F3 o32;
    F3 inv[kLightSamples];
    int ogrp;
    int ref;                  // next node / leaf (kNoRef: done)
    uint32_t rays;            // the lines that entered ref's box
    int top;
    int tc;                   // cached top entry (0: empty; a real entry has a ray bit)
};
// a strided view: a per-lane local array (stride 1, scratch memory) or a
// column of a shared-memory array (stride = block size; the walk kernels)
template <class E>   // int* / PT_LDS int*
struct ShadowStackT {
    E e;
    int stride;
    // entries from nl on in global memory (g, stride gs): see ClosestStack
    int* g = nullptr;
    int gs = 0;
    int nl = 1 << 30;
    PT_HD int get(int i) const { return i < nl ? e[i * stride] : g[(i - nl) * gs]; }
    PT_HD void set(int i, int v) const {
        if (i < nl) e[i * stride] = v;
        else g[(i - nl) * gs] = v;
    }
};
using ShadowStack = ShadowStackT<int*>;
using ShadowStackLds = ShadowStackT<PT_LDS int*>;
// push3 for the one-ray shadow walk's stack (refs only)
template <class KS>
PT_HD void push3_ref(const KS& K, int& top, int& tc, bool v1, bool v2, bool v3, int r1, int r2, int r3) {
    if (top + 3 <= K.nl) {
        int p = top;
        K.e[p * K.stride] = tc;
        p += (v1 && tc != kNoRef) ? 1 : 0;
        K.e[p * K.stride] = r3;
        p += v3 ? 1 : 0;
        K.e[p * K.stride] = r2;
        p += v2 ? 1 : 0;
        top = p;
    } else {
        if (v1 && tc != kNoRef) K.set(top++, tc);
        if (v3) K.set(top++, r3);
        if (v2) K.set(top++, r2);
    }
    tc = v1 ? r1 : tc;
}
#ifndef PT_PUSH3
#define PT_PUSH3 1
#endif
template <bool COUNT>
PT_HD int strav_pop(ShadowTrav& T, const ShadowStack& K, const SceneK& S, const ShadowSet* sh) {
    const uint32_t open = shadow_open<COUNT>(S, sh);
    while (T.tc != 0) {
        const int e = T.tc;
        T.tc = T.top > 0 ? K.get(--T.top) : 0;
        T.rays = (uint32_t)e & open & 7u;
        if (T.rays) return e >> 3;
    }
    return kNoRef;
}
template <bool COUNT>
PT_HD void strav_init(ShadowTrav& T, const SceneK& S, F3 o32, int ogrp, const ShadowSet* sh,
                      int root) {
    T.o32 = o32;
    T.ogrp = ogrp;
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) T.inv[k] = rcp_dir(sh->d32[k]);
    T.top = 0;
    T.tc = 0;
    uint32_t rays = 0;
    const BNode R = S.bnode[0];
    const F3 l = {R.lo[0] - o32.x, R.lo[1] - o32.y, R.lo[2] - o32.z};
    const F3 h = {R.hi[0] - o32.x, R.hi[1] - o32.y, R.hi[2] - o32.z};
    const uint32_t open = shadow_open<COUNT>(S, sh);
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k)
        if (((open >> k) & 1u) && box_hit(l, h, T.inv[k], sh->hhi[k])) rays |= 1u << k;
    T.rays = rays;
    T.ref = rays ? root : kNoRef;
}
// one internal node (T.ref >= 0): the nearer child (by the smallest |t| of
// its rays) next, the farther stacked with its rays
template <bool COUNT>
PT_HD void strav_node(ShadowTrav& T, const ShadowStack& K, const SceneK& S, const ShadowSet* sh) {
    const CNode C = S.cnode[T.ref];
    uint32_t m0 = 0, m1 = 0;
    float d0 = INFINITY, d1 = INFINITY;
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) {
        if (!((T.rays >> k) & 1u)) continue;
        const float e0 = cbox_dist(C.lo0, C.hi0, T.o32, T.inv[k], sh->hhi[k]);
        const float e1 = cbox_dist(C.lo1, C.hi1, T.o32, T.inv[k], sh->hhi[k]);
        m0 |= e0 < INFINITY ? 1u << k : 0u;
        m1 |= e1 < INFINITY ? 1u << k : 0u;
        d0 = fminf(d0, e0);
        d1 = fminf(d1, e1);
    }
    const bool near0 = d0 <= d1;
    const uint32_t mn = near0 ? m0 : m1, mf = near0 ? m1 : m0;
    const int rn = near0 ? C.c0 : C.c1, rf = near0 ? C.c1 : C.c0;
    if (mf) {
        if (T.tc != 0) K.set(T.top++, T.tc);
        T.tc = (int)(((uint32_t)rf << 3) | mf);
    }
    if (mn) {
        T.ref = rn;
        T.rays = mn;
    } else {
        T.ref = strav_pop<COUNT>(T, K, S, sh);
    }
}
// the units of leaf `ref` (<= -2) against the rays `rays` that reached it
template <bool COUNT, bool UC = false>
PT_HD void strav_units(const ShadowTrav& T, const SceneK& S, ShadowSet* sh, const Spill& sp,
                       Counters* cnt, int ref, uint32_t rays) {
    const int code = ~ref, u0 = code >> 3, nu = code & 7;
    for (int i = 0; i < nu; ++i) {
        const UnitF U = bvh_unit<UC>(S, u0 + i);
        fused_unit<false, COUNT, false, 1>(S, U, origin_u(U, T.o32), U.grp == T.ogrp, true, false, sh,
                                 F3{0.f, 0.f, 0.f}, nullptr, sp, cnt, rays);
    }
}
// the leaf T.ref with the rays that reached it, then the next entry
template <bool COUNT, bool UC = false>
PT_HD void strav_leaf(ShadowTrav& T, const ShadowStack& K, const SceneK& S, ShadowSet* sh,
                      const Spill& sp, Counters* cnt) {
    strav_units<COUNT, UC>(T, S, sh, sp, cnt, T.ref, T.rays);
    T.ref = strav_pop<COUNT>(T, K, S, sh);
}
// one "while-while" round; returns true when the traversal has ended
template <bool COUNT>
PT_HD bool strav_step(ShadowTrav& T, const ShadowStack& K, const SceneK& S, ShadowSet* sh,
                      const Spill& sp, Counters* cnt) {
    while (T.ref >= 0) strav_node<COUNT>(T, K, S, sh);
    if (T.ref != kNoRef) strav_leaf<COUNT>(T, K, S, sh, sp, cnt);
    return T.ref == kNoRef;
}
template <bool COUNT>
PT_HD void bvh_shadow(const SceneK& S, F3 o32, int ogrp, ShadowSet* sh, const Spill& sp,
                      Counters* cnt) {
    ShadowTrav T;
    int buf[kBvhStack];
    const ShadowStack K{buf, 1};
    strav_init<COUNT>(T, S, o32, ogrp, sh, S.bvh_root);
    while (!strav_step<COUNT>(T, K, S, sh, sp, cnt)) {
    }
}

// ------------------------------------------------ 4-wide walks (QNode) --
PT_HD float q_step(uint32_t ex, int a) {   // 2^(byte a - 127)
    const uint32_t b = ((ex >> (8 * a)) & 0xffu) << 23;
    float f;
    memcpy(&f, &b, sizeof f);
    return f;
}
PT_HD float q_byte(uint32_t w, int c) { return (float)((w >> (8 * c)) & 0xffu); }
// child c's decoded box (exact: pt_prepare.h checks it) relative to o, as
// cbox_dist forms it
PT_HD void q_box(const QNode& Q, int c, const float st[3], F3 o, F3* l, F3* h) {
    l->x = fmaf(q_byte(Q.qlo[0], c), st[0], Q.org[0]) - o.x;
    l->y = fmaf(q_byte(Q.qlo[1], c), st[1], Q.org[1]) - o.y;
    l->z = fmaf(q_byte(Q.qlo[2], c), st[2], Q.org[2]) - o.z;
    h->x = fmaf(q_byte(Q.qhi[0], c), st[0], Q.org[0]) - o.x;
    h->y = fmaf(q_byte(Q.qhi[1], c), st[1], Q.org[1]) - o.y;
    h->z = fmaf(q_byte(Q.qhi[2], c), st[2], Q.org[2]) - o.z;
}
// A line's slab parameters on a node's grid: child c's bound q (in grid
// steps) lies at line parameter t = q A + B with A = step inv (exact: the
// step is a power of two) and B = (org - o) inv, one fma per bound instead of
// decoding the box and subtracting the origin (q_box).  Rounding: B errs by
// ~2u |org - o| |inv| and the fma by u|t|, i.e. a few u X in distance along
// the line, far inside the boxes' 64 u X inflation (pt_prepare.h), so the
// test stays conservative (hc_qbvh_check).
#ifndef PT_QLINE
#define PT_QLINE 1
#endif
struct QLine { float A[3], B[3]; };
PT_HD QLine q_line(const QNode& Q, const float st[3], F3 o, F3 inv) {
    QLine L;
    L.A[0] = st[0] * inv.x; L.B[0] = (Q.org[0] - o.x) * inv.x;
    L.A[1] = st[1] * inv.y; L.B[1] = (Q.org[1] - o.y) * inv.y;
    L.A[2] = st[2] * inv.z; L.B[2] = (Q.org[2] - o.z) * inv.z;
    return L;
}
// The same from the node's exponent bytes: A = inv * 2^(byte - 127) is one
// ldexp (exact, as the product by the power-of-two step is: the builder's
// bytes are >= 1 and |inv| >= 1, so no result is subnormal).
PT_HD QLine q_line_ex(const QNode& Q, F3 o, F3 inv) {
    QLine L;
    L.A[0] = ldexpf(inv.x, (int)(Q.ex & 0xffu) - 127); L.B[0] = (Q.org[0] - o.x) * inv.x;
    L.A[1] = ldexpf(inv.y, (int)((Q.ex >> 8) & 0xffu) - 127); L.B[1] = (Q.org[1] - o.y) * inv.y;
    L.A[2] = ldexpf(inv.z, (int)((Q.ex >> 16) & 0xffu) - 127); L.B[2] = (Q.org[2] - o.z) * inv.z;
    return L;
}
// child c: the smallest |t| of the (two-sided) line inside its box, INFINITY
// when the box is not met within |t| <= R.  max(tmin, -tmax, 0) is that
// distance (tmin > 0: tmin; tmax < 0: -tmax; else 0), and the interval meets
// [-R, R] exactly when it is <= R.
PT_HD float q_child_dist(const QNode& Q, int c, const QLine& L, float R) {
    const float x0 = fmaf(q_byte(Q.qlo[0], c), L.A[0], L.B[0]), x1 = fmaf(q_byte(Q.qhi[0], c), L.A[0], L.B[0]);
    const float y0 = fmaf(q_byte(Q.qlo[1], c), L.A[1], L.B[1]), y1 = fmaf(q_byte(Q.qhi[1], c), L.A[1], L.B[1]);
    const float z0 = fmaf(q_byte(Q.qlo[2], c), L.A[2], L.B[2]), z1 = fmaf(q_byte(Q.qhi[2], c), L.A[2], L.B[2]);
    const float tmin = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
    const float tmax = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
    const float d = fmaxf(fmaxf(tmin, -tmax), 0.0f);
    return ((tmin <= tmax) & (d <= R)) ? d : INFINITY;
}
// The same distance with the node's code words ordered along the line:
// near[a] holds the bounds the line meets first on axis a (qlo when A[a] > 0,
// qhi when A[a] < 0; A is never zero, rcp_dir).  fma(q, A, B) is monotone in
// q, so the near bound's t IS min(x0, x1) and the far bound's max(x0, x1):
// bit for bit the same result without the per-child min / max pairs (one
// word select per axis and node instead; hc_qbvh_check compares the two).
struct QSlabs { uint32_t near[3], far[3]; };
PT_HD QSlabs q_slabs(const QNode& Q, const QLine& L) {
    QSlabs s;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const bool neg = L.A[a] < 0.0f;
        s.near[a] = neg ? Q.qhi[a] : Q.qlo[a];
        s.far[a] = neg ? Q.qlo[a] : Q.qhi[a];
    }
    return s;
}
PT_HD float q_child_dist_s(const QSlabs& s, int c, const QLine& L, float R) {
    const float xn = fmaf(q_byte(s.near[0], c), L.A[0], L.B[0]), xf = fmaf(q_byte(s.far[0], c), L.A[0], L.B[0]);
    const float yn = fmaf(q_byte(s.near[1], c), L.A[1], L.B[1]), yf = fmaf(q_byte(s.far[1], c), L.A[1], L.B[1]);
    const float zn = fmaf(q_byte(s.near[2], c), L.A[2], L.B[2]), zf = fmaf(q_byte(s.far[2], c), L.A[2], L.B[2]);
    const float tmin = fmaxf(fmaxf(xn, yn), zn);
    const float tmax = fminf(fminf(xf, yf), zf);
    const float d = fmaxf(fmaxf(tmin, -tmax), 0.0f);
    return ((tmin <= tmax) & (d <= R)) ? d : INFINITY;
}
#ifndef PT_QSLABS
#define PT_QSLABS 1
#endif
#if PT_QSLABS
#define PT_QDIST(Q, S, c, L, R) q_child_dist_s((S), (c), (L), (R))
#else
#define PT_QDIST(Q, S, c, L, R) ((Q).ref[c] != kNoRef ? q_child_dist((Q), (c), (L), (R)) : INFINITY)
#endif
// 4 (distance, ref, rays) triples in ascending distance (sorting network)
PT_HD void q_sort4(float d[4], int r[4], uint32_t m[4]) {
    auto cs = [&](int i, int j) {
        const bool sw = d[j] < d[i];
        const float td = sw ? d[j] : d[i], ud = sw ? d[i] : d[j];
        const int tr = sw ? r[j] : r[i], ur = sw ? r[i] : r[j];
        const uint32_t tm = sw ? m[j] : m[i], um = sw ? m[i] : m[j];
        d[i] = td; d[j] = ud; r[i] = tr; r[j] = ur; m[i] = tm; m[j] = um;
    };
    cs(0, 1); cs(2, 3); cs(0, 2); cs(1, 3); cs(1, 2);
}
// 4 (distance, ref) pairs in ascending distance: q_sort4's network and tie
// order (an exchange only when d[j] < d[i]; d is >= 0 or +inf, so its bit
// pattern orders as the float does) on the pairs packed as 64-bit words.
// Through q_sort4 the compiler tracked the refs as a permutation of the four
// loaded words and rebuilt each with a chain of index compares.
PT_HD uint32_t f32_bits(float x) { uint32_t b; memcpy(&b, &x, 4); return b; }
PT_HD float bits_f32(uint32_t b) { float x; memcpy(&x, &b, 4); return x; }
PT_HD void q_sort4_pairs(float d[4], int r[4]) {
    uint64_t k[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) k[c] = ((uint64_t)f32_bits(d[c]) << 32) | (uint32_t)r[c];
    auto cs = [&](int i, int j) {
        const uint64_t a = k[i], b = k[j];
        const bool sw = (uint32_t)(b >> 32) < (uint32_t)(a >> 32);
        k[i] = sw ? b : a;
        k[j] = sw ? a : b;
    };
    cs(0, 1); cs(2, 3); cs(0, 2); cs(1, 3); cs(1, 2);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        d[c] = bits_f32((uint32_t)(k[c] >> 32));
        r[c] = (int)(uint32_t)k[c];
    }
}
#ifndef PT_QSORT_PAIRS
#define PT_QSORT_PAIRS 1
#endif
// one 4-wide node of the shadow walk (T.ref >= 0 a QNode): nearest child
// next, the others stacked farthest first
template <bool COUNT>
PT_HD void strav_qnode(ShadowTrav& T, const ShadowStack& K, const SceneK& S, const ShadowSet* sh) {
    const QNode Q = S.qnode[T.ref];
    float d[4];
    int r[4];
    uint32_t m[4];
#if PT_QLINE
    QLine L[kLightSamples];
    QSlabs SL[kLightSamples];
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) {
        L[k] = q_line_ex(Q, T.o32, T.inv[k]);
        SL[k] = q_slabs(Q, L[k]);
    }
#else
    const float st[3] = {q_step(Q.ex, 0), q_step(Q.ex, 1), q_step(Q.ex, 2)};
#endif
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#if !PT_QLINE
        F3 l, h;
        q_box(Q, c, st, T.o32, &l, &h);
#endif
        float dc = INFINITY;
        uint32_t mc = 0;
#pragma unroll
        for (int k = 0; k < kLightSamples; ++k) {
            // every ray computed, closed ones masked (no per-ray branch)
#if PT_QLINE
            const float e0 = PT_QDIST(Q, SL[k], c, L[k], sh->hhi[k]);
#else
            const float e0 = box_dist(l, h, T.inv[k], sh->hhi[k]);
#endif
            const float e = ((T.rays >> k) & 1u) ? e0 : INFINITY;
            mc |= e < INFINITY ? 1u << k : 0u;
            dc = fminf(dc, e);
        }
        r[c] = Q.ref[c];
#if PT_QLINE   // (no child: an empty box, no line meets it)
        d[c] = dc;
        m[c] = mc;
#else
        d[c] = r[c] != kNoRef ? dc : INFINITY;
        m[c] = r[c] != kNoRef ? mc : 0u;
#endif
    }
    q_sort4(d, r, m);
#pragma unroll
    for (int c = 3; c >= 1; --c) {
        if (m[c]) {
            if (T.tc != 0) K.set(T.top++, T.tc);
            T.tc = (int)(((uint32_t)r[c] << 3) | m[c]);
        }
    }
    if (m[0]) {
        T.ref = r[0];
        T.rays = m[0];
    } else {
        T.ref = strav_pop<COUNT>(T, K, S, sh);
    }
}
// one 4-wide node of the closest walk
template <class KS>
PT_HD void ctrav_qnode(ClosestTrav& T, const KS& K, const SceneK& S, const ClosestAcc* ca) {
    const QNode Q = S.qnode[T.ref];
    float d[4];
    int r[4];
#if !PT_QSORT_PAIRS
    uint32_t m[4] = {0u, 0u, 0u, 0u};
#endif
#if PT_QLINE
    const QLine L = q_line_ex(Q, T.o32, T.inv);
    const QSlabs SL = q_slabs(Q, L);
#else
    const float st[3] = {q_step(Q.ex, 0), q_step(Q.ex, 1), q_step(Q.ex, 2)};
#endif
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        r[c] = Q.ref[c];
#if PT_QLINE
        d[c] = PT_QDIST(Q, SL, c, L, ca->b1);   // (no child: an empty box, INFINITY)
#else
        F3 l, h;
        q_box(Q, c, st, T.o32, &l, &h);
        d[c] = r[c] != kNoRef ? box_dist(l, h, T.inv, ca->b1) : INFINITY;
#endif
    }
#if PT_QSORT_PAIRS
    q_sort4_pairs(d, r);
#else
    q_sort4(d, r, m);
#endif
#if PT_PUSH3
    push3(K, T.top, T.tref, T.tdist, d[1] < INFINITY, d[2] < INFINITY, d[3] < INFINITY, r[1], d[1], r[2], d[2],
          r[3], d[3]);
#else
#pragma unroll
    for (int c = 3; c >= 1; --c)
        if (d[c] < INFINITY) ctrav_push(T, K, r[c], d[c]);
#endif
    T.ref = d[0] < INFINITY ? r[0] : ctrav_pop(T, K, ca->b1);
}

// ----------------------------------------------- one-ray shadow walks --
// The wavefront path walks every open shadow ray of a bounce on its own (a
// work-item per ray) instead of the 3 rays as a packet.  A packet node visit
// tests 3 lines against 4 boxes whether or not each line entered the node;
// per ray a visit tests 1 line.  On K5 (host count, 48² × 2 spp) the packet
// makes 77 node visits per query, the one-ray walks 128 in total (44 per ray):
// ~40% fewer box tests, and fewer registers per work-item.
// Semantics as the packet: rays 0, 1 end at their first occluder; ray 2 (the
// leaked colour, main.py:70) tracks its lowest occluding object and ends when
// no BVH object can be lower.  Visit order does not change any result (§6).
struct Shadow1 {
    F3 d32;
    float hlo, hhi;
    int k;          // the light sample
    bool occ;       // occluded
    int key2, leak; // ray 2: lowest occluding object (n_obj: none) and the leaked colour's object
};
PT_HD bool shadow1_open(const SceneK& S, const Shadow1& r) {
    return r.k == kLightSamples - 1 ? r.key2 > S.bvh_min_obj : !r.occ;
}
// the f64 decisions of a unit's ambiguous tests for the ray (a0, a1)
// (inline: an out-of-line call's frame made the walk 2x slower)
// LRNG: the spill home is a wavefront path record's (stride 1) whose light
// points are not kept (PT_WF_LRNG): draw the point again from its RNG key
// (wf_light).  Every caller says which home it passes.
template <bool LRNG>
PT_HD void shadow1_fallback(const SceneK& S, const UnitF& U, bool a0, bool a1, Shadow1* r,
                      const Spill& sp) {
    const bool last = r->k == kLightSamples - 1;
    const D3 P = sp.get3(kSpP);
    const D3 L = LRNG ? wf_light(S, sp, r->k) : sp.get3(kSpL + 3 * r->k);
    for (int i = 0; i < 2; ++i) {
        if (!(i == 0 ? a0 : a1)) continue;
        if (last ? (U.obj >= r->key2) : r->occ) continue;   // decided meanwhile
        D3 Q;
        double sqd;
        if (eval64(S.trid[U.t[i]], P, unit(L - P), &Q, &sqd) && !(sqd < kZero) &&
            sqd < squared_dist(P, L)) {
            r->occ = true;
            if (last) {
                r->key2 = U.obj;
                r->leak = U.obj;
            }
        }
    }
}
// one BVH unit against the ray (fused_unit's shadow part for one ray, its
// f64 fallback included: same verdicts, same decisions)
template <bool LRNG>
PT_HD void shadow1_unit(const SceneK& S, const UnitF& U, F3 o32, int ogrp, Shadow1* r,
                        const Spill& sp) {
    const OriginU O = origin_u(U, o32);
    const bool coplanar = U.grp == ogrp;
    const bool last = r->k == kLightSamples - 1;
    const bool need = last ? (U.obj < r->key2) : !r->occ;
    const RayPlane p = ray_plane(U, O.h, r->d32, r->hlo, r->hhi);
    const Verdict v0 = classify_tri(U.tri[0], p, O.bo0, O.co0, r->d32);
    bool c = v0.cand & !coplanar;
    const bool a0 = v0.amb & !coplanar;
    bool a1 = false;
    if (U.count == 2) {   // (the 64-B walk records are single triangles: count 1)
        const Verdict v1 = classify_tri(U.tri[1], p, O.bo1, O.co1, r->d32);
        c |= v1.cand & !coplanar;
        a1 = v1.amb & !coplanar;
    }
    if (c) {
        r->occ = true;
        if (last && U.obj < r->key2) {
            r->key2 = U.obj;
            r->leak = U.obj;
        }
    }
    if (need && (a0 | a1)) shadow1_fallback<LRNG>(S, U, a0, a1, r, sp);
}
struct ShadowTrav1 {
    F3 o32, inv;
    int ogrp;
    int ref;    // next node / leaf code / kNoRef
    int top;    // entries in the stack array
    int tc;     // cached top entry (kNoRef: empty)
};
PT_HD void s1_init(ShadowTrav1& T, const SceneK& S, F3 o32, int ogrp, const Shadow1& r, int root) {
    T.o32 = o32;
    T.inv = rcp_dir(r.d32);
    T.ogrp = ogrp;
    T.top = 0;
    T.tc = kNoRef;
    const BNode R = S.bnode[0];
    const F3 l = {R.lo[0] - o32.x, R.lo[1] - o32.y, R.lo[2] - o32.z};
    const F3 h = {R.hi[0] - o32.x, R.hi[1] - o32.y, R.hi[2] - o32.z};
    T.ref = (shadow1_open(S, r) && box_hit(l, h, T.inv, r.hhi)) ? root : kNoRef;
}
// next stacked entry, or kNoRef when the ray is closed or the stack empty
template <class KS>
PT_HD int s1_pop(ShadowTrav1& T, const KS& K, const SceneK& S, const Shadow1& r) {
    if (!shadow1_open(S, r)) return kNoRef;
    const int e = T.tc;
    T.tc = T.top > 0 ? K.get(--T.top) : kNoRef;
    return e;
}
// one 4-wide node: nearest child next, the others stacked farthest first
template <class KS>
PT_HD void s1_qnode(ShadowTrav1& T, const KS& K, const SceneK& S, const Shadow1& r) {
    const QNode Q = S.qnode[T.ref];
    const QLine L = q_line_ex(Q, T.o32, T.inv);
    const QSlabs SL = q_slabs(Q, L);
    float d[4];
    int rf[4];
#if !PT_QSORT_PAIRS
    uint32_t m[4] = {0u, 0u, 0u, 0u};
#endif
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        rf[c] = Q.ref[c];
        d[c] = PT_QDIST(Q, SL, c, L, r.hhi);   // (no child: an empty box, INFINITY)
    }
#if PT_QSORT_PAIRS
    q_sort4_pairs(d, rf);
#else
    q_sort4(d, rf, m);
#endif
#if PT_PUSH3
    push3_ref(K, T.top, T.tc, d[1] < INFINITY, d[2] < INFINITY, d[3] < INFINITY, rf[1], rf[2], rf[3]);
#else
#pragma unroll
    for (int c = 3; c >= 1; --c) {
        if (d[c] < INFINITY) {
            if (T.tc != kNoRef) K.set(T.top++, T.tc);
            T.tc = rf[c];
        }
    }
#endif
    T.ref = d[0] < INFINITY ? rf[0] : s1_pop(T, K, S, r);
}
// the units of leaf `ref` (<= -2)
template <bool UC, bool LRNG>
PT_HD void s1_units(const ShadowTrav1& T, const SceneK& S, Shadow1* r, const Spill& sp, int ref) {
    const int code = ~ref, u0 = code >> 3, nu = code & 7;
    for (int i = 0; i < nu && shadow1_open(S, *r); ++i)
        shadow1_unit<LRNG>(S, bvh_unit<UC>(S, u0 + i), T.o32, T.ogrp, r, sp);
}

// Standalone query (primary rays, the batched intersect_objects API).  d need
// not be normalised (utils.py:110).  ogrp: coplanar group of the triangle the
// origin lies on (-1: none).
// BVH = false: the instantiation for scenes without meshes (no BVH code)
// eye: o may lie anywhere in the box of the triangles and the eye (primary
// rays: the unit_eye records), else on a scene surface (the `unit` records).
template <bool FORCE64, bool COUNT, bool BVH = true>
PT_HD int closest(const SceneK& S, D3 o, D3 d, int ogrp, const Spill& sp, D3* P, Counters* cnt,
                  bool eye) {
    const D3 dn = unit(d);
    ClosestAcc acc = closest_init();
    if (!FORCE64) {
        sp.put3(kSpP, o);
        sp.put3(kSpNd, d);
        const F3 o32 = to_f3(o - ld3(S.center));
        const F3 o32u = eye ? o32 : to_f3(o - ld3(S.center_s));
        const UnitF* units = eye ? S.unit_eye : S.unit;
        const F3 d32 = to_f3(dn);
        for (int u = 0; u < S.n_unit; ++u) {
            const UnitF U = units[u];
            closest_unit<COUNT>(S, U, origin_u(U, o32u), d32, U.grp == ogrp, sp, kSpP, kSpNd,
                                &acc, cnt);
        }
        if (BVH && S.n_bnode) {   // the meshes: closest ray only
            if (S.bvh_depth < kBvhStack) {
                bvh_closest<COUNT>(S, o32, ogrp, d32, &acc, sp, cnt);
            } else {
                ShadowSet none = {};
                bvh_pass<false, COUNT>(S, o32, ogrp, false, true, &none, d32, &acc, sp, cnt);
            }
        }
    }
    return closest_finish<FORCE64, COUNT, BVH>(S, acc, o, dn, P, cnt);
}

// Standalone compute_color (batched API): u = the 12 light-sampling uniforms.
template <bool FORCE64, bool COUNT, bool BVH = true>
PT_HD D3 nee(const SceneK& S, D3 P, D3 n, int obj, int ogrp, const double u[12],
             const Spill& sp, Counters* cnt) {
    ShadowSet sh;
    sp.put3(kSpP, P);
    shadow_setup<COUNT>(S, P, n, u, &sh, sp);
    const F3 o32 = to_f3(P - ld3(S.center)), o32u = to_f3(P - ld3(S.center_s));
    for (int u = 0; u < S.n_obj_unit; ++u) {
        if (PT_WAVE_ALL(sh.occ[0] && sh.occ[1] && sh.occ[2])) break;
        const UnitF U = S.unit[u];
        const OriginU O = FORCE64 ? OriginU{0.f, 0.f, 0.f, 0.f, 0.f} : origin_u(U, o32u);
        fused_unit<FORCE64, COUNT, false, 1>(S, U, O, U.grp == ogrp, true, false, &sh, F3{0.f, 0.f, 0.f},
                                   nullptr, sp, cnt);
    }
    if (BVH && S.n_bnode)
        bvh_pass<FORCE64, COUNT>(S, o32, ogrp, true, false, &sh, F3{0.f, 0.f, 0.f}, nullptr, sp, cnt);
    return shadow_color<COUNT>(S, obj, sh, cnt);
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
        const double cphi = sqrt_d(u_phi);
        const double sphi = sqrt_d(1.0 - u_phi);   // sin(arccos(sqrt(u)))
        const double th = kTau * u_theta;          // in [0, 6.28)
        double st, ct;
        sincos_small(th, &st, &ct);
        const D3 nd = rotate_y(R, d3(sphi * ct, sphi * st, cphi));
        *kf = m.kd * dot(nd, n);
        return nd;
    }
    // "specular": r = 2 (n.d) n - d, normalised, rotated; k *= ks (e.r)^n
    const double nd2 = dot(n, d_old) * 2;
    const D3 r = unit(d3(nd2 * n.x - d_old.x, nd2 * n.y - d_old.y, nd2 * n.z - d_old.z));
    const D3 e = unit(ld3(S.kd + kKdEye) - P);
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

// Phase clocks (dev builds only, -DPT_PHASE_CLOCKS; scripts/phase_clocks.py):
// shader-clock cycles (s_memtime) a wave spends in each part of the bounce
// loop, summed over waves into pt_phase_clk[]: 0 RNG + light samples + next
// ray, 1 the uniform units' fused pass, 2 the BVH and the light's units,
// 3 the colour, the next hit and path regeneration, 4 loop iterations,
// 5 the primary ray, 6 the whole lane (k_render)
#if defined(PT_PHASE_CLOCKS) && defined(__HIP__)
__device__ unsigned long long pt_phase_clk[8];   // (both passes: the host reads it)
#endif
#if defined(PT_PHASE_CLOCKS) && defined(__HIP_DEVICE_COMPILE__)
#define PT_STAMP(t) const uint64_t t = (uint64_t)__builtin_amdgcn_s_memtime()
#define PT_PHASE(i, v) ph[i] += (v)
// one value v into pt_phase_clk[i]: the maximum over the wave's ACTIVE
// lanes (an inactive partner of the xor butterfly counts as 0: its
// registers are not this value), added once per wave
__device__ inline void pt_phase_flush_at(int i, uint64_t v) {
    const uint64_t act = __ballot(1);
    const int lane = (int)__lane_id();
    for (int m = 32; m >= 1; m >>= 1) {
        uint64_t o = (uint64_t)__shfl_xor((unsigned long long)v, m);
        if (!((act >> (lane ^ m)) & 1ull)) o = 0;
        v = o > v ? o : v;
    }
    if (lane == __ffsll((unsigned long long)act) - 1) atomicAdd(&pt_phase_clk[i], (unsigned long long)v);
}
// the sum over the wave's active lanes into pt_phase_clk[i]
__device__ inline void pt_phase_flush_sum(int i, uint64_t v) {
    const uint64_t act = __ballot(1);
    const int lane = (int)__lane_id();
    for (int m = 32; m >= 1; m >>= 1) {
        uint64_t o = (uint64_t)__shfl_xor((unsigned long long)v, m);
        if (!((act >> (lane ^ m)) & 1ull)) o = 0;
        v += o;
    }
    if (lane == __ffsll((unsigned long long)act) - 1) atomicAdd(&pt_phase_clk[i], (unsigned long long)v);
}
// a wave's time in a phase is its last lane's (active in every iteration);
// slot 7: the lanes' own iteration counts summed (tail utilisation = slot 7
// / (64 x slot 4) for full waves)
#define PT_PHASE_FLUSH(n)                                     \
    do {                                                      \
        for (int i_ = 0; i_ < (n); ++i_) pt_phase_flush_at(i_, ph[i_]); \
        pt_phase_flush_sum(7, ph[4]);                         \
    } while (0)
#define PT_PHASE_FLUSH_AT(i, v) pt_phase_flush_at((i), (v))
#else
#define PT_STAMP(t)
#define PT_PHASE(i, v)
#define PT_PHASE_FLUSH(n)
#define PT_PHASE_FLUSH_AT(i, v)
#endif

// Sample scheduling of the bounce loop (render_loop): which sample a lane
// traces next once its path ends.  LaneSched: the lane's own samples
// sample0, sample0 + stride, ... (the host build, counting launches, BVH
// scenes, the wavefront kernels' order); pt_hip.hip's WavePool: the samples
// of a wave's pixels, handed out as lanes free up.
struct LaneSched {
    const LaneJob& J;
    int tri0;
    int si;
    PT_HD uint32_t sample() const { return (uint32_t)(J.sample0 + si * J.sample_stride); }
    PT_HD uint32_t pixel() const { return J.pixel; }
    // after an iteration; `done`: this lane's path ended.  Starts the lane's
    // next sample from the cached primary hit (primary rays are identical for
    // every sample, main.py:191); false when it has none left.
    template <bool COUNT>
    PT_HD bool advance(const SceneK& S, bool done, const Spill& sp, int* tri, D3*, Counters* cnt) {
        if (!done) return true;
        if (++si >= J.n_samples) return false;
        *tri = tri0;
        sp.put3(kSpP, sp.get3(kSpP0));
        sp.put3(kSpNd, d3(sp.get(kSpD0), sp.get(kSpD0 + 1), 0.0 - S.kd[kKdEye + 2]));
        if (COUNT) {
            bump<COUNT>(cnt, &Counters::closest_tests, (uint32_t)S.n_tri);
            bump<COUNT>(cnt, &Counters::ray_bounces, 1);
        }
        return true;
    }
};

// The bounce loop: paths are regenerated in place (Sched::advance), so a
// wave keeps tracing until all its lanes are out of samples.  The lane's
// first path starts at tri, origin and direction in the homes kSpP / kSpNd;
// sample colours are added to *acc.
template <bool FORCE64, bool COUNT, bool BVH, class Sched>
PT_HD void render_loop(const SceneK& S, const LaneJob& J, int tri, const Spill& sp, Counters* cnt,
                       Sched& q, D3* accp) {
    D3 acc = *accp;
    int b = 0;
    double k = 1.0;
    bool active = true;
#if defined(PT_PHASE_CLOCKS) && defined(__HIP_DEVICE_COMPILE__)
    uint64_t ph[5] = {0, 0, 0, 0, 0};
#endif
    while (active) {
        PT_STAMP(c0);
        const D3 P = sp.get3(kSpP);   // this bounce's origin
        const uint32_t sample = q.sample();
        const uint32_t pixel = q.pixel();
        const int obj = S.tri_obj[tri];
        const TriS R = S.tris[tri];
        const Mat& m = S.mat[obj];
        const int ogrp = S.tri_grp[tri];
        // RNG: the 16 slots of this bounce (4 Philox blocks in lockstep):
        // 0..11 light sampling, 12..14 the bounce, 15 Russian roulette
        ShadowSet sh;
#if PT_RNG_PERBLOCK
        // one Philox block per light sample, drawn where it is used (fewer
        // live registers than the four blocks in lockstep)
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < kLightSamples; ++k) {
            uint32_t c[4];
            rng_block(J.seed, pixel, sample, (uint32_t)b, (uint32_t)k, c);
            shadow_setup_k<COUNT>(S, P, ld3(R.n), k, u_of(c[0]), u_of(c[1]), u_of(c[2]), u_of(c[3]),
                                  &sh, sp);
        }
        sh.key2 = COUNT ? S.n_tri : S.n_obj;
        sh.leak = S.n_obj - 1;
        rng_block(J.seed, pixel, sample, (uint32_t)b, 3u, &w[12]);
#else
        uint32_t w[16];
        rng_blocks4(J.seed, pixel, sample, (uint32_t)b, w);
        {
            double u12[12];
#pragma unroll
            for (int i = 0; i < 12; ++i) u12[i] = u_of(w[i]);
            shadow_setup<COUNT>(S, P, ld3(R.n), u12, &sh, sp);
        }
#endif
        // next ray (main.py:236-268): it does not depend on the colour
        double kf;
        const D3 nd = bounce(S, R, m, P, sp.get3(kSpNd), u_of(w[12]), u_of(w[13]), u_of(w[14]),
                             &kf);
        const double kn = k * kf;
        bool trace = (b + 1 < J.bounces);
        double kk = kn;
        if (trace && J.rr_depth >= 0 && b >= J.rr_depth) {   // build extension
            double q = fabs(kn);
            q = q < 0.05 ? 0.05 : (q > 1.0 ? 1.0 : q);
            if (u_of(w[15]) >= q) trace = false;
            else kk = kn / q;
        }
        // one pass: 3 shadow rays + the next ray's closest hit, same origin
        sp.put3(kSpNd, nd);
        const F3 o32u = to_f3(P - ld3(S.kd + kKdCenterS));   // the uniform units' frame
        const F3 n32 = to_f3(unit(nd));
        ClosestAcc ca = closest_init();
        const bool any_trace = PT_WAVE_ANY(trace);
        PT_STAMP(c1);
        PT_PHASE(0, c1 - c0);
        if (!FORCE64 && !COUNT && PT_MARGIN) {   // occlusion as margins (> 0: occluded)
            float oc[kLightSamples] = {-1.0f, -1.0f, -1.0f};
            for (int u = 0; u < S.n_obj_unit; ++u) {
                const UnitF U = S.unit[u];
                const OriginU O = PT_QUAD ? origin_q(U, o32u) : origin_u(U, o32u);
#if PT_VOTE_MIN3   // (oc is never NaN: the three compares as one minimum)
                const bool do_shadow = PT_WAVE_ANY(!(min3f(oc[0], oc[1], oc[2]) > 0.0f));
#else
                const bool do_shadow =
                    PT_WAVE_ANY(!(oc[0] > 0.0f && oc[1] > 0.0f && oc[2] > 0.0f));
#endif
                fused_unit<FORCE64, COUNT, true>(S, U, O, U.grp == ogrp, do_shadow, any_trace,
                                                 &sh, n32, &ca, sp, cnt, 15u, oc);
            }
#pragma unroll
            for (int k = 0; k < kLightSamples; ++k) sh.occ[k] = oc[k] > 0.0f;
        } else {
            for (int u = 0; u < S.n_obj_unit; ++u) {
                const UnitF U = S.unit[u];
                const OriginU O = FORCE64 ? OriginU{0.f, 0.f, 0.f, 0.f, 0.f} : origin_u(U, o32u);
                const bool do_shadow = PT_WAVE_ANY(!(sh.occ[0] && sh.occ[1] && sh.occ[2]));
                fused_unit<FORCE64, COUNT>(S, U, O, U.grp == ogrp, do_shadow, any_trace, &sh, n32,
                                           &ca, sp, cnt);
            }
        }
        PT_STAMP(c2);
        PT_PHASE(1, c2 - c1);
        if (BVH && S.n_bnode) {   // the meshes: shadows as a packet, the closest ray ordered
            const F3 o32 = to_f3(P - ld3(S.kd + kKdCenter));   // the BVH's frame
            const bool ordered = !FORCE64 && S.bvh_depth < kBvhStack;
            if (ordered) {
                bvh_shadow<COUNT>(S, o32, ogrp, &sh, sp, cnt);
                if (trace) bvh_closest<COUNT>(S, o32, ogrp, n32, &ca, sp, cnt);
            } else {
                bvh_pass<FORCE64, COUNT>(S, o32, ogrp, true, !FORCE64 && trace, &sh, n32, &ca, sp,
                                         cnt);
            }
        }
        if (!FORCE64 && any_trace) {
            for (int u = S.n_obj_unit; u < S.n_unit; ++u) {   // the light's units
                const UnitF U = S.unit[u];
#if PT_LIGHT_QUAD && PT_QUAD && PT_MARGIN
                if (!COUNT) {   // the render loop's unit form (one pair of forms for a quad)
                    uint32_t amb = 0;
                    closest_unit_m(U, origin_q(U, o32u), U.grp == ogrp, n32, &ca, &amb);
                    if (amb) fused_fallback<FORCE64, COUNT, true, 2>(S, U, amb, &sh, &ca, sp, cnt, nullptr);   // rare
                    continue;
                }
#endif
                closest_unit<COUNT>(S, U, origin_u(U, o32u), n32, U.grp == ogrp, sp, kSpP, kSpNd,
                                    &ca, cnt);
            }
        }
        PT_STAMP(c3);
        PT_PHASE(2, c3 - c2);
        {   // l_k . n again from the homes, with shadow_setup's operations:
            // recomputed rather than carried across the unit loops (-0.05 ms)
            const D3 Pc = sp.get3(kSpP), nc = ld3(S.tris[tri].n);
#pragma unroll
            for (int j = 0; j < kLightSamples; ++j)
                sh.ln[j] = dot(unit(sp.get3(kSpL + 3 * j) - Pc), nc);
        }
        const D3 col = shadow_color<COUNT>(S, obj, sh, cnt);
        acc = acc + col * k;   // main.py:230-231 (k before this bounce's update)
        k = kk;
        bool done = !trace;
        if (trace) {
            D3 Pn;
            // the hit point goes straight to the origin slot (overwritten below
            // when the path ends here)
            const int tn = closest_finish<FORCE64, COUNT, BVH>(S, ca, sp.get3(kSpP),
                                                          unit(sp.get3(kSpNd)), &Pn, cnt, &sp);
            if (tn < 0) {
                bump<COUNT>(cnt, &Counters::escapes, 1);
                done = true;
            } else if (tn >= S.n_obj_tri) {   // light: main.py:214-215
                acc = acc + ld3(S.kd + kKdLightRgb) * k;
                bump<COUNT>(cnt, &Counters::light_hits, 1);
                done = true;
            } else {
                tri = tn;
                ++b;
            }
        }
        active = q.template advance<COUNT>(S, done, sp, &tri, &acc, cnt);
        if (done) {
            b = 0;
            k = 1.0;
        }
        PT_STAMP(c4);
        PT_PHASE(3, c4 - c3);
        PT_PHASE(4, 1);
    }
    PT_PHASE_FLUSH(5);
    *accp = acc;
}

// All samples of one lane for one pixel (LaneSched); returns the SUM of
// sample colours.
template <bool FORCE64, bool COUNT, bool BVH = true>
PT_HD D3 render_lane(const SceneK& S, const LaneJob& J, D3 d0, int tri0, D3 P0,
                     const Spill& sp, Counters* cnt) {
    D3 acc = d3(0, 0, 0);
    if (J.n_samples <= 0 || J.bounces <= 0) return acc;   // main.py:192 never runs
    if (tri0 < 0 || tri0 >= S.n_obj_tri) {   // primary ray escapes or hits the light
        const D3 v = tri0 < 0 ? d3(0, 0, 0) : ld3(S.kd + kKdLightRgb);
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
    sp.put(kSpD0, d0.x);
    sp.put(kSpD0 + 1, d0.y);
    sp.put3(kSpP0, P0);
    sp.put3(kSpP, P0);
    sp.put3(kSpNd, d0);   // incoming direction of bounce 0 (main.py:191)
    if (COUNT) {   // the cached primary trace, counted per sample
        bump<COUNT>(cnt, &Counters::closest_tests, (uint32_t)S.n_tri);
        bump<COUNT>(cnt, &Counters::ray_bounces, 1);
    }
    LaneSched q{J, tri0, 0};
    render_loop<FORCE64, COUNT, BVH>(S, J, tri0, sp, cnt, q, &acc);
    return acc;
}

}  // namespace pt
