// pt_wavefront.h — the wavefront form of the render loop for scenes with a
// BVH (large meshes, BASELINE config K5).
//
// Why: in the single kernel (k_render) each lane runs its own BVH walks
// (bvh_shadow, bvh_closest) inside the bounce loop.  Walk lengths vary by
// orders of magnitude (an occluded shadow ray ends after a few nodes, an
// unoccluded one crosses the whole mesh), so a wave waits for its longest
// walk: measured VALU lane utilisation 9.7% on K5 (80% on the Cornell box).
// Here the bounce loop of main.py:186-271 is cut at the walks:
//
//   shade    (one work-item per path slot): finish the previous bounce with
//            the walks' results (colour, main.py:208-231; next hit,
//            main.py:197-205), then start the next bounce — RNG, light
//            samples, next ray (main.py:236-268), the fused pass over the
//            uniform units — and append the slot to the shadow / closest
//            query lists;
//   shadow   (persistent, dynamic fetch): the BVH shadow walks;
//   closest  (persistent, dynamic fetch): the BVH closest-hit walks.
//
// A query work-item takes the next query from its list (one atomic per wave)
// as soon as its walk ends, so the waves stay full until the list drains.
// The per-slot arithmetic is that of render_lane (pt_path.h) in the same
// order, so the framebuffer is bitwise identical to k_render's (tested).
// Path state lives in HBM between the kernels: WfPath (256 B per slot, the
// f64 spill home included) and the query records.
#pragma once
#include <stddef.h>

#include "pt_path.h"

namespace pt {

// kWfBegin: the slot's pending work is finished and its next bounce is to be
// started (the split shade step: wf_finish, then wf_begin_bounce)
enum : int32_t { kWfDone = 0, kWfPrimary = 1, kWfBounce = 2, kWfBegin = 3 };

// Two 128-B lines per slot: the first holds everything a shade step reads
// and writes (the per-step fields and the spill slots P, Nd), the second the
// slot's RNG key in the light-point slots (written once; PT_WF_LRNG: the f64
// fallbacks redraw a light point from it, Spill::light — with PT_WF_LRNG=0
// the points themselves, written per bounce) and the primary hit (read when
// a sample restarts).
struct alignas(128) WfPath {
    double acc[3];            // sum of this slot's sample colours
    double k, kk;             // throughput before / after the pending bounce
    double ln[kLightSamples]; // l_k . n of the pending bounce's light samples
    int32_t tri, tri0, si;    // the pending bounce's triangle, the primary hit's, the sample
    uint32_t sb;              // state | trace << 2 | b << 3 (the bounce index)
    double sp[kSpillSlots];   // the spill home of pt_path.h (Spill{sp, 1}): P, Nd | key (L), D0, P0
    double pad[2];
    PT_HD int state() const { return (int)(sb & 3u); }
    PT_HD bool trace() const { return ((sb >> 2) & 1u) != 0; }
    PT_HD int b() const { return (int)(sb >> 3); }
    PT_HD void set(int state, bool trace, int b) { sb = (uint32_t)state | (trace ? 4u : 0u) | ((uint32_t)b << 3); }
    // the slot's RNG key in the light-point slots (Spill::light)
    PT_HD void put_rkey(const LaneJob& J) {
        const uint64_t w[3] = {J.seed, (uint64_t)J.pixel | (uint64_t)(uint32_t)J.sample0 << 32,
                               (uint64_t)(uint32_t)J.sample_stride};
        __builtin_memcpy(&sp[kSpL], w, sizeof(w));
    }
};
static_assert(sizeof(WfPath) == 256, "WfPath is 256 B");
static_assert(offsetof(WfPath, si) + 8 == offsetof(WfPath, sp) && offsetof(WfPath, sb) + 4 == offsetof(WfPath, sp),
              "Spill::light reads si and sb just below the home");
static_assert(offsetof(WfPath, sp) + (kSpNd + 3) * sizeof(double) <= 128,
              "P and Nd in the first line");

// shadow walks: in = the state after the uniform units, out = the final
// state.  The one-ray walks of a query write disjoint fields: ray 0 / 1 its
// wocc entry, ray 2 bit 2 of occ and leak.
struct alignas(16) WfShadowQ {
    float o[3];
    int32_t ogrp;
    float d[kLightSamples][3];
    float hlo[kLightSamples], hhi[kLightSamples];
    int32_t occ;              // bit k: shadow ray k occluded (the uniform units; ray 2's walk)
    int32_t key2, leak;
    int32_t wocc[2];          // rays 0, 1: occluded by the BVH (their walks)
};
static_assert(sizeof(WfShadowQ) == 96, "WfShadowQ is 96 B");

// closest walk: in = the candidates of the uniform units, out = all candidates
struct alignas(16) WfClosestQ {
    float o[3];
    int32_t ogrp;
    float d[3];
    int32_t i1;
    float a1, a2, b1;
    int32_t pad;
};
static_assert(sizeof(WfClosestQ) == 48, "WfClosestQ is 48 B");

PT_HD void wf_put_shadow(WfShadowQ* q, F3 o32, int ogrp, const ShadowSet& sh) {
    q->o[0] = o32.x; q->o[1] = o32.y; q->o[2] = o32.z;
    q->ogrp = ogrp;
    int occ = 0;
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) {
        q->d[k][0] = sh.d32[k].x; q->d[k][1] = sh.d32[k].y; q->d[k][2] = sh.d32[k].z;
        q->hlo[k] = sh.hlo[k];
        q->hhi[k] = sh.hhi[k];
        occ |= sh.occ[k] ? 1 << k : 0;
    }
    q->occ = occ;
    q->key2 = sh.key2;
    q->leak = sh.leak;
    q->wocc[0] = q->wocc[1] = 0;
}
// the walk's view of a query (count-mode fields unused: the wavefront path
// does not count)
PT_HD void wf_get_shadow(const SceneK& S, const WfShadowQ& q, F3* o32, int* ogrp, ShadowSet* sh) {
    *o32 = F3{q.o[0], q.o[1], q.o[2]};
    *ogrp = q.ogrp;
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) {
        sh->d32[k] = F3{q.d[k][0], q.d[k][1], q.d[k][2]};
        sh->hlo[k] = q.hlo[k];
        sh->hhi[k] = q.hhi[k];
        sh->occ[k] = (q.occ >> k) & 1;
        sh->first[k] = S.n_tri;
        sh->ln[k] = 0.0;
    }
    sh->key2 = q.key2;
    sh->leak = q.leak;
}
// a one-ray walk's view of shadow ray k of a query
PT_HD void wf_get_shadow1(const WfShadowQ& q, int k, F3* o32, int* ogrp, Shadow1* r) {
    *o32 = F3{q.o[0], q.o[1], q.o[2]};
    *ogrp = q.ogrp;
    r->d32 = F3{q.d[k][0], q.d[k][1], q.d[k][2]};
    r->hlo = q.hlo[k];
    r->hhi = q.hhi[k];
    r->k = k;
    r->occ = false;   // (only open rays are walked)
    r->key2 = q.key2;
    r->leak = q.leak;
}
// its result into the query record (fields of ray k only)
// (only an occluded ray writes: wocc is 0 from wf_put_shadow, and a ray's
// leak changes only when it is occluded — an unoccluded ray's walk leaves
// the query record's lines untouched, PT_WF_PUT_OCC)
#ifndef PT_WF_PUT_OCC
#define PT_WF_PUT_OCC 1
#endif
PT_HD void wf_put_shadow1(WfShadowQ* q, const Shadow1& r) {
    if (PT_WF_PUT_OCC && !r.occ) return;
    if (r.k < kLightSamples - 1) {
        q->wocc[r.k] = r.occ ? 1 : 0;
    } else {
        if (r.occ) q->occ |= 1 << r.k;
        q->leak = r.leak;
    }
}
// list entries of the shadow walks: (slot << 2) | ray
PT_HD int32_t wf_shadow_entry(int32_t slot, int k) { return (slot << 2) | k; }

PT_HD void wf_put_closest(WfClosestQ* q, F3 o32, int ogrp, F3 d32, const ClosestAcc& c) {
    q->o[0] = o32.x; q->o[1] = o32.y; q->o[2] = o32.z;
    q->ogrp = ogrp;
    q->d[0] = d32.x; q->d[1] = d32.y; q->d[2] = d32.z;
    q->i1 = c.i1;
    q->a1 = c.a1; q->a2 = c.a2; q->b1 = c.b1;
}
PT_HD ClosestAcc wf_get_acc(const WfClosestQ& q) {
    ClosestAcc c;
    c.a1 = q.a1; c.a2 = q.a2; c.b1 = q.b1; c.i1 = q.i1;
    return c;
}

// What a shade step asks for next (bit k < 3: a walk of shadow ray k, bit 3:
// a closest walk)
enum : uint32_t { kWfWantShadow = 7u, kWfWantClosest = 8u };

// Start the slot (shade step 0): the primary ray's uniform part, as closest()
// does for it in k_render; the BVH part is a closest query.
PT_HD uint32_t wf_start(const SceneK& S, const LaneJob& J, D3 d0, WfPath* W, WfClosestQ* cq) {
    W->acc[0] = W->acc[1] = W->acc[2] = 0.0;
    W->set(kWfDone, false, 0);
    if (J.n_samples <= 0 || J.bounces <= 0) return 0;   // main.py:192 never runs
    const Spill sp{W->sp, 1};
    const D3 eye = ld3(S.eye);
    const D3 dn = unit(d0);
    sp.put3(kSpP, eye);
    sp.put3(kSpNd, d0);
    const F3 o32 = to_f3(eye - ld3(S.center));
    const F3 d32 = to_f3(dn);
    ClosestAcc acc = closest_init();
    for (int u = 0; u < S.n_unit; ++u) {   // from the eye: the unit_eye records
        const UnitF U = S.unit_eye[u];
        closest_unit<false>(S, U, origin_u(U, o32), d32, U.grp == -1, sp, kSpP, kSpNd, &acc,
                            nullptr);
    }
    wf_put_closest(cq, o32, -1, d32, acc);
    W->set(kWfPrimary, false, 0);
    return kWfWantClosest;
}

// The body of render_lane's loop up to its walks: RNG, light samples, next
// ray, the fused pass over the uniform units (pt_path.h render_lane).
// The sort key of a query origin (the BVH frame, PT_WF_BIN, render_wavefront):
// 4 bits per axis over the root node's grid, in Morton order (neighbouring
// cells get neighbouring keys)
PT_HD uint32_t wf_cell(const SceneK& S, F3 o) {
    if (S.qroot < 0) return 0;
    const QNode& Q = S.qnode[S.qroot];
    const float v[3] = {o.x, o.y, o.z};
    uint32_t c[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float f = (v[a] - Q.org[a]) * (16.0f / (255.0f * q_step(Q.ex, a)));
        const int i = (int)f;
        c[a] = (uint32_t)(f > 0.0f ? (i > 15 ? 15 : i) : 0);
    }
    uint32_t m = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int a = 0; a < 3; ++a) m |= ((c[a] >> b) & 1u) << (3 * b + a);
    return m;
}
// KEY: the origin's cell in bits 16..27 of the result (k_wf_shade takes it off)
template <bool KEY = false>
PT_HD uint32_t wf_begin_bounce(const SceneK& S, const LaneJob& J, WfPath* W, WfShadowQ* shq,
                               WfClosestQ* cq) {
    const Spill sp{W->sp, 1};
    const D3 P = sp.get3(kSpP);
    const int tri = W->tri, b = W->b();
    const uint32_t sample = (uint32_t)(J.sample0 + W->si * J.sample_stride);
    const int obj = S.tri_obj[tri];
    const TriS R = S.tris[tri];
    const Mat& m = S.mat[obj];
    const int ogrp = S.tri_grp[tri];
    ShadowSet sh;
    uint32_t w[16];
#if PT_RNG_PERBLOCK   // as render_lane: one Philox block per light sample, where it is used
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) {
        uint32_t c[4];
        rng_block(J.seed, J.pixel, sample, (uint32_t)b, (uint32_t)k, c);
        shadow_setup_k<false, !PT_WF_LRNG>(S, P, ld3(R.n), k, u_of(c[0]), u_of(c[1]), u_of(c[2]),
                                           u_of(c[3]), &sh, sp);
    }
    sh.key2 = S.n_obj;
    sh.leak = S.n_obj - 1;
    rng_block(J.seed, J.pixel, sample, (uint32_t)b, 3u, &w[12]);
#else
    // (shadow_setup stores the light points into the home's kSpL slots, where
    // a PT_WF_LRNG record keeps its RNG key: the two switches exclude each
    // other)
    static_assert(!PT_WF_LRNG, "PT_WF_LRNG needs PT_RNG_PERBLOCK (the light points must not overwrite the key)");
    rng_blocks4(J.seed, J.pixel, sample, (uint32_t)b, w);
    {
        double u12[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) u12[i] = u_of(w[i]);
        shadow_setup<false>(S, P, ld3(R.n), u12, &sh, sp);
    }
#endif
    double kf;
    const D3 nd = bounce(S, R, m, P, sp.get3(kSpNd), u_of(w[12]), u_of(w[13]), u_of(w[14]), &kf);
    const double kn = W->k * kf;
    bool trace = (b + 1 < J.bounces);
    double kk = kn;
    if (trace && J.rr_depth >= 0 && b >= J.rr_depth) {   // build extension
        double q = fabs(kn);
        q = q < 0.05 ? 0.05 : (q > 1.0 ? 1.0 : q);
        if (u_of(w[15]) >= q) trace = false;
        else kk = kn / q;
    }
    sp.put3(kSpNd, nd);
    const F3 o32 = to_f3(P - ld3(S.kd + kKdCenter));      // the BVH's frame (the walks)
    const F3 o32u = to_f3(P - ld3(S.kd + kKdCenterS));   // the uniform units' frame
    const F3 n32 = to_f3(unit(nd));
    ClosestAcc ca = closest_init();
    const bool any_trace = PT_WAVE_ANY(trace);
    {
        float oc[kLightSamples] = {-1.0f, -1.0f, -1.0f};
        for (int u = 0; u < S.n_obj_unit; ++u) {
            const UnitF U = S.unit[u];
            const OriginU O = PT_QUAD ? origin_q(U, o32u) : origin_u(U, o32u);
            const bool do_shadow = PT_WAVE_ANY(!(oc[0] > 0.0f && oc[1] > 0.0f && oc[2] > 0.0f));
            fused_unit<false, false, true, 3, PT_WF_LRNG != 0>(S, U, O, U.grp == ogrp, do_shadow, any_trace,
                                                               &sh, n32, &ca, sp, nullptr, 15u, oc);
        }
#pragma unroll
        for (int k = 0; k < kLightSamples; ++k) sh.occ[k] = oc[k] > 0.0f;
    }
    if (any_trace) {
        for (int u = S.n_obj_unit; u < S.n_unit; ++u) {   // the light's units
            const UnitF U = S.unit[u];
            closest_unit<false>(S, U, origin_u(U, o32u), n32, U.grp == ogrp, sp, kSpP, kSpNd, &ca,
                                nullptr);
        }
    }
    uint32_t want = KEY ? wf_cell(S, o32) << 16 : 0u;
    wf_put_shadow(shq, o32, ogrp, sh);
    want |= shadow_open<false>(S, &sh);   // the rays still open, one walk each
    if (trace) {
        wf_put_closest(cq, o32, ogrp, n32, ca);
        want |= kWfWantClosest;
    }
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) W->ln[k] = sh.ln[k];
    W->kk = kk;
    W->set(kWfBounce, trace, b);
    return want;
}

// Shade step >= 1, first half: finish the pending work of the slot with the
// walks' results (the colour, the next hit, path end / next sample).  Returns
// true when the slot's next bounce is to be started (state kWfBegin; the
// second half is wf_begin_bounce).  pq: the slot's primary query (the GPU
// shares one per pixel, k_wf_primary; the host emulation has one per slot, cq)
PT_HD bool wf_finish(const SceneK& S, const LaneJob& J, D3 d0, WfPath* W, const WfShadowQ* shq,
                     const WfClosestQ* cq, const WfClosestQ* pq) {
    const Spill sp{W->sp, 1};
    if (W->state() == kWfPrimary) {   // k_render: closest(eye, d0) then render_lane's prologue
        D3 P0 = d3(0, 0, 0);
        const int tri0 = closest_finish<false, false, true>(S, wf_get_acc(*pq), ld3(S.eye), unit(d0),
                                                            &P0, nullptr);
        if (tri0 < 0 || tri0 >= S.n_obj_tri) {   // primary ray escapes or hits the light
            const D3 v = tri0 < 0 ? d3(0, 0, 0) : ld3(S.kd + kKdLightRgb);
            D3 acc = d3(0, 0, 0);
            for (int i = 0; i < J.n_samples; ++i) acc = acc + v;
            W->acc[0] = acc.x; W->acc[1] = acc.y; W->acc[2] = acc.z;
            W->set(kWfDone, false, 0);
            return false;
        }
        W->si = 0;
        W->set(kWfBegin, false, 0);   // (b = 0; begin_bounce sets the state)
        W->tri = tri0;
        W->tri0 = tri0;
        W->k = 1.0;
        sp.put(kSpD0, d0.x);
        sp.put(kSpD0 + 1, d0.y);
        sp.put3(kSpP0, P0);
        sp.put3(kSpP, P0);
        sp.put3(kSpNd, d0);   // incoming direction of bounce 0 (main.py:191)
        return true;
    }
    if (W->state() != kWfBounce) return false;
    // the colour of the pending bounce (main.py:208-231)
    ShadowSet sh;
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) {
        sh.occ[k] = (shq->occ >> k) & 1;
        sh.ln[k] = W->ln[k];
        sh.first[k] = S.n_tri;
    }
    sh.leak = shq->leak;
    for (int k = 0; k < kLightSamples - 1; ++k) sh.occ[k] = sh.occ[k] | (shq->wocc[k] != 0);
    const D3 col = shadow_color<false>(S, S.tri_obj[W->tri], sh, nullptr);   // the pending bounce's object
    D3 acc = ld3(W->acc);
    double k = W->k;
    acc = acc + col * k;   // main.py:230-231 (k before this bounce's update)
    k = W->kk;
    bool done = !W->trace();
    int tri = W->tri, b = W->b(), si = W->si;
    if (!done) {
        D3 Pn;
        const int tn = closest_finish<false, false, true>(S, wf_get_acc(*cq), sp.get3(kSpP),
                                                         unit(sp.get3(kSpNd)), &Pn, nullptr, &sp);
        if (tn < 0) {
            done = true;
        } else if (tn >= S.n_obj_tri) {   // light: main.py:214-215
            acc = acc + ld3(S.kd + kKdLightRgb) * k;
            done = true;
        } else {
            tri = tn;
            ++b;
        }
    }
    if (done) {
        ++si;
        if (si < J.n_samples) {   // next sample from the cached primary hit
            b = 0;
            tri = W->tri0;
            k = 1.0;
            sp.put3(kSpP, sp.get3(kSpP0));
            sp.put3(kSpNd, d3(sp.get(kSpD0), sp.get(kSpD0 + 1), 0.0 - S.eye[2]));
        }
    }
    W->acc[0] = acc.x; W->acc[1] = acc.y; W->acc[2] = acc.z;
    W->k = k;
    W->tri = tri;
    W->si = si;
    if (si >= J.n_samples) {
        W->set(kWfDone, false, 0);
        return false;
    }
    W->set(kWfBegin, false, b);   // (begin_bounce sets the state and trace)
    return true;
}

// Shade step >= 1: wf_finish, then the next bounce's start.  Returns the
// queries wanted.  (One call site of wf_begin_bounce: round 4 started the
// next bounce from two, inlined twice — 141 instead of 113 VGPRs for
// k_wf_shade, the same time)
template <bool KEY = false>
PT_HD uint32_t wf_shade(const SceneK& S, const LaneJob& J, D3 d0, WfPath* W, WfShadowQ* shq,
                        WfClosestQ* cq, const WfClosestQ* pq) {
    return wf_finish(S, J, d0, W, shq, cq, pq) ? wf_begin_bounce<KEY>(S, J, W, shq, cq) : 0u;
}

}  // namespace pt
