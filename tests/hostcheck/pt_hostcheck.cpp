// pt_hostcheck.cpp — TEST INFRASTRUCTURE.  Compiles the render kernel's own
// per-lane code (pathtracerpython_amd/csrc/pt_path.h, pt_core.h, pt_prepare.h)
// for the host with g++, so the CPU test suite can check the kernel logic —
// in particular the f32 filter's "certain" verdicts — against the oracle and
// against its own FORCE_F64 mode without a GPU.  Never used by the product.
#define __host__
#define __device__
#define __forceinline__ inline
#include <cstddef>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <random>

#include "../../pathtracerpython_amd/csrc/pt_path.h"
#include "../../pathtracerpython_amd/csrc/pt_wavefront.h"
#include "../../pathtracerpython_amd/csrc/pt_prepare.h"

using namespace pt;

extern "C" {

// sizes and field offsets of the C-ABI structs as the C++ compiler lays
// them out (the ctypes mirror in _abi.py must agree)
int hc_abi_layout(int64_t* out) {
    out[0] = (int64_t)sizeof(pt_scene_desc);
    out[1] = (int64_t)sizeof(pt_render_params);
    out[2] = (int64_t)sizeof(pt_stats);
    out[3] = (int64_t)offsetof(pt_stats, shadow_queries);
    out[4] = (int64_t)offsetof(pt_stats, shade_ms);
    out[5] = (int64_t)offsetof(pt_stats, closest_launches);
    out[6] = (int64_t)offsetof(pt_scene_desc, light_rgb);
    out[7] = (int64_t)offsetof(pt_render_params, sample_begin);
    return 0;
}

// Render the band of p on the host with the kernel's lane code (split = 1).
// out: rows*W*3 float64 in image orientation.  counters[8] (optional).
int hc_render(const pt_scene_desc* d, const pt_render_params* p, int force64,
              double* out, uint64_t* counters) {
    HostScene H;
    if (!prepare_scene(d, &H).empty()) return -1;
    bind_host(&H);
    int32_t first, rows;
    if (!band_layout(p, &first, &rows)) return -2;
    Counters c = {};
    double spill_mem[kSpillSlots];
    const Spill sp{spill_mem, 1};
    for (int r = 0; r < rows; ++r) {
        const int iy = first + r * p->row_step;
        for (int ix = 0; ix < p->width; ++ix) {
            const D3 eye = ld3(H.k.eye);
            const double x = linspace_at(H.k.ortho[0], H.k.ortho[2], p->width, ix);
            const double y = linspace_at(H.k.ortho[1], H.k.ortho[3], p->height, iy);
            const D3 d0 = d3(x - eye.x, y - eye.y, 0.0 - eye.z);
            LaneJob J;
            J.seed = p->seed;
            J.pixel = (uint32_t)ix * (uint32_t)p->height + (uint32_t)iy;
            J.sample0 = p->sample_begin;
            J.sample_stride = 1;
            J.n_samples = p->spp;
            J.bounces = p->bounces;
            J.rr_depth = (p->flags & PT_FLAG_RR) ? p->rr_depth : -1;
            D3 P0 = d3(0, 0, 0);
            int tri0 = -1;
            D3 acc;
            // counters requested: the count-mode lane code (exact first
            // occluders); else the render kernel's own (object-level) one
            if (force64) {
                if (p->bounces > 0) tri0 = closest<true, false>(H.k, eye, d0, -1, sp, &P0, &c, true);
                acc = counters ? render_lane<true, true>(H.k, J, d0, tri0, P0, sp, &c)
                               : render_lane<true, false>(H.k, J, d0, tri0, P0, sp, &c);
            } else {
                if (p->bounces > 0) tri0 = closest<false, false>(H.k, eye, d0, -1, sp, &P0, &c, true);
                acc = counters ? render_lane<false, true>(H.k, J, d0, tri0, P0, sp, &c)
                               : render_lane<false, false>(H.k, J, d0, tri0, P0, sp, &c);
            }
            double* o = out + ((size_t)(rows - 1 - r) * p->width + ix) * 3;
            o[0] = acc.x / p->spp; o[1] = acc.y / p->spp; o[2] = acc.z / p->spp;
        }
    }
    if (counters) {
        uint32_t v[8] = {c.closest_tests, c.shadow_tests, c.ray_bounces, c.shading_points,
                         c.light_hits, c.escapes, c.fallbacks, c.rescans};
        for (int i = 0; i < 8; ++i) counters[i] = v[i];
    }
    return 0;
}

// The wavefront form of the render (pt_wavefront.h) run on the host: every
// shade step over all slots, then every pending shadow and closest walk to
// completion, as the GPU's shade / walk kernels do (split = 1, one slot per
// pixel).  Must equal hc_render (force64 = 0, no counters) bit for bit.
// steps_out (optional): shade steps that found work.
// walk_stats (optional, int64[8]): shadow rays walked, node visits, leaves,
// leaf units; the same for the closest walks.
// depth_hist (optional, int64[2][32]): node visits of the shadow / closest
// walks by QNode depth (root = 0)
int hc_render_wavefront2(const pt_scene_desc* d, const pt_render_params* p, double* out,
                         int32_t* steps_out, int64_t* walk_stats, int64_t* depth_hist);
int hc_render_wavefront(const pt_scene_desc* d, const pt_render_params* p, double* out,
                        int32_t* steps_out, int64_t* walk_stats) {
    return hc_render_wavefront2(d, p, out, steps_out, walk_stats, nullptr);
}
int hc_render_wavefront2(const pt_scene_desc* d, const pt_render_params* p, double* out,
                         int32_t* steps_out, int64_t* walk_stats, int64_t* depth_hist) {
    int64_t ws[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HostScene H;
    if (!prepare_scene(d, &H).empty()) return -1;
    bind_host(&H);
    std::vector<int> qdepth(H.qnode.size(), 0);
    if (depth_hist && H.k.qroot >= 0) {   // depth of every QNode (refs point deeper)
        std::vector<int> st{H.k.qroot};
        while (!st.empty()) {
            const int q = st.back();
            st.pop_back();
            for (int c = 0; c < 4; ++c) {
                const int r = H.qnode[q].ref[c];
                if (r >= 0) { qdepth[r] = qdepth[q] + 1; st.push_back(r); }
            }
        }
    }
    auto hist = [&](int kind, int ref) {
        if (depth_hist && ref >= 0) ++depth_hist[kind * 32 + std::min(qdepth[ref], 31)];
    };
    if (H.k.n_bnode == 0 || H.k.n_qnode == 0 || H.k.qstack > kBvhStack) return -3;
    int32_t first, rows;
    if (!band_layout(p, &first, &rows)) return -2;
    const size_t n = (size_t)rows * p->width;
    std::vector<WfPath> W(n);
    std::vector<WfShadowQ> SQ(n);
    std::vector<WfClosestQ> CQ(n);
    std::vector<LaneJob> J(n);
    std::vector<D3> D0(n);
    for (int r = 0; r < rows; ++r) {
        const int iy = first + r * p->row_step;
        for (int ix = 0; ix < p->width; ++ix) {
            const size_t i = (size_t)r * p->width + ix;
            const D3 eye = ld3(H.k.eye);
            const double x = linspace_at(H.k.ortho[0], H.k.ortho[2], p->width, ix);
            const double y = linspace_at(H.k.ortho[1], H.k.ortho[3], p->height, iy);
            D0[i] = d3(x - eye.x, y - eye.y, 0.0 - eye.z);
            J[i].seed = p->seed;
            J[i].pixel = (uint32_t)ix * (uint32_t)p->height + (uint32_t)iy;
            J[i].sample0 = p->sample_begin;
            J[i].sample_stride = 1;
            J[i].n_samples = p->spp;
            J[i].bounces = p->bounces;
            J[i].rr_depth = (p->flags & PT_FLAG_RR) ? p->rr_depth : -1;
        }
    }
    std::vector<uint32_t> want(n);
    int32_t busy = 0;
    for (int step = 0;; ++step) {
        bool any = false;
        for (size_t i = 0; i < n; ++i) {
            want[i] = 0;
            if (step == 0) {   // (k_wf_shade's step 0: the slot's RNG key, then k_wf_primary)
                W[i].put_rkey(J[i]);
                want[i] = wf_start(H.k, J[i], D0[i], &W[i], &CQ[i]);
            }
            else if (W[i].state() != kWfDone) {
                want[i] = wf_shade(H.k, J[i], D0[i], &W[i], &SQ[i], &CQ[i], &CQ[i]);
                any = true;
            }
        }
        if (step > 0 && !any) break;
        ++busy;
        for (size_t i = 0; i < n; ++i) {
            const Spill sp{W[i].sp, 1};
            for (int k = 0; k < kLightSamples; ++k) {   // one walk per open shadow ray, as k_wf_shadow
                if (!((want[i] >> k) & 1u)) continue;
                Shadow1 r;
                F3 o32;
                int ogrp;
                wf_get_shadow1(SQ[i], k, &o32, &ogrp, &r);
                ++ws[0];
                ShadowTrav1 T;
                int buf[kBvhStackLocal];
                const ShadowStack K{buf, 1};
                s1_init(T, H.k, o32, ogrp, r, H.k.qroot);
                while (T.ref != kNoRef) {   // the walk, counted
                    while (T.ref >= 0) { hist(0, T.ref); s1_qnode(T, K, H.k, r); ++ws[1]; }
                    if (T.ref != kNoRef) {
                        ++ws[2];
                        ws[3] += (~T.ref) & 7;
                        if (H.k.bunitc) s1_units<true, PT_WF_LRNG != 0>(T, H.k, &r, sp, T.ref);
                        else s1_units<false, PT_WF_LRNG != 0>(T, H.k, &r, sp, T.ref);
                        T.ref = s1_pop(T, K, H.k, r);
                    }
                }
                wf_put_shadow1(&SQ[i], r);
            }
            if (want[i] & kWfWantClosest) {
                ClosestAcc ca = wf_get_acc(CQ[i]);
                ClosestTrav T;
                ClosestStackLocal L;
                const ClosestStack K = L.view();
                const WfClosestQ& q = CQ[i];
                ctrav_init(T, H.k, F3{q.o[0], q.o[1], q.o[2]}, q.ogrp, F3{q.d[0], q.d[1], q.d[2]}, ca.b1,
                           H.k.qroot);
                ++ws[4];
                while (T.ref != kNoRef) {   // ctrav_step, counted
                    while (T.ref >= 0) { hist(1, T.ref); ctrav_qnode(T, K, H.k, &ca); ++ws[5]; }
                    if (T.ref != kNoRef) {
                        ++ws[6];
                        ws[7] += (~T.ref) & 7;
                        if (H.k.bunitc) ctrav_leaf<false, true>(T, K, H.k, &ca, sp, nullptr);   // as k_wf_closest
                        else ctrav_leaf<false>(T, K, H.k, &ca, sp, nullptr);
                    }
                }
                CQ[i].a1 = ca.a1; CQ[i].a2 = ca.a2; CQ[i].b1 = ca.b1; CQ[i].i1 = ca.i1;
            }
        }
    }
    for (int r = 0; r < rows; ++r)
        for (int ix = 0; ix < p->width; ++ix) {
            const size_t i = (size_t)r * p->width + ix;
            double* o = out + ((size_t)(rows - 1 - r) * p->width + ix) * 3;
            o[0] = W[i].acc[0] / p->spp; o[1] = W[i].acc[1] / p->spp; o[2] = W[i].acc[2] / p->spp;
        }
    if (steps_out) *steps_out = busy;
    if (walk_stats) memcpy(walk_stats, ws, sizeof(ws));
    return 0;
}

// BVH shape: out[6] = {n_bnode, bvh_depth, n_qnode, qstack, n_bunitc, bvh_obj1}
int hc_bvh_info(const pt_scene_desc* d, int32_t* out) {
    HostScene H;
    if (!prepare_scene(d, &H).empty()) return -1;
    out[0] = H.k.n_bnode;
    out[1] = H.k.bvh_depth;
    out[2] = H.k.n_qnode;
    out[3] = H.k.qstack;
    out[4] = (int32_t)H.bunitc.size();   // the walks' 64-B unit form (0: not used)
    out[5] = H.k.bvh_obj1;
    return 0;
}

// Filter self-test: random lines (origins at the eye or on triangles,
// directions random) against every triangle; compares classify() with the
// f64 evaluation.  out[0] = wrong certain verdicts (must be 0), out[1] =
// ambiguous verdicts, out[2] = tests, out[3] = certain candidates, out[4] =
// shadow tests where the margin form (margin_plane/margin_tri) differs from
// classify_tri other than by "ambiguous" for a certain miss (must be 0).
int hc_filter_selftest(const pt_scene_desc* d, int64_t n_rays, uint64_t seed, int64_t* out) {
    HostScene H;
    if (!prepare_scene(d, &H).empty()) return -1;
    bind_host(&H);
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::normal_distribution<double> N(0.0, 1.0);
    int64_t wrong = 0, amb = 0, tests = 0, cand = 0, mdiff = 0;
    const D3 C = ld3(H.k.center), Cs = ld3(H.k.center_s);
    for (int64_t i = 0; i < n_rays; ++i) {
        D3 o;
        if (i % 4 == 0) {
            o = ld3(H.k.eye);
        } else {   // a point on a random triangle (as hit points are)
            const TriD& T = H.trid[rng() % H.trid.size()];
            double a = U(rng), b = U(rng);
            if (a + b > 1) { a = 1 - a; b = 1 - b; }
            o = ld3(T.v1) + (ld3(T.v2) - ld3(T.v1)) * a + (ld3(T.v3) - ld3(T.v1)) * b;
        }
        D3 dir = d3(N(rng), N(rng), N(rng));
        if (i % 3 == 0) {   // aim near a random vertex: many near-edge lines
            const TriD& T = H.trid[rng() % H.trid.size()];
            dir = ld3(T.v1) + d3(N(rng), N(rng), N(rng)) * 1e-3 - o;
        } else if (i % 3 == 1 && (i / 3) % 2 == 0) {
            // aim at a point of a random edge, off by 1e-2 .. 1e-9: lines
            // grazing edges (e.g. from the ceiling across a wall's top edge)
            const TriD& T = H.trid[rng() % H.trid.size()];
            const D3 vv[3] = {ld3(T.v1), ld3(T.v2), ld3(T.v3)};
            const int e = (int)(rng() % 3);
            const double a = U(rng), sc = pow(10.0, -2.0 - 7.0 * U(rng));
            dir = vv[e] + (vv[(e + 1) % 3] - vv[e]) * a + d3(N(rng), N(rng), N(rng)) * sc - o;
        }
        const D3 dn = unit(dir);
        const bool at_eye = i % 4 == 0;
        // frames: the eye's origins test unit_eye, surface origins `unit`
        // (surface frame); the BVH units are in the frame with the eye
        const F3 o32 = to_f3(o - C), o32s = to_f3(o - Cs), d32 = to_f3(dn);
        const double lim = 0.5 + 40.0 * U(rng);   // a shadow range
        const float hlo = (float)(sqrt(lim) * (1 - 1e-6)), hhi = (float)(sqrt(lim) * (1 + 1e-6));
        for (int u = 0; u < H.k.n_unit + H.k.n_bunit; ++u) {   // uniform and BVH units
            const bool uni = u < H.k.n_unit;
            const UnitF& U = uni ? (at_eye ? H.unit_eye[u] : H.unit[u]) : H.bunit[u - H.k.n_unit];
            const OriginU O = origin_u(U, (uni && !at_eye) ? o32s : o32);
            const RayPlane pc = ray_plane(U, O.h, d32, INFINITY, INFINITY);
            const RayPlane ps = ray_plane(U, O.h, d32, hlo, hhi);
            for (int i = 0; i < U.count; ++i) {
                const TriB& B = U.tri[i];
                const float bo = i ? O.bo1 : O.bo0, co = i ? O.co1 : O.co0;
                D3 Q; double sqd;
                const bool h = eval64(H.trid[U.t[i]], o, dn, &Q, &sqd);
                // closest semantics
                int st = verdict_code(classify_tri(B, pc, bo, co, d32));
                const bool ref_c = h && sqd > kZero;
                ++tests;
                if (st == kAmb) ++amb;
                else if ((st == kCand) != ref_c) ++wrong;
                else if (st == kCand) {
                    ++cand;
                    const double sq = sqrt(sqd);   // the |t| interval must cover the truth
                    if (sq < (double)pc.at - pc.dt || sq > (double)pc.at + pc.dt) ++wrong;
                }
                // shadow semantics
                st = verdict_code(classify_tri(B, ps, bo, co, d32));
                const bool ref_s = h && !(sqd < kZero) && sqd < lim;
                ++tests;
                if (st == kAmb) ++amb;
                else if ((st == kCand) != ref_s) ++wrong;
                // the render loop's margin form (shadow_unit_m) of the same test
                float cm, nm, mc, ma;
                margin_plane(U, ps, hlo, hhi, INFINITY, &cm, &nm);
                margin_tri(B, ps, bo, co, d32, cm, nm, &mc, &ma);
                const int ms = mc > 0.0f ? kCand : (ma >= 0.0f ? kAmb : kMiss);
                if (ms != kAmb && (ms == kCand) != ref_s) ++wrong;
                if (ms != st && !(st == kMiss && ms == kAmb)) ++mdiff;
            }
            if (uni) {   // the render loop's unit form (quad_m): both members' tests
                float cm, nm;
                margin_plane(U, ps, hlo, hhi, INFINITY, &cm, &nm);
                const OriginU Oq = origin_q(U, at_eye ? o32 : o32s);
                const QuadM qs = quad_m(U, ps, Oq, d32), qc = quad_m(U, pc, Oq, d32);
                {   // the merged unit margins (PT_MMERGE, margin_unit) against the members'
                    float c0, a0, c1, a1, cu, au;
                    margin_m(qs.m0, ps, cm, nm, &c0, &a0);
                    margin_m(qs.m1, ps, cm, nm, &c1, &a1);
                    margin_unit(cm, nm, fmaxf(qs.m0, qs.m1), ps.del, &cu, &au);
                    const bool occ = c0 > 0.0f || c1 > 0.0f;
                    if ((cu > 0.0f) != occ) ++mdiff;                           // occlusion: same verdict
                    if (!occ && (a0 >= 0.0f || a1 >= 0.0f) && !(au >= 0.0f)) ++mdiff;   // no lost f64 test
                }
                for (int i = 0; i < 2; ++i) {
                    D3 Q; double sqd;
                    const bool h = i < U.count && eval64(H.trid[U.t[i]], o, dn, &Q, &sqd);
                    float mc, ma;
                    margin_m(i ? qs.m1 : qs.m0, ps, cm, nm, &mc, &ma);
                    const int ms = mc > 0.0f ? kCand : (ma >= 0.0f ? kAmb : kMiss);
                    const bool ref_s = h && !(sqd < kZero) && sqd < lim;
                    ++tests;
                    if (ms == kAmb) ++amb;
                    else if ((ms == kCand) != ref_s) ++wrong;
                    const int vc = verdict_code(verdict_m(i ? qc.m1 : qc.m0, pc));
                    const bool ref_c = h && sqd > kZero;
                    ++tests;
                    if (vc == kAmb) ++amb;
                    else if ((vc == kCand) != ref_c) ++wrong;
                    {   // the render loop's lean closest range (PT_CLOSEST_LEAN): no wrong certain verdict
                        RayPlane pl = pc;
                        pl.rcand = (fabsf(pl.q) > U.qhi) & (pl.at - pl.dt > kTzHi);
                        pl.rmiss = pl.at + pl.dt < kTzLo;
                        const int vl = verdict_code(verdict_m(i ? qc.m1 : qc.m0, pl));
                        if (vl != kAmb && (vl == kCand) != ref_c) ++wrong;
                        if (vl != vc && !(vc == kMiss && vl == kAmb)) ++mdiff;
                    }
                }
            }
        }
    }
    out[0] = wrong; out[1] = amb; out[2] = tests; out[3] = cand; out[4] = mdiff;
    return 0;
}

// BVH check.  Structure: every BVH unit in exactly one leaf, child boxes
// inside their parent's, every triangle vertex inside its leaf's box, skip
// links consistent with the depth-first layout.  Conservativeness: random
// lines (as in the filter self-test); for every BVH triangle the f64
// reference says the line meets at sqd, a traversal with the kernel's f32
// line and range sqrt(sqd) (1 + 1e-6) must reach that triangle's leaf.
// out: [0] structural errors, [1] missed hits, [2] hits checked, [3] nodes.
int hc_bvh_check(const pt_scene_desc* d, int64_t n_rays, uint64_t seed, int64_t* out) {
    HostScene H;
    if (!prepare_scene(d, &H).empty()) return -1;
    bind_host(&H);
    const SceneK& K = H.k;
    int64_t bad = 0, missed = 0, checked = 0;
    const int N = K.n_bnode;
    std::vector<int> seen(K.n_bunit, 0), leaf_of(K.n_bunit, -1);
    // structure: parent of node i+1 is i when i is internal; check via a stack walk
    std::vector<int> st;
    for (int i = 0; i < N; ++i) {
        const BNode& B = H.bnode[i];
        for (int a = 0; a < 3; ++a)
            if (!(B.lo[a] <= B.hi[a])) ++bad;
        if (B.leaf >= 0) {
            const int u0 = B.leaf >> 3, nu = B.leaf & 7;
            if (nu < 1 || u0 + nu > K.n_bunit) { ++bad; continue; }
            if (B.skip != (i + 1 < N ? i + 1 : -1)) ++bad;
            for (int q = u0; q < u0 + nu; ++q) {
                seen[q]++;
                leaf_of[q] = i;
                const UnitF& U = H.bunit[q];
                for (int m = 0; m < U.count; ++m) {
                    const TriD& T = H.trid[U.t[m]];
                    const double* vs[3] = {T.v1, T.v2, T.v3};
                    for (int v = 0; v < 3; ++v)
                        for (int a = 0; a < 3; ++a) {
                            const double x = vs[v][a] - K.center[a];
                            if (!(B.lo[a] <= x && x <= B.hi[a])) ++bad;
                        }
                }
            }
        } else {
            if (i + 1 >= N) { ++bad; continue; }
            const BNode& C = H.bnode[i + 1];   // first child
            for (int a = 0; a < 3; ++a)
                if (!(B.lo[a] <= C.lo[a] && C.hi[a] <= B.hi[a])) ++bad;
            if (!(B.skip == -1 || (B.skip > i + 1 && B.skip <= N))) ++bad;
        }
    }
    for (int q = 0; q < K.n_bunit; ++q)
        if (seen[q] != 1) ++bad;
    // conservativeness
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> U01(0.0, 1.0);
    std::vector<char> visited(N);
    for (int64_t r = 0; r < n_rays && K.n_bunit > 0; ++r) {
        // origin: a point on a random BVH triangle or at the eye; random direction
        D3 o;
        if (r % 4 == 0) {
            o = ld3(K.eye);
        } else {
            const UnitF& U = H.bunit[(size_t)(U01(rng) * K.n_bunit) % K.n_bunit];
            const TriD& T = H.trid[U.t[0]];
            double a = U01(rng), b = U01(rng);
            if (a + b > 1) { a = 1 - a; b = 1 - b; }
            o = ld3(T.v1) * (1 - a - b) + ld3(T.v2) * a + ld3(T.v3) * b;
        }
        D3 dir = d3(U01(rng) - 0.5, U01(rng) - 0.5, U01(rng) - 0.5);
        const D3 dn = unit(dir);
        const F3 o32 = to_f3(o - ld3(K.center)), inv = rcp_dir(to_f3(dn));
        for (int q = 0; q < K.n_bunit; ++q) {
            const UnitF& U = H.bunit[q];
            for (int m = 0; m < U.count; ++m) {
                D3 Q; double sqd;
                if (!eval64(H.trid[U.t[m]], o, dn, &Q, &sqd)) continue;
                const float R = (float)(sqrt(sqd) * (1 + 1e-6));
                ++checked;
                std::fill(visited.begin(), visited.end(), 0);
                int node = 0;
                while (node >= 0) {
                    const BNode& B = H.bnode[node];
                    const F3 l = {B.lo[0] - o32.x, B.lo[1] - o32.y, B.lo[2] - o32.z};
                    const F3 h = {B.hi[0] - o32.x, B.hi[1] - o32.y, B.hi[2] - o32.z};
                    const bool hit = box_hit(l, h, inv, R);
                    if (hit) visited[node] = 1;
                    node = (hit && B.leaf < 0) ? node + 1 : B.skip;
                }
                if (!visited[leaf_of[q]]) ++missed;
            }
        }
    }
    out[0] = bad; out[1] = missed; out[2] = checked; out[3] = N;
    return 0;
}

// 4-wide walk check (QNode, the wavefront walks' child test): random lines as
// in hc_bvh_check; for every BVH triangle the f64 line meets at sqd, a walk
// of the QNode tree that enters every child whose test (the kernels'
// q_child_dist / box_dist) passes within |t| <= sqrt(sqd)(1 + 1e-6) must
// reach that triangle's leaf; the sign-ordered child test the walks use
// (q_child_dist_s, on q_line_ex's slab parameters) must equal q_child_dist
// bit for bit on every child tested, and reject every absent child.
// out: [0] missed hits, [1] hits checked, [2] QNodes, [3] child tests whose
// two forms differ, [4] child tests compared.
int hc_qbvh_check(const pt_scene_desc* d, int64_t n_rays, uint64_t seed, int64_t* out) {
    HostScene H;
    if (!prepare_scene(d, &H).empty()) return -1;
    bind_host(&H);
    const SceneK& K = H.k;
    int64_t missed = 0, checked = 0, slab_diff = 0, slab_n = 0;
    if (K.n_qnode == 0) { out[0] = out[1] = out[2] = out[3] = out[4] = 0; return 0; }
    // leaf of every BVH unit: the leaf codes in the QNode refs
    std::vector<int> leaf_of(K.n_bunit, 0);
    for (int q = 0; q < K.n_qnode; ++q)
        for (int c = 0; c < 4; ++c) {
            const int r = H.qnode[q].ref[c];
            if (r <= -2) {
                const int code = ~r, u0 = code >> 3, nu = code & 7;
                for (int i = 0; i < nu; ++i) leaf_of[u0 + i] = r;
            }
        }
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> U01(0.0, 1.0);
    std::vector<int> reached;
    for (int64_t r = 0; r < n_rays; ++r) {
        D3 o;
        if (r % 4 == 0) {
            o = ld3(K.eye);
        } else {
            const UnitF& U = H.bunit[(size_t)(U01(rng) * K.n_bunit) % K.n_bunit];
            const TriD& T = H.trid[U.t[0]];
            double a = U01(rng), b = U01(rng);
            if (a + b > 1) { a = 1 - a; b = 1 - b; }
            o = ld3(T.v1) * (1 - a - b) + ld3(T.v2) * a + ld3(T.v3) * b;
        }
        const D3 dn = unit(d3(U01(rng) - 0.5, U01(rng) - 0.5, U01(rng) - 0.5));
        const F3 o32 = to_f3(o - ld3(K.center)), inv = rcp_dir(to_f3(dn));
        for (int q = 0; q < K.n_bunit; ++q) {
            const UnitF& U = H.bunit[q];
            for (int m = 0; m < U.count; ++m) {
                D3 Q; double sqd;
                if (!eval64(H.trid[U.t[m]], o, dn, &Q, &sqd)) continue;
                const float R = (float)(sqrt(sqd) * (1 + 1e-6));
                ++checked;
                reached.clear();
                std::vector<int> st{K.qroot};
                while (!st.empty()) {
                    const int n = st.back();
                    st.pop_back();
                    if (n <= -2) { reached.push_back(n); continue; }
                    const QNode& N = H.qnode[n];
                    const float step[3] = {q_step(N.ex, 0), q_step(N.ex, 1), q_step(N.ex, 2)};
#if PT_QLINE
                    const QLine L = q_line(N, step, o32, inv);
                    const QSlabs SL = q_slabs(N, L);
#endif
                    const QLine LX = q_line_ex(N, o32, inv);
                    if (memcmp(&LX, &L, sizeof L) != 0) ++slab_diff;   // the walks' ldexp form
                    for (int c = 0; c < 4; ++c) {
                        if (N.ref[c] == kNoRef) {   // an empty box: no line meets it
                            ++slab_n;
                            if (q_child_dist_s(SL, c, L, INFINITY) != INFINITY) ++slab_diff;
                            continue;
                        }
#if PT_QLINE
                        const float e = q_child_dist(N, c, L, R);
                        const float es = q_child_dist_s(SL, c, L, R);
                        ++slab_n;
                        if (memcmp(&e, &es, sizeof e) != 0) ++slab_diff;
#else
                        F3 l, h;
                        q_box(N, c, step, o32, &l, &h);
                        const float e = box_dist(l, h, inv, R);
#endif
                        if (e < INFINITY) st.push_back(N.ref[c]);
                    }
                }
                if (std::find(reached.begin(), reached.end(), leaf_of[q]) == reached.end()) ++missed;
            }
        }
    }
    out[0] = missed; out[1] = checked; out[2] = K.n_qnode; out[3] = slab_diff; out[4] = slab_n;
    return 0;
}

// The kernel's RNG (rng_blocks4): the 16 words of one (pixel, sample, bounce).
void hc_rng4(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t bounce, uint32_t* out) {
    rng_blocks4(seed, pixel, sample, bounce, out);
}

// Bounce-loop iterations of every lane of a single-kernel launch with `split`
// lanes per pixel (lane c of a pixel runs samples c, c + split, ...), the
// pixels of the selected rows in launch order: out[pixel * split + c] (dev
// tool: the lane-utilisation bound of a wave is sum / (64 max) over its 64).
int hc_lane_iters(const pt_scene_desc* d, const pt_render_params* p, int32_t split,
                  int32_t* out) {
    HostScene H;
    if (!prepare_scene(d, &H).empty()) return -1;
    bind_host(&H);
    int32_t first, rows;
    if (!band_layout(p, &first, &rows)) return -2;
    double spill_mem[kSpillSlots];
    const Spill sp{spill_mem, 1};
    const D3 eye = ld3(H.k.eye);
    for (int r = 0; r < rows; ++r) {
        const int iy = first + r * p->row_step;
        for (int ix = 0; ix < p->width; ++ix) {
            const double x = linspace_at(H.k.ortho[0], H.k.ortho[2], p->width, ix);
            const double y = linspace_at(H.k.ortho[1], H.k.ortho[3], p->height, iy);
            const D3 d0 = d3(x - eye.x, y - eye.y, 0.0 - eye.z);
            Counters c0 = {};
            D3 P0 = d3(0, 0, 0);
            const int tri0 = p->bounces > 0 ? closest<false, false>(H.k, eye, d0, -1, sp, &P0, &c0, true) : -1;
            for (int c = 0; c < split; ++c) {
                LaneJob J;
                J.seed = p->seed;
                J.pixel = (uint32_t)ix * (uint32_t)p->height + (uint32_t)iy;
                J.sample0 = p->sample_begin + c;
                J.sample_stride = split;
                J.n_samples = c < p->spp ? (p->spp - c + split - 1) / split : 0;
                J.bounces = p->bounces;
                J.rr_depth = (p->flags & PT_FLAG_RR) ? p->rr_depth : -1;
                Counters cnt = {};
                render_lane<false, true>(H.k, J, d0, tri0, P0, sp, &cnt);
                out[((size_t)r * p->width + ix) * split + c] = (int32_t)cnt.shading_points;
            }
        }
    }
    return 0;
}

}  // extern "C"
