// pt_hostcheck.cpp — TEST INFRASTRUCTURE.  Compiles the render kernel's own
// per-lane code (pathtracerpython_amd/csrc/pt_path.h, pt_core.h, pt_prepare.h)
// for the host with g++, so the CPU test suite can check the kernel logic —
// in particular the f32 filter's "certain" verdicts — against the oracle and
// against its own FORCE_F64 mode without a GPU.  Never used by the product.
#define __host__
#define __device__
#define __forceinline__ inline
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <random>

#include "../../pathtracerpython_amd/csrc/pt_path.h"
#include "../../pathtracerpython_amd/csrc/pt_prepare.h"

using namespace pt;

extern "C" {

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
            if (force64) {
                if (p->bounces > 0) tri0 = closest<true, false>(H.k, eye, d0, -1, sp, &P0, &c);
                acc = render_lane<true, true>(H.k, J, d0, tri0, P0, sp, &c);
            } else {
                if (p->bounces > 0) tri0 = closest<false, false>(H.k, eye, d0, -1, sp, &P0, &c);
                acc = render_lane<false, true>(H.k, J, d0, tri0, P0, sp, &c);
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

// Filter self-test: random lines (origins at the eye or on triangles,
// directions random) against every triangle; compares classify() with the
// f64 evaluation.  out[0] = wrong certain verdicts (must be 0), out[1] =
// ambiguous verdicts, out[2] = tests, out[3] = certain candidates.
int hc_filter_selftest(const pt_scene_desc* d, int64_t n_rays, uint64_t seed, int64_t* out) {
    HostScene H;
    if (!prepare_scene(d, &H).empty()) return -1;
    bind_host(&H);
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::normal_distribution<double> N(0.0, 1.0);
    int64_t wrong = 0, amb = 0, tests = 0, cand = 0;
    const D3 C = ld3(H.k.center);
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
        }
        const D3 dn = unit(dir);
        const F3 o32 = to_f3(o - C), d32 = to_f3(dn);
        const double lim = 0.5 + 40.0 * U(rng);   // a shadow range
        const float hlo = (float)(sqrt(lim) * (1 - 1e-6)), hhi = (float)(sqrt(lim) * (1 + 1e-6));
        for (int u = 0; u < H.k.n_unit; ++u) {
            const UnitF& U = H.unit[u];
            const OriginU O = origin_u(U, o32);
            const RayPlane pc = ray_plane(U, O.h, d32, INFINITY, INFINITY);
            const RayPlane ps = ray_plane(U, O.h, d32, hlo, hhi);
            for (int i = 0; i < U.count; ++i) {
                const TriB& B = U.tri[i];
                const float bo = i ? O.bo1 : O.bo0, co = i ? O.co1 : O.co0;
                D3 Q; double sqd;
                const bool h = eval64(H.trid[B.t], o, dn, &Q, &sqd);
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
            }
        }
    }
    out[0] = wrong; out[1] = amb; out[2] = tests; out[3] = cand;
    return 0;
}

}  // extern "C"
