// Dev experiment (host only): node visits of the one-ray shadow walks when a
// walk starts at the leaf of its origin's triangle and climbs (bottom-up),
// against the shipped top-down nearest-first walk, on the rays of a host
// wavefront render of the K5 scene.  The 4-wide tree is QBuilder's (opening
// the two-child tree's largest-area child) with exact f32 boxes; within a
// subtree both walks go nearest-first with a stack; the bottom-up walk tests
// the origin's leaf, then each ancestor's other children (nearest-first,
// each subtree to completion) until the ray closes or the root is done.  Every
// walk's result must equal the shipped walk's (checked).
//   driven by scripts/micro/bottomup_count.py
#include "../../tests/hostcheck/pt_hostcheck.cpp"

#include <vector>

namespace {
struct BNode4 {
    int n;
    int32_t ref[4];
    float lo[4][3], hi[4][3];
};
struct Tree4 {
    std::vector<BNode4> node;
    std::vector<int32_t> parent, pslot;   // per node: parent node (-1: root), slot in it
    std::vector<int32_t> leaf_parent, leaf_slot;   // per unit: the node holding its leaf
    int32_t root = kNoRef;
    int32_t build(const HostScene& H, int32_t ref, int32_t par, int32_t slot) {
        if (ref < 0) {
            const int u = (~ref) >> 3;
            leaf_parent[u] = par;
            leaf_slot[u] = slot;
            return ref;
        }
        struct Ch { int32_t ref; float lo[3], hi[3]; };
        std::vector<Ch> ch;
        auto open = [&](int32_t r) {
            const CNode& C = H.cnode[r];
            ch.push_back(Ch{C.c0, {C.lo0[0], C.lo0[1], C.lo0[2]}, {C.hi0[0], C.hi0[1], C.hi0[2]}});
            ch.push_back(Ch{C.c1, {C.lo1[0], C.lo1[1], C.lo1[2]}, {C.hi1[0], C.hi1[1], C.hi1[2]}});
        };
        auto area = [](const Ch& c) {
            const double e0 = (double)c.hi[0] - c.lo[0], e1 = (double)c.hi[1] - c.lo[1], e2 = (double)c.hi[2] - c.lo[2];
            return e0 * e1 + e1 * e2 + e2 * e0;
        };
        open(ref);
        while ((int)ch.size() < 4) {
            int best = -1;
            for (int i = 0; i < (int)ch.size(); ++i)
                if (ch[i].ref >= 0 && (best < 0 || area(ch[i]) > area(ch[best]))) best = i;
            if (best < 0) break;
            const int32_t r = ch[best].ref;
            ch.erase(ch.begin() + best);
            open(r);
        }
        const int32_t me = (int32_t)node.size();
        node.push_back(BNode4{});
        parent.push_back(par);
        pslot.push_back(slot);
        BNode4 W{};
        W.n = (int)ch.size();
        for (int c = 0; c < W.n; ++c)
            for (int a = 0; a < 3; ++a) { W.lo[c][a] = ch[c].lo[a]; W.hi[c][a] = ch[c].hi[a]; }
        for (int c = 0; c < W.n; ++c) W.ref[c] = build(H, ch[c].ref, me, c);
        node[me] = W;
        return me;
    }
};
struct Count { int64_t rays = 0, visits = 0, units = 0, mismatches = 0, occluded = 0, occ_visits = 0; };

// children of node q met within R except slot `skip`, nearest first
int children(const Tree4& T, int q, int skip, F3 o, F3 inv, float R, int32_t* ref) {
    const BNode4& W = T.node[q];
    int n = 0;
    float d[4];
    for (int c = 0; c < W.n; ++c) {
        if (c == skip) continue;
        const float e = cbox_dist(W.lo[c], W.hi[c], o, inv, R);
        if (e < INFINITY) { ref[n] = W.ref[c]; d[n] = e; ++n; }
    }
    for (int i = 1; i < n; ++i)
        for (int j = i; j > 0 && d[j] < d[j - 1]; --j) { std::swap(d[j], d[j - 1]); std::swap(ref[j], ref[j - 1]); }
    return n;
}
// walk the subtrees on the stack to completion (or until the ray closes)
void drain(const Tree4& T, const SceneK& S, ShadowTrav1& tv, Shadow1& r, const Spill& sp,
           std::vector<int32_t>& st, Count* c, int64_t* v) {
    while (!st.empty() && shadow1_open(S, r)) {
        int32_t x = st.back();
        st.pop_back();
        while (x >= 0) {
            ++*v;
            int32_t ref[4];
            const int n = children(T, x, -1, tv.o32, tv.inv, r.hhi, ref);
            for (int i = n - 1; i >= 1; --i) st.push_back(ref[i]);
            x = n ? ref[0] : kNoRef;
        }
        if (x != kNoRef) {
            c->units += (~x) & 7;
            if (S.bunitc) s1_units<true, PT_WF_LRNG != 0>(tv, S, &r, sp, x);
            else s1_units<false, PT_WF_LRNG != 0>(tv, S, &r, sp, x);
        }
    }
}
void shadow_topdown(const Tree4& T, const SceneK& S, F3 o32, int ogrp, Shadow1 r, const Spill& sp, Count* c,
                    const Shadow1& expect) {
    ++c->rays;
    ShadowTrav1 tv;
    tv.o32 = o32; tv.inv = rcp_dir(r.d32); tv.ogrp = ogrp;
    std::vector<int32_t> st;
    const BNode R0 = S.bnode[0];
    const F3 l = {R0.lo[0] - o32.x, R0.lo[1] - o32.y, R0.lo[2] - o32.z};
    const F3 h = {R0.hi[0] - o32.x, R0.hi[1] - o32.y, R0.hi[2] - o32.z};
    if (shadow1_open(S, r) && box_hit(l, h, tv.inv, r.hhi)) st.push_back(T.root);
    int64_t v = 0;
    drain(T, S, tv, r, sp, st, c, &v);
    c->visits += v;
    if (r.occ) { ++c->occluded; c->occ_visits += v; }
    if (r.occ != expect.occ || r.key2 != expect.key2 || r.leak != expect.leak) ++c->mismatches;
}
// bottom-up from the origin triangle's unit u (-1: not a BVH unit -> top-down)
void shadow_bottomup(const Tree4& T, const SceneK& S, int u, F3 o32, int ogrp, Shadow1 r, const Spill& sp,
                     Count* c, const Shadow1& expect) {
    if (u < 0) { shadow_topdown(T, S, o32, ogrp, r, sp, c, expect); return; }
    ++c->rays;
    ShadowTrav1 tv;
    tv.o32 = o32; tv.inv = rcp_dir(r.d32); tv.ogrp = ogrp;
    std::vector<int32_t> st;
    int64_t v = 0;
    // the origin's own leaf (its unit is the origin's triangle: coplanar, no hit — tested anyway)
    if (shadow1_open(S, r)) {
        const int32_t leaf = ~((u << 3) | 1);
        c->units += 1;
        if (S.bunitc) s1_units<true, PT_WF_LRNG != 0>(tv, S, &r, sp, leaf);
        else s1_units<false, PT_WF_LRNG != 0>(tv, S, &r, sp, leaf);
    }
    int32_t cur = T.leaf_parent[u], from = T.leaf_slot[u];
    while (cur >= 0 && shadow1_open(S, r)) {
        ++v;
        int32_t ref[4];
        const int n = children(T, cur, from, tv.o32, tv.inv, r.hhi, ref);
        for (int i = n - 1; i >= 0; --i) st.push_back(ref[i]);
        drain(T, S, tv, r, sp, st, c, &v);
        from = T.pslot[cur];
        cur = T.parent[cur];
    }
    c->visits += v;
    if (r.occ) { ++c->occluded; c->occ_visits += v; }
    if (r.occ != expect.occ || r.key2 != expect.key2 || r.leak != expect.leak) ++c->mismatches;
}
}  // namespace

extern "C" {
// out: top-down {rays visits units mismatches occluded occ_visits}, bottom-up {...}
int bu_count(const pt_scene_desc* d, const pt_render_params* p, int64_t* out) {
    HostScene H;
    if (!prepare_scene(d, &H).empty()) return -1;
    bind_host(&H);
    if (H.k.n_bnode == 0 || H.k.n_qnode == 0 || H.k.qstack > kBvhStack) return -3;
    Tree4 T;
    T.leaf_parent.assign(H.k.n_bunit, -1);
    T.leaf_slot.assign(H.k.n_bunit, -1);
    T.root = T.build(H, H.k.bvh_root, -1, -1);
    std::vector<int32_t> unit_of_tri(H.k.n_tri, -1);
    for (int u = 0; u < H.k.n_bunit; ++u) unit_of_tri[H.bunit[u].t[0]] = u;
    Count ctd, cbu;
    int32_t first, rows;
    if (!band_layout(p, &first, &rows)) return -2;
    const size_t n = (size_t)rows * p->width;
    std::vector<WfPath> W(n);
    std::vector<WfShadowQ> SQ(n);
    std::vector<WfClosestQ> CQ(n);
    std::vector<LaneJob> J(n);
    std::vector<D3> D0(n);
    for (int rr = 0; rr < rows; ++rr) {
        const int iy = first + rr * p->row_step;
        for (int ix = 0; ix < p->width; ++ix) {
            const size_t i = (size_t)rr * p->width + ix;
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
        for (size_t i = 0; i < n; ++i) {
            const Spill sp{W[i].sp, 1};
            for (int k = 0; k < kLightSamples; ++k) {
                if (!((want[i] >> k) & 1u)) continue;
                Shadow1 r;
                F3 o32;
                int ogrp;
                wf_get_shadow1(SQ[i], k, &o32, &ogrp, &r);
                const Shadow1 r0 = r;
                ShadowTrav1 T1;   // the shipped walk: the reference result
                int buf[kBvhStackLocal];
                const ShadowStack K{buf, 1};
                s1_init(T1, H.k, o32, ogrp, r, H.k.qroot);
                while (T1.ref != kNoRef) {
                    while (T1.ref >= 0) s1_qnode(T1, K, H.k, r);
                    if (T1.ref != kNoRef) {
                        if (H.k.bunitc) s1_units<true, PT_WF_LRNG != 0>(T1, H.k, &r, sp, T1.ref);
                        else s1_units<false, PT_WF_LRNG != 0>(T1, H.k, &r, sp, T1.ref);
                        T1.ref = s1_pop(T1, K, H.k, r);
                    }
                }
                shadow_topdown(T, H.k, o32, ogrp, r0, sp, &ctd, r);
                const int tri = W[i].tri;
                shadow_bottomup(T, H.k, tri >= 0 ? unit_of_tri[tri] : -1, o32, ogrp, r0, sp, &cbu, r);
                wf_put_shadow1(&SQ[i], r);
            }
            if (want[i] & kWfWantClosest) {   // the shipped closest walk (to keep the render going)
                ClosestAcc ca = wf_get_acc(CQ[i]);
                ClosestTrav T2;
                ClosestStackLocal L;
                const ClosestStack K = L.view();
                const WfClosestQ& q = CQ[i];
                ctrav_init(T2, H.k, F3{q.o[0], q.o[1], q.o[2]}, q.ogrp, F3{q.d[0], q.d[1], q.d[2]}, ca.b1,
                           H.k.qroot);
                while (T2.ref != kNoRef) {
                    while (T2.ref >= 0) ctrav_qnode(T2, K, H.k, &ca);
                    if (T2.ref != kNoRef) {
                        if (H.k.bunitc) ctrav_leaf<false, true>(T2, K, H.k, &ca, sp, nullptr);
                        else ctrav_leaf<false>(T2, K, H.k, &ca, sp, nullptr);
                    }
                }
                CQ[i].a1 = ca.a1; CQ[i].a2 = ca.a2; CQ[i].b1 = ca.b1; CQ[i].i1 = ca.i1;
            }
        }
    }
    const Count* cc[2] = {&ctd, &cbu};
    for (int j = 0; j < 2; ++j) {
        int64_t* o = out + 6 * j;
        o[0] = cc[j]->rays; o[1] = cc[j]->visits; o[2] = cc[j]->units; o[3] = cc[j]->mismatches;
        o[4] = cc[j]->occluded; o[5] = cc[j]->occ_visits;
    }
    return 0;
}
}
