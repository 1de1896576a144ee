// Dev experiment (host only): node visits of N-wide BVH walks (N = 4, 8) on
// the rays of a host wavefront render, against the shipped 4-wide QNode walks.
// The N-wide trees open the two-child tree's largest-area internal child
// until a node has N children (QBuilder's rule) and keep exact f32 boxes (no
// quantisation); children are visited nearest-first, the others stacked
// farthest-first, leaves tested with the shipped unit code, so each walk's
// result must equal the shipped walk's (checked).
//   g++ -O2 -std=c++17 -fPIC -shared -ffp-contract=off -o wide.so wide_bvh_count.cpp
// Driven by scripts/micro/wide_bvh_count.py.
#include "../../tests/hostcheck/pt_hostcheck.cpp"

#include <vector>

namespace {
struct WNode {
    int n;
    int32_t ref[8];
    float lo[8][3], hi[8][3];
};
struct WTree {
    std::vector<WNode> node;
    int32_t root = kNoRef;
    int32_t build(const HostScene& H, int32_t ref, int N) {
        if (ref < 0) return ref;
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
        while ((int)ch.size() < N) {
            int best = -1;
            for (int i = 0; i < (int)ch.size(); ++i)
                if (ch[i].ref >= 0 && (best < 0 || area(ch[i]) > area(ch[best]))) best = i;
            if (best < 0) break;
            const int32_t r = ch[best].ref;
            ch.erase(ch.begin() + best);
            open(r);
        }
        const int32_t me = (int32_t)node.size();
        node.push_back(WNode{});
        WNode W{};
        W.n = (int)ch.size();
        for (int c = 0; c < W.n; ++c) {
            for (int a = 0; a < 3; ++a) { W.lo[c][a] = ch[c].lo[a]; W.hi[c][a] = ch[c].hi[a]; }
        }
        for (int c = 0; c < W.n; ++c) W.ref[c] = build(H, ch[c].ref, N);
        node[me] = W;
        return me;
    }
};
// SAH-optimal collapse of the two-child tree into N-wide nodes (dynamic
// programme after Ylitie, Karras & Laine 2017, section 3.1): cost of a node
// visit 1 per unit of box area, of a leaf-unit test cl; D(x, j) = the least
// cost of subtree x spread over j child slots of its parent.
struct DpCollapse {
    const HostScene& H;
    int N;
    double cl;
    struct Box { float lo[3], hi[3]; };
    std::vector<std::vector<double>> D;     // [cnode][j], j = 1..N
    std::vector<std::vector<int>> how;      // [cnode][j]: 0 = one slot, -1 = as j-1, k > 0 = split (k, j-k)
    std::vector<double> A;                  // box area of each cnode
    static double area(const float* lo, const float* hi) {
        const double e0 = (double)hi[0] - lo[0], e1 = (double)hi[1] - lo[1], e2 = (double)hi[2] - lo[2];
        return e0 * e1 + e1 * e2 + e2 * e0;
    }
    DpCollapse(const HostScene& h, int n, double c) : H(h), N(n), cl(c) {
        const size_t m = H.cnode.size();
        D.assign(m, std::vector<double>(N + 1, 0.0));
        how.assign(m, std::vector<int>(N + 1, 0));
        A.assign(m, 0.0);
        std::vector<char> done(m, 0);
        // post-order over the internal nodes
        std::vector<std::pair<int, int>> st;
        if (H.k.bvh_root >= 0) st.push_back({H.k.bvh_root, 0});
        while (!st.empty()) {
            auto [r, phase] = st.back();
            st.pop_back();
            const CNode& C = H.cnode[r];
            if (phase == 0) {
                st.push_back({r, 1});
                if (C.c0 >= 0) st.push_back({C.c0, 0});
                if (C.c1 >= 0) st.push_back({C.c1, 0});
                continue;
            }
            float lo[3], hi[3];
            for (int a = 0; a < 3; ++a) { lo[a] = std::min(C.lo0[a], C.lo1[a]); hi[a] = std::max(C.hi0[a], C.hi1[a]); }
            A[r] = area(lo, hi);
            const double a0 = area(C.lo0, C.hi0), a1 = area(C.lo1, C.hi1);
            auto Dc = [&](int x, double ax, int j) { return x < 0 ? ax * cl : D[x][j]; };
            // as one wide node: its visit + the best spread of the N slots
            double node = INFINITY;
            for (int j = 1; j < N; ++j) node = std::min(node, Dc(C.c0, a0, j) + Dc(C.c1, a1, N - j));
            node += A[r];
            D[r][1] = node;
            how[r][1] = 0;
            for (int j = 2; j <= N; ++j) {
                D[r][j] = D[r][j - 1];
                how[r][j] = -1;
                for (int k = 1; k < j; ++k) {
                    const double c = Dc(C.c0, a0, k) + Dc(C.c1, a1, j - k);
                    if (c < D[r][j]) { D[r][j] = c; how[r][j] = k; }
                }
            }
        }
    }
    // the slots of subtree x spread over j slots: (ref, box) pairs
    void expand(int x, const float* lo, const float* hi, int j, std::vector<std::pair<int32_t, Box>>* out) const {
        Box b;
        for (int a = 0; a < 3; ++a) { b.lo[a] = lo[a]; b.hi[a] = hi[a]; }
        if (x < 0) { out->push_back({x, b}); return; }
        while (j > 1 && how[x][j] == -1) --j;
        if (j == 1 || how[x][j] == 0) { out->push_back({x, b}); return; }
        const int k = how[x][j];
        const CNode& C = H.cnode[x];
        expand(C.c0, C.lo0, C.hi0, k, out);
        expand(C.c1, C.lo1, C.hi1, j - k, out);
    }
    // children of the wide node made from cnode r
    void children(int r, std::vector<std::pair<int32_t, Box>>* out) const {
        const CNode& C = H.cnode[r];
        const double a0 = area(C.lo0, C.hi0), a1 = area(C.lo1, C.hi1);
        auto Dc = [&](int x, double ax, int j) { return x < 0 ? ax * cl : D[x][j]; };
        int best = 1;
        double bc = INFINITY;
        for (int j = 1; j < N; ++j) {
            const double c = Dc(C.c0, a0, j) + Dc(C.c1, a1, N - j);
            if (c < bc) { bc = c; best = j; }
        }
        expand(C.c0, C.lo0, C.hi0, best, out);
        expand(C.c1, C.lo1, C.hi1, N - best, out);
    }
};

struct WTreeDp {
    // builds WNodes with DpCollapse's child choice
    static int32_t build(WTree& T, const DpCollapse& P, int32_t ref) {
        if (ref < 0) return ref;
        std::vector<std::pair<int32_t, DpCollapse::Box>> ch;
        P.children(ref, &ch);
        const int32_t me = (int32_t)T.node.size();
        T.node.push_back(WNode{});
        WNode W{};
        W.n = (int)ch.size();
        for (int c = 0; c < W.n; ++c)
            for (int a = 0; a < 3; ++a) { W.lo[c][a] = ch[c].second.lo[a]; W.hi[c][a] = ch[c].second.hi[a]; }
        for (int c = 0; c < W.n; ++c) W.ref[c] = build(T, P, ch[c].first);
        T.node[me] = W;
        return me;
    }
};
int g_build = 0;      // 0: open the largest-area child (QBuilder's rule); 1: SAH dynamic programme
// bounce-0 occluder hint experiment: [0] bounce-0 shadow rays walked, [1] with a hint,
// [2] closed by the walk, [3] closed by the hint alone, [4] node visits of those,
// [5] node visits of all bounce-0 walks
int64_t g_hint[6];
std::vector<int> g_hint_unit;
bool g_hint_hit_pending = false;
ShadowTrav1 tv_dummy;
double g_cleaf = 0.33;

struct Count { int64_t queries = 0, visits = 0, boxes = 0, leaves = 0, units = 0, mismatches = 0, maxstack = 0; };

int g_order = 0;   // 0: all children nearest-first; 1: the nearest first, the rest in node order
// children of node q met within R, nearest first
int wide_children(const WTree& T, int q, F3 o, F3 inv, float R, int32_t* ref, float* d) {
    const WNode& W = T.node[q];
    int n = 0;
    for (int c = 0; c < W.n; ++c) {
        const float e = cbox_dist(W.lo[c], W.hi[c], o, inv, R);
        if (e < INFINITY) { ref[n] = W.ref[c]; d[n] = e; ++n; }
    }
    if (g_order == 1) {   // the nearest to the front, the others keep node order
        int m = 0;
        for (int i = 1; i < n; ++i) if (d[i] < d[m]) m = i;
        for (int j = m; j > 0; --j) { std::swap(d[j], d[j - 1]); std::swap(ref[j], ref[j - 1]); }
        return n;
    }
    for (int i = 1; i < n; ++i)   // insertion sort, ascending
        for (int j = i; j > 0 && d[j] < d[j - 1]; --j) { std::swap(d[j], d[j - 1]); std::swap(ref[j], ref[j - 1]); }
    return n;
}

void shadow_wide(const WTree& T, const SceneK& S, F3 o32, int ogrp, Shadow1 r, const Spill& sp, Count* c,
                 const Shadow1& expect) {
    ++c->queries;
    const F3 inv = rcp_dir(r.d32);
    const BNode R0 = S.bnode[0];
    const F3 l = {R0.lo[0] - o32.x, R0.lo[1] - o32.y, R0.lo[2] - o32.z};
    const F3 h = {R0.hi[0] - o32.x, R0.hi[1] - o32.y, R0.hi[2] - o32.z};
    std::vector<int32_t> st;
    if (shadow1_open(S, r) && box_hit(l, h, inv, r.hhi)) st.push_back(T.root);
    ShadowTrav1 tv;
    tv.o32 = o32; tv.inv = inv; tv.ogrp = ogrp;
    while (!st.empty() && shadow1_open(S, r)) {
        int32_t x = st.back();
        st.pop_back();
        while (x >= 0) {
            ++c->visits;
            c->boxes += T.node[x].n;
            int32_t ref[8];
            float d[8];
            const int n = wide_children(T, x, o32, inv, r.hhi, ref, d);
            for (int i = n - 1; i >= 1; --i) st.push_back(ref[i]);
            c->maxstack = std::max<int64_t>(c->maxstack, (int64_t)st.size());
            x = n ? ref[0] : kNoRef;
        }
        if (x != kNoRef) {
            ++c->leaves;
            c->units += (~x) & 7;
            if (S.bunitc) s1_units<true, PT_WF_LRNG != 0>(tv, S, &r, sp, x);
            else s1_units<false, PT_WF_LRNG != 0>(tv, S, &r, sp, x);
        }
    }
    if (r.occ != expect.occ || r.key2 != expect.key2 || r.leak != expect.leak) ++c->mismatches;
}

void closest_wide(const WTree& T, const SceneK& S, const WfClosestQ& q, ClosestAcc ca, const Spill& sp,
                  Count* c, const WfClosestQ& expect) {
    ++c->queries;
    ClosestTrav tv;
    const F3 o32{q.o[0], q.o[1], q.o[2]}, d32{q.d[0], q.d[1], q.d[2]};
    tv.o32 = o32; tv.d32 = d32; tv.inv = rcp_dir(d32); tv.ogrp = q.ogrp;
    std::vector<std::pair<int32_t, float>> st;
    if (node_dist(S, 0, o32, tv.inv, ca.b1) < INFINITY) st.push_back({T.root, 0.f});
    while (!st.empty()) {
        const auto e = st.back();
        st.pop_back();
        if (e.second > ca.b1) continue;
        int32_t x = e.first;
        while (x >= 0) {
            ++c->visits;
            c->boxes += T.node[x].n;
            int32_t ref[8];
            float d[8];
            const int n = wide_children(T, x, o32, tv.inv, ca.b1, ref, d);
            for (int i = n - 1; i >= 1; --i) st.push_back({ref[i], d[i]});
            c->maxstack = std::max<int64_t>(c->maxstack, (int64_t)st.size());
            x = n ? ref[0] : kNoRef;
        }
        if (x != kNoRef) {
            ++c->leaves;
            c->units += (~x) & 7;
            if (S.bunitc) ctrav_units<false, true>(tv, S, &ca, sp, nullptr, x);
            else ctrav_units<false>(tv, S, &ca, sp, nullptr, x);
        }
    }
    if (ca.i1 != expect.i1 || ca.b1 != expect.b1) ++c->mismatches;
}
}  // namespace

extern "C" {
// out: for N in {4, 8}: shadow {queries visits boxes leaves units mismatches maxstack}, closest {...}
// (14 per N), then the shipped walks' stats (8: hc_render_wavefront's walk_stats)
int wx_count(const pt_scene_desc* d, const pt_render_params* p, int64_t* out, int order) {
    g_order = order;
    if (const char* b = getenv("WX_BUILD")) g_build = atoi(b);
    if (const char* c = getenv("WX_CLEAF")) g_cleaf = atof(c);
    HostScene H;
    if (!prepare_scene(d, &H).empty()) return -1;
    bind_host(&H);
    if (H.k.n_bnode == 0 || H.k.n_qnode == 0 || H.k.qstack > kBvhStack) return -3;
    WTree T4, T8;
    if (g_build == 1) {
        const DpCollapse P4(H, 4, g_cleaf), P8(H, 8, g_cleaf);
        T4.root = WTreeDp::build(T4, P4, H.k.bvh_root);
        T8.root = WTreeDp::build(T8, P8, H.k.bvh_root);
    } else {
        T4.root = T4.build(H, H.k.bvh_root, 4);
        T8.root = T8.build(H, H.k.bvh_root, 8);
    }
    Count cs[2], cc[2];
    int64_t ws[8] = {0, 0, 0, 0, 0, 0, 0, 0};
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
    g_hint_unit.assign(n * 3, -1);
    memset(g_hint, 0, sizeof g_hint);
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
                ShadowTrav1 T;
                int buf[kBvhStackLocal];
                const ShadowStack K{buf, 1};
                s1_init(T, H.k, o32, ogrp, r, H.k.qroot);
                ++ws[0];
                // hint experiment: the unit that closed this slot's previous
                // bounce-0 ray k, tested alone first
                const bool b0 = W[i].b() == 0;
                if (b0) {
                    ++g_hint[0];
                    const int hu = g_hint_unit[i * 3 + k];
                    if (hu >= 0) {
                        ++g_hint[1];
                        Shadow1 rh = r0;
                        tv_dummy.o32 = o32; tv_dummy.ogrp = ogrp;
                        if (H.k.bunitc) shadow1_unit<PT_WF_LRNG != 0>(H.k, bvh_unit<true>(H.k, hu), o32, ogrp, &rh, sp);
                        else shadow1_unit<PT_WF_LRNG != 0>(H.k, bvh_unit<false>(H.k, hu), o32, ogrp, &rh, sp);
                        if (!shadow1_open(H.k, rh)) g_hint_hit_pending = true;
                    }
                }
                int64_t v0 = ws[1];
                int closer = -1;
                while (T.ref != kNoRef) {
                    while (T.ref >= 0) { s1_qnode(T, K, H.k, r); ++ws[1]; }
                    if (T.ref != kNoRef) {
                        ++ws[2];
                        ws[3] += (~T.ref) & 7;
                        const bool was_open = shadow1_open(H.k, r);
                        if (H.k.bunitc) s1_units<true, PT_WF_LRNG != 0>(T, H.k, &r, sp, T.ref);
                        else s1_units<false, PT_WF_LRNG != 0>(T, H.k, &r, sp, T.ref);
                        if (was_open && !shadow1_open(H.k, r)) closer = ~T.ref >> 3;
                        T.ref = s1_pop(T, K, H.k, r);
                    }
                }
                if (b0) {
                    if (!shadow1_open(H.k, r)) ++g_hint[2];          // bounce-0 rays closed by the BVH
                    if (g_hint_hit_pending) { ++g_hint[3]; g_hint[4] += ws[1] - v0; }   // visits a hint saves
                    g_hint[5] += ws[1] - v0;
                    g_hint_unit[i * 3 + k] = closer;   // (-1: open: no hint next time)
                }
                g_hint_hit_pending = false;
                shadow_wide(T4, H.k, o32, ogrp, r0, sp, &cs[0], r);
                shadow_wide(T8, H.k, o32, ogrp, r0, sp, &cs[1], r);
                wf_put_shadow1(&SQ[i], r);
            }
            if (want[i] & kWfWantClosest) {
                const ClosestAcc ca0 = wf_get_acc(CQ[i]);
                ClosestAcc ca = ca0;
                ClosestTrav T;
                ClosestStackLocal L;
                const ClosestStack K = L.view();
                const WfClosestQ q = CQ[i];
                ctrav_init(T, H.k, F3{q.o[0], q.o[1], q.o[2]}, q.ogrp, F3{q.d[0], q.d[1], q.d[2]}, ca.b1,
                           H.k.qroot);
                ++ws[4];
                while (T.ref != kNoRef) {
                    while (T.ref >= 0) { ctrav_qnode(T, K, H.k, &ca); ++ws[5]; }
                    if (T.ref != kNoRef) {
                        ++ws[6];
                        ws[7] += (~T.ref) & 7;
                        if (H.k.bunitc) ctrav_leaf<false, true>(T, K, H.k, &ca, sp, nullptr);
                        else ctrav_leaf<false>(T, K, H.k, &ca, sp, nullptr);
                    }
                }
                CQ[i].a1 = ca.a1; CQ[i].a2 = ca.a2; CQ[i].b1 = ca.b1; CQ[i].i1 = ca.i1;
                closest_wide(T4, H.k, q, ca0, sp, &cc[0], CQ[i]);
                closest_wide(T8, H.k, q, ca0, sp, &cc[1], CQ[i]);
            }
        }
    }
    for (int w = 0; w < 2; ++w) {
        const Count* a[2] = {&cs[w], &cc[w]};
        for (int j = 0; j < 2; ++j) {
            int64_t* o = out + w * 14 + j * 7;
            o[0] = a[j]->queries; o[1] = a[j]->visits; o[2] = a[j]->boxes; o[3] = a[j]->leaves;
            o[4] = a[j]->units; o[5] = a[j]->mismatches; o[6] = a[j]->maxstack;
        }
    }
    memcpy(out + 28, ws, sizeof ws);
    fprintf(stderr, "hint: bounce0_rays %lld with_hint %lld closed %lld hint_closes %lld visits_saved %lld bounce0_visits %lld all_shadow_visits %lld\n",
            (long long)g_hint[0], (long long)g_hint[1], (long long)g_hint[2], (long long)g_hint[3],
            (long long)g_hint[4], (long long)g_hint[5], (long long)ws[1]);
    return 0;
}
}
