// pt_prepare.h — host-side scene preparation: pt_scene_desc (include/pt_capi.h)
// -> the device records of pt_core.h, including the f32 filter's rigorous
// error constants.  Host-only C++.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/pt_capi.h"
#include "pt_core.h"

namespace pt {

struct HostScene {
    std::vector<double> kd;       // SceneK::kd
    std::vector<UnitF> unit;
    std::vector<UnitF> unit_eye;
    std::vector<UnitF> bunit;
    std::vector<UnitC> bunitc;   // bunit in 64-B form (empty: not representable)
    std::vector<BNode> bnode;
    std::vector<CNode> cnode;
    std::vector<QNode> qnode;
    std::vector<int32_t> tri_grp;
    std::vector<TriD> trid;
    std::vector<TriS> tris;
    std::vector<int32_t> tri_obj;
    std::vector<Mat> mat;
    std::vector<int32_t> light_tri;
    std::vector<double> light_cum;
    SceneK k{};   // pointers unset; constants filled
};

constexpr int kBvhMinTris = 64;   // objects this large are traversed through the BVH
// Units per leaf: 1 since the one-ray shadow walks (K5 512^2 x 64: 1 / 2 / 3 /
// 4 -> 93.2 / 94.6 / 100.9 / 107.8 ms; a unit test costs about a third of a
// node visit, but a leaf box prunes its unit before its record is loaded)
#ifndef PT_BVH_LEAF
#define PT_BVH_LEAF 1
#endif
constexpr int kBvhLeaf = PT_BVH_LEAF;   // units per leaf (at most 7: 3 bits of BNode::leaf)
#ifndef PT_BVH_BINS
#define PT_BVH_BINS 64   // K5: 16 / 64 bins -> 1130 / 1115 ms (shadow visits per ray 47.1 / 46.3)
#endif
constexpr int kBvhBins = PT_BVH_BINS;
constexpr int kBvhStackHost = 48;   // = kBvhStack (pt_path.h)

// outward rounding to f32
inline float f32_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = nextafterf(f, -INFINITY);
    return f;
}
inline float f32_upb(double x) {
    float f = (float)x;
    if ((double)f < x) f = nextafterf(f, INFINITY);
    return f;
}

// Binned-SAH BVH over H->bunit (reordered into leaf order), depth-first with
// skip links.  Unit boxes are in centred coordinates, inflated by
// delta = 64 u X: the f32 line the kernel traverses with (centred origin and
// direction rounded to f32) stays within ~20 u X of the exact line for every
// |t| <= 2 sqrt(3) X, slab arithmetic included, so a box test with the f32
// line never rejects a unit the exact line meets.
struct BvhBuilder {
    struct Item { double lo[3], hi[3], c[3]; };
    HostScene* H;
    double delta;
    std::vector<Item> it;
    std::vector<int> idx;
    std::vector<UnitF> ordered;

    static double area(const double* lo, const double* hi) {
        const double e0 = hi[0] - lo[0], e1 = hi[1] - lo[1], e2 = hi[2] - lo[2];
        return (e0 < 0 || e1 < 0 || e2 < 0) ? 0.0 : 2 * (e0 * e1 + e1 * e2 + e2 * e0);
    }
    int bin_of(double c, double lo, double ext) const {
        int q = (int)((c - lo) / ext * kBvhBins);
        return std::min(std::max(q, 0), kBvhBins - 1);
    }
    // SAH split position in [b, e) (partitions idx), or -1 for a leaf
    int split(int b, int e) {
        if (e - b <= kBvhLeaf) return -1;
        double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = b; i < e; ++i)
            for (int a = 0; a < 3; ++a) {
                clo[a] = std::min(clo[a], it[idx[i]].c[a]);
                chi[a] = std::max(chi[a], it[idx[i]].c[a]);
            }
        double best = INFINITY;
        int best_axis = -1, best_bin = -1;
        for (int a = 0; a < 3; ++a) {
            const double ext = chi[a] - clo[a];
            if (!(ext > 0)) continue;
            int bc[kBvhBins] = {0};
            double blo[kBvhBins][3], bhi[kBvhBins][3];
            for (int q = 0; q < kBvhBins; ++q)
                for (int z = 0; z < 3; ++z) { blo[q][z] = INFINITY; bhi[q][z] = -INFINITY; }
            for (int i = b; i < e; ++i) {
                const Item& I = it[idx[i]];
                const int q = bin_of(I.c[a], clo[a], ext);
                bc[q]++;
                for (int z = 0; z < 3; ++z) {
                    blo[q][z] = std::min(blo[q][z], I.lo[z]);
                    bhi[q][z] = std::max(bhi[q][z], I.hi[z]);
                }
            }
            double la[kBvhBins], lc[kBvhBins];
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            int c = 0;
            for (int q = 0; q < kBvhBins - 1; ++q) {   // left of boundary q+1
                c += bc[q];
                for (int z = 0; z < 3; ++z) { lo[z] = std::min(lo[z], blo[q][z]); hi[z] = std::max(hi[z], bhi[q][z]); }
                la[q] = area(lo, hi);
                lc[q] = c;
            }
            for (int z = 0; z < 3; ++z) { lo[z] = INFINITY; hi[z] = -INFINITY; }
            c = 0;
            for (int q = kBvhBins - 1; q > 0; --q) {   // right of boundary q
                c += bc[q];
                for (int z = 0; z < 3; ++z) { lo[z] = std::min(lo[z], blo[q][z]); hi[z] = std::max(hi[z], bhi[q][z]); }
                const double cost = la[q - 1] * lc[q - 1] + area(lo, hi) * c;
                if (lc[q - 1] > 0 && c > 0 && cost < best) { best = cost; best_axis = a; best_bin = q; }
            }
        }
        int mid = -1;
        if (best_axis >= 0) {
            const int a = best_axis;
            const double lo = clo[a], ext = chi[a] - clo[a];
            mid = (int)(std::partition(idx.begin() + b, idx.begin() + e,
                                       [&](int i) { return bin_of(it[i].c[a], lo, ext) < best_bin; }) -
                        idx.begin());
        }
        if (mid <= b || mid >= e) mid = (b + e) / 2;   // coincident centroids: halve
        return mid;
    }
    int depth = 0;
    int build(int b, int e, int level = 0) {   // returns the subtree's root node
        depth = std::max(depth, level);
        BNode N{};
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = b; i < e; ++i)
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], it[idx[i]].lo[a]);
                hi[a] = std::max(hi[a], it[idx[i]].hi[a]);
            }
        for (int a = 0; a < 3; ++a) {
            N.lo[a] = f32_down(lo[a] - delta);
            N.hi[a] = f32_upb(hi[a] + delta);
        }
        N.leaf = -1;
        const int node = (int)H->bnode.size();
        H->bnode.push_back(N);
        const int mid = split(b, e);
        if (mid < 0) {
            H->bnode[node].leaf = ((int32_t)ordered.size() << 3) | (e - b);
            for (int i = b; i < e; ++i) ordered.push_back(H->bunit[idx[i]]);
        } else {
            build(b, mid, level + 1);
            build(mid, e, level + 1);
        }
        H->bnode[node].skip = (int)H->bnode.size();   // the node after this subtree
        return node;
    }
};

// 4-wide quantised form of the two-child tree (QNode): each node takes the
// two children of a binary node and keeps opening its internal child of
// largest surface area until it has 4 children.  Returns the subtree's QNode
// index (or the leaf code); *stack = the most stack entries a nearest-first
// walk of the subtree can hold (3 per level at most).
struct QBuilder {
    HostScene* H;
    double X;   // the BVH frame's half extent (the boxes' inflation is 64 u X)
    struct Child { int32_t ref; float lo[3], hi[3]; };
    static double area(const Child& c) {
        const double e0 = (double)c.hi[0] - c.lo[0], e1 = (double)c.hi[1] - c.lo[1],
                     e2 = (double)c.hi[2] - c.lo[2];
        return e0 * e1 + e1 * e2 + e2 * e0;
    }
    // one axis: grid origin / step / codes with exact f32 decode.  An absent
    // child is the empty box lo 255, hi 0: a line's slab parameters on the
    // axis are fma(255, A, B) and B (A = step inv, B = (org - o) inv), and the
    // walks test no child reference, so the box must stay empty after
    // rounding: 255 step has to exceed half an ulp of |org - o| <= 4 X, i.e.
    // 255 step >= 2^-20 X (4x margin).  The 64 u X inflation of every box
    // already gives 255 step >= 2^-19 X; the check keeps it a checked fact
    // (a node that failed it would send the scene to the single kernel).
    static bool quantise(const Child* ch, int n, int a, QNode* Q, double X) {
        double plo = INFINITY, phi = -INFINITY;
        for (int c = 0; c < n; ++c) { plo = std::min(plo, (double)ch[c].lo[a]); phi = std::max(phi, (double)ch[c].hi[a]); }
        int e = (int)floor(log2(std::max(phi - plo, 1e-30) / 255.0)) - 1;
        for (; e < 127; ++e) {
            if (e < -126) continue;
            const double step = ldexp(1.0, e);
            const double org = floor(plo / step) * step;
            if ((double)(float)org != org || ceil((phi - org) / step) > 255.0) continue;
            bool ok = true;
            uint32_t lo = 0, hi = 0;
            for (int c = 0; c < n && ok; ++c) {
                const double ql = floor(((double)ch[c].lo[a] - org) / step);
                const double qh = ceil(((double)ch[c].hi[a] - org) / step);
                const float dl = fmaf((float)ql, (float)step, (float)org);   // the kernel's decode
                const float dh = fmaf((float)qh, (float)step, (float)org);
                ok = ql >= 0 && qh <= 255 && (double)dl == org + ql * step &&
                     (double)dh == org + qh * step && dl <= ch[c].lo[a] && dh >= ch[c].hi[a];
                lo |= (uint32_t)ql << (8 * c);
                hi |= (uint32_t)qh << (8 * c);
            }
            if (!ok) continue;
            if (n < 4 && !(255.0 * step >= ldexp(X, -20))) return false;
            for (int c = n; c < 4; ++c) lo |= 255u << (8 * c);   // no child: an empty box
            Q->org[a] = (float)org;
            Q->ex |= (uint32_t)(e + 127) << (8 * a);
            Q->qlo[a] = lo;
            Q->qhi[a] = hi;
            return true;
        }
        return false;
    }
    bool failed = false;   // some node could not be quantised exactly
    int32_t build(int32_t ref, int* stack) {
        *stack = 0;
        if (ref < 0) return ref;   // a leaf
        std::vector<Child> ch;
        auto open = [&](int32_t r) {
            const CNode& C = H->cnode[r];
            Child a{C.c0, {C.lo0[0], C.lo0[1], C.lo0[2]}, {C.hi0[0], C.hi0[1], C.hi0[2]}};
            Child b{C.c1, {C.lo1[0], C.lo1[1], C.lo1[2]}, {C.hi1[0], C.hi1[1], C.hi1[2]}};
            ch.push_back(a);
            ch.push_back(b);
        };
        open(ref);
        while (ch.size() < 4) {
            int best = -1;
            for (int i = 0; i < (int)ch.size(); ++i)
                if (ch[i].ref >= 0 && (best < 0 || area(ch[i]) > area(ch[best]))) best = i;
            if (best < 0) break;
            const int32_t r = ch[best].ref;
            ch.erase(ch.begin() + best);
            open(r);
        }
        const int32_t q = (int32_t)H->qnode.size();
        H->qnode.push_back(QNode{});
        QNode Q{};
        for (int c = 0; c < 4; ++c) Q.ref[c] = kNoRef;
        for (int a = 0; a < 3; ++a)
            if (!quantise(ch.data(), (int)ch.size(), a, &Q, X)) failed = true;
        int deepest = 0;
        for (int c = 0; c < (int)ch.size() && !failed; ++c) {
            int sub = 0;
            const int32_t r = build(ch[c].ref, &sub);
            Q.ref[c] = r;
            deepest = std::max(deepest, sub);
        }
        *stack = deepest + (int)ch.size() - 1;
        H->qnode[q] = Q;
        return q;
    }
};

inline void build_bvh(HostScene* H, double X) {
    H->bnode.clear();
    H->cnode.clear();
    H->qnode.clear();
    SceneK& K = H->k;
    K.n_bnode = 0;
    K.n_bunit = (int32_t)H->bunit.size();
    K.bvh_min_tri = K.n_tri;
    K.bvh_min_obj = K.n_obj;
    K.bvh_depth = 0;
    K.n_qnode = 0;
    K.qroot = kNoRef;
    K.qstack = kBvhStackHost + 1;   // no 4-wide form
    const int n = (int)H->bunit.size();
    if (n == 0) return;
    BvhBuilder B;
    B.H = H;
    B.delta = 64.0 / 16777216.0 * X;
    B.it.resize(n);
    for (int i = 0; i < n; ++i) {
        const UnitF& U = H->bunit[i];
        BvhBuilder::Item& I = B.it[i];
        for (int a = 0; a < 3; ++a) { I.lo[a] = INFINITY; I.hi[a] = -INFINITY; }
        for (int m = 0; m < U.count; ++m) {
            const TriD& T = H->trid[U.t[m]];
            K.bvh_min_tri = std::min(K.bvh_min_tri, U.t[m]);
            K.bvh_min_obj = std::min(K.bvh_min_obj, U.obj);
            const double* vs[3] = {T.v1, T.v2, T.v3};
            for (int v = 0; v < 3; ++v)
                for (int a = 0; a < 3; ++a) {
                    const double x = vs[v][a] - K.center[a];
                    I.lo[a] = std::min(I.lo[a], x);
                    I.hi[a] = std::max(I.hi[a], x);
                }
        }
        for (int a = 0; a < 3; ++a) I.c[a] = 0.5 * (I.lo[a] + I.hi[a]);
        B.idx.push_back(i);
    }
    B.ordered.reserve(n);
    B.build(0, n);
    const int total = (int)H->bnode.size();
    for (BNode& N : H->bnode)
        if (N.skip >= total) N.skip = -1;
    H->bunit.swap(B.ordered);
    K.n_bnode = total;
    K.bvh_depth = B.depth;
    // two-child form: internal node i has children i + 1 and bnode[i + 1].skip
    std::vector<int32_t> cidx(total, -1);
    for (int i = 0; i < total; ++i)
        if (H->bnode[i].leaf < 0) cidx[i] = (int32_t)H->cnode.size(), H->cnode.push_back(CNode{});
    auto ref = [&](int i) { return H->bnode[i].leaf >= 0 ? ~H->bnode[i].leaf : cidx[i]; };
    for (int i = 0; i < total; ++i) {
        if (cidx[i] < 0) continue;
        const int a = i + 1, b = H->bnode[a].skip;
        CNode& C = H->cnode[cidx[i]];
        for (int k = 0; k < 3; ++k) {
            C.lo0[k] = H->bnode[a].lo[k];
            C.hi0[k] = H->bnode[a].hi[k];
            C.lo1[k] = H->bnode[b].lo[k];
            C.hi1[k] = H->bnode[b].hi[k];
        }
        C.c0 = ref(a);
        C.c1 = ref(b);
    }
    K.bvh_root = ref(0);
    QBuilder QB{H, X};
    int qs = 0;
    const int32_t qr = QB.build(K.bvh_root, &qs);
    if (!QB.failed) {
        K.qroot = qr;
        K.n_qnode = (int32_t)H->qnode.size();
        K.qstack = qs + 1;
    } else {
        H->qnode.clear();
    }
}

inline D3 tri_vertex(const pt_scene_desc* d, int t, int v) {
    return ld3(d->tri_v + 9 * t + 3 * v);
}

// rotate((0,1,0), arccos(n_y), .) matrix, main.py:148-162 literal formula
inline void rotation_for_normal(const double* n, TriS* R) {
    const double angle = acos(0.0 * n[0] + 1.0 * n[1] + 0.0 * n[2]);
    const double a = cos(angle / 2.0), sn = sin(angle / 2.0);
    const double b = -0.0 * sn, c = -1.0 * sn, dd = -0.0 * sn;
    const double aa = a * a, bb = b * b, cc = c * c, d2 = dd * dd;
    const double ac = a * c, bd = b * dd;
    R->r00 = aa + bb - cc - d2;
    R->r02 = 2 * (bd - ac);
    R->r11 = aa + cc - bb - d2;
    R->r20 = 2 * (bd + ac);
    R->r22 = aa + d2 - bb - cc;
}

inline float f32_up(double x) {   // round to f32, never below x (x >= 0)
    float f = (float)x;
    if ((double)f < x) f = nextafterf(f, INFINITY);
    return f;
}

// The 64-B form of the BVH units (UnitC, pt_core.h), when every unit is a
// single non-degenerate triangle: eo and eh rounded up to bfloat16, eq / qhi
// the maxima over the units (each unit's own bound is <= what the kernel
// uses: conservative), ed derived from g in the kernel, the object read from
// tri_obj.
inline void build_unitc(HostScene* H) {
    SceneK& K = H->k;
    H->bunitc.clear();
    K.bvh_eh = K.bvh_eq = K.bvh_qhi = 0.f;
    K.bvh_obj1 = -1;
    if (H->bunit.empty()) return;
    int obj1 = H->bunit[0].obj;
    for (const UnitF& U : H->bunit) {
        if (U.count != 1 || !(U.eh >= 0.f) || !(U.eh < 1e30f) || !(U.eo > 0.f) || !(U.eo < 1e30f) ||
            !(U.qhi < INFINITY))
            return;
        K.bvh_eh = std::max(K.bvh_eh, U.eh);
        K.bvh_eq = std::max(K.bvh_eq, U.eq);
        K.bvh_qhi = std::max(K.bvh_qhi, U.qhi);
        if (U.obj != obj1) obj1 = -1;
        // ed must not exceed what the kernel derives from g
        if (!(U.ed <= U.g * kEdPerG)) return;
    }
    K.bvh_obj1 = obj1;
    H->bunitc.resize(H->bunit.size());
    for (size_t i = 0; i < H->bunit.size(); ++i) {
        const UnitF& U = H->bunit[i];
        UnitC& C = H->bunitc[i];
        for (int a = 0; a < 3; ++a) C.n[a] = U.n[a];
        C.cn = U.cn;
        C.tri = U.tri[0];
        C.t = U.t[0];
        C.grp = U.grp;
        C.g = U.g;
        C.eoeh = bf16_up(U.eo) | bf16_up(U.eh) << 16;
    }
}

// Returns "" on success, else an error message.
inline std::string prepare_scene(const pt_scene_desc* d, HostScene* H) {
    if (!d) return "null scene descriptor";
    if (d->n_tri <= 0 || d->n_obj_tri < 0 || d->n_obj_tri >= d->n_tri)
        return "need 0 <= n_obj_tri < n_tri (the light must have triangles)";
    if (d->n_obj <= 0) return "need at least one object";
    if (!d->tri_v || !d->tri_n || !d->tri_area || !d->tri_obj || !d->mat)
        return "null array in scene descriptor";
    const int T = d->n_tri;
    for (int t = 0; t < T; ++t) {
        const int o = d->tri_obj[t];
        if (t < d->n_obj_tri ? (o < 0 || o >= d->n_obj) : (o != d->n_obj))
            return "tri_obj out of range (objects first, then light = n_obj)";
    }
    // Two coordinate frames for the f32 filter, each a box centre and half
    // extent X bounding every origin expressed in it:
    //   "all" (C, X): the triangles and the eye — primary rays start at the
    //       eye; the BVH records and unit_eye use it;
    //   "surface" (Cs, Xs): the triangles alone — every later ray starts on a
    //       scene surface; the uniform units (`unit`) use it, so their error
    //       bounds, which grow with X, are not inflated by the eye's distance
    //       (Cornell: Xs = 8.1 vs X = 19.2).
    double lo[3], hi[3];
    for (int i = 0; i < 3; ++i) lo[i] = INFINITY, hi[i] = -INFINITY;
    for (int t = 0; t < T; ++t)
        for (int v = 0; v < 3; ++v)
            for (int i = 0; i < 3; ++i) {
                const double x = d->tri_v[9 * t + 3 * v + i];
                if (!isfinite(x)) return "non-finite vertex";
                lo[i] = std::min(lo[i], x);
                hi[i] = std::max(hi[i], x);
            }
    for (int i = 0; i < 3; ++i)
        if (!isfinite(d->eye[i])) return "non-finite eye";
    double Cs[3], Xs = 0.0;
    for (int i = 0; i < 3; ++i) {
        Cs[i] = 0.5 * (lo[i] + hi[i]);
        Xs = std::max(Xs, 0.5 * (hi[i] - lo[i]));
    }
    Xs = Xs * 1.001 + 1e-6;
    for (int i = 0; i < 3; ++i) {
        lo[i] = std::min(lo[i], d->eye[i]);
        hi[i] = std::max(hi[i], d->eye[i]);
    }
    double C[3], X = 0.0;
    for (int i = 0; i < 3; ++i) {
        C[i] = 0.5 * (lo[i] + hi[i]);
        X = std::max(X, 0.5 * (hi[i] - lo[i]));
    }
    X = X * 1.001 + 1e-6;
    const double u = 1.0 / 16777216.0;   // f32 unit roundoff

    H->trid.assign(T, TriD{});
    H->tris.assign(T, TriS{});
    H->tri_obj.assign(d->tri_obj, d->tri_obj + T);
    // per-triangle f32 filter data, before grouping into units
    struct PlaneD { double n[3], cn, eh, eq; bool ok; };
    std::vector<PlaneD> pl(T);
    std::vector<TriB> tb(T);
    struct TriE { float eo, ed, g; };   // barycentric bound coefficients
    std::vector<TriE> te(T);
    std::vector<PlaneD> pls(T);          // the same in the surface frame
    std::vector<TriB> tbs(T);
    std::vector<TriE> tes(T);
    const D3 Cd = d3(C[0], C[1], C[2]), Cds = d3(Cs[0], Cs[1], Cs[2]);
    auto l1 = [](double a, double b, double c) { return fabs(a) + fabs(b) + fabs(c); };
    // bound on |aff3(f32(G), f32(C), f32(x)) - (G.x + C)| for |x_i| <= Xb (see below)
    auto aff_err = [u](const double G[3], double Cc, double Xb) {
        double e = fabs((double)(float)Cc - Cc), g1 = 0.0;
        int k = 0;
        for (int i = 0; i < 3; ++i) {
            const double g = (double)(float)G[i];
            e += fabs(g - G[i]) * Xb;
            if (g != 0.0) {
                e += u * fabs(g) * Xb;
                ++k;
            }
            g1 += fabs(g);
        }
        return e + k * u * (g1 * Xb + fabs((double)(float)Cc)) * (1 + 4 * u) + 1e-30;
    };
    const double s = 1.25;   // safety factor over the first-order bounds below
    // The barycentric forms of triangle t in frame f (0: "all", 1: "surface")
    // with its vertices taken from vertex `rot` on (rot = 1: v2, v3, v1;
    // 2: v3, v1, v2): beta = weight of the second, gamma of the third.  The
    // inside test (every weight > 0) does not depend on the labelling.
    // Returns false for a degenerate triangle (forms left zero).
    auto tri_forms = [&](int t, int rot, int f, TriB* B, TriE* BE) {
        *B = TriB{};
        *BE = TriE{};
        const D3 vv[3] = {tri_vertex(d, t, 0), tri_vertex(d, t, 1), tri_vertex(d, t, 2)};
        const D3 Cf = f ? Cds : Cd;
        const double Xf = f ? Xs : X;
        const D3 w1 = vv[rot % 3] - Cf, w2 = vv[(rot + 1) % 3] - Cf, w3 = vv[(rot + 2) % 3] - Cf;
        const D3 e1 = w2 - w1, e2 = w3 - w1, N = cross(e1, e2);
        const double NN = dot(N, N);
        if (!(NN > 0.0)) return false;
        const D3 gb = cross(e2, N) * (1.0 / NN), gc = cross(N, e1) * (1.0 / NN);
        const double cb = -dot(gb, w1), cc = -dot(gc, w1);
        B->gb[0] = (float)gb.x; B->gb[1] = (float)gb.y; B->gb[2] = (float)gb.z; B->cb = (float)cb;
        B->gc[0] = (float)gc.x; B->gc[1] = (float)gc.y; B->gc[2] = (float)gc.z; B->cc = (float)cc;
        // Error bounds of the kernel's f32 forms (aff3 / lin3, pt_core.h):
        // an affine form g.x + c at |x_i| <= X with g = f32(G), c = f32(C),
        // x = f32(x_exact), evaluated as aff3's fma chain, errs by at most
        //   sum_i |g_i - G_i| X + |c - C|           (coefficient rounding, exact)
        // + u sum_i |g_i| X                        (input rounding)
        // + k u (|g|_1 X + |c|)                    (one rounding per fma
        //   whose product is nonzero: an fma with g_i = 0 returns its addend
        //   exactly), k = nonzero coefficients;
        // a direction form g.d (|d_i| <= 1, lin3) likewise with X = 1, c = 0.
        // For a general plane this is <= 5u(|g|_1 X + |c|); for an
        // axis-aligned one (walls: g one-hot and exact) ~2u(X + |c|), which
        // decides most tests of lines grazing their edges in f32.  The
        // safety factor s covers second-order terms and the reference's own
        // f64 rounding (~1e-16 relative).
        const double gbd[3] = {gb.x, gb.y, gb.z}, gcd[3] = {gc.x, gc.y, gc.z};
        const double gb1 = l1(B->gb[0], B->gb[1], B->gb[2]) * (1 + 4 * u);
        const double gc1 = l1(B->gc[0], B->gc[1], B->gc[2]) * (1 + 4 * u);
        // x2: one bound for beta, gamma (error <= del/2) and alpha (<= del)
        BE->eo = f32_up(2 * (s * std::max(aff_err(gbd, cb, Xf), aff_err(gcd, cc, Xf)) + 8 * u));
        BE->ed = f32_up(2 * s * std::max(aff_err(gbd, 0.0, 1.0), aff_err(gcd, 0.0, 1.0)));
        BE->g = f32_up(2 * std::max(gb1, gc1) * (1 + 1e-3));
        return true;
    };
    for (int t = 0; t < T; ++t) {
        const D3 v1 = tri_vertex(d, t, 0), v2 = tri_vertex(d, t, 1), v3 = tri_vertex(d, t, 2);
        TriD& E = H->trid[t];
        // reference plane normal: normalize(cross(v1 - v2, v3 - v2)), utils.py:109-111
        const D3 cr = cross(v1 - v2, v3 - v2);
        const double cn = sqrt(dot(cr, cr));
        E.vp[0] = cr.x / cn; E.vp[1] = cr.y / cn; E.vp[2] = cr.z / cn;  // v / norm(v)
        E.cvp = E.vp[0] * v1.x + E.vp[1] * v1.y + E.vp[2] * v1.z;
        const D3 e12 = v1 - v2, e23 = v2 - v3, e31 = v3 - v1;
        const double* src[6] = {&v1.x, &v2.x, &v3.x, &e12.x, &e23.x, &e31.x};
        double* dst[6] = {E.v1, E.v2, E.v3, E.e12, E.e23, E.e31};
        for (int j = 0; j < 6; ++j) memcpy(dst[j], src[j], 3 * sizeof(double));

        TriS& R = H->tris[t];
        memcpy(R.n, d->tri_n + 3 * t, 3 * sizeof(double));
        rotation_for_normal(R.n, &R);

        // f32 filter data in centred coordinates, once per frame (f = 0: "all",
        // f = 1: "surface"); only the constants and the X-dependent bounds
        // differ between the frames
        for (int f = 0; f < 2; ++f) {
            const D3 Cf = f ? Cds : Cd;
            const double Xf = f ? Xs : X;
            const D3 w1 = v1 - Cf;
            PlaneD& P = f ? pls[t] : pl[t];
            const bool formed = tri_forms(t, 0, f, f ? &tbs[t] : &tb[t], f ? &tes[t] : &te[t]);
            P.ok = (cn > 0.0) && formed && isfinite(cn);
            if (!P.ok) {   // degenerate: the reference's NaN normal never hits
                (f ? tbs[t] : tb[t]) = TriB{};
                (f ? tes[t] : te[t]) = TriE{};
                continue;
            }
            const double chn = -(E.vp[0] * w1.x + E.vp[1] * w1.y + E.vp[2] * w1.z);
            for (int i = 0; i < 3; ++i) P.n[i] = E.vp[i];
            P.cn = chn;
            const double nd3[3] = {E.vp[0], E.vp[1], E.vp[2]};
            const double n1 = l1((float)P.n[0], (float)P.n[1], (float)P.n[2]) * (1 + 4 * u);
            P.eh = s * aff_err(nd3, chn, Xf);
            // q's own error, plus 8u n1 >= 8u|q| covering the rounding of 1/q and t
            P.eq = s * aff_err(nd3, 0.0, 1.0) + 8 * u * n1;
        }
    }
    // coplanar groups: triangle t joins the group of an earlier
    // representative r when every vertex of t lies within 1e-12 of r's plane
    // and every vertex of r within 1e-12 of t's plane (f64).  Members' planes
    // then agree to ~1e-9 anywhere in the scene box, so a line from a hit
    // point on one member meets another member's plane at
    // |t| <= 1e-9 / |q| < 1e-4 (|q| > 1e-5, else the reference's parallel
    // reject fires): squared distance < 1e-5, never a usable hit.  Candidate
    // representatives are found by hashing the quantised plane; a missed
    // grouping only costs speed, never correctness.
    H->tri_grp.assign(T, -1);
    {
        std::unordered_map<uint64_t, std::vector<int>> buckets;
        int n_groups = 0;
        std::vector<int> grp_of_rep;
        auto plane_dist = [&](int plane_t, D3 x) {
            const TriD& P = H->trid[plane_t];
            return fabs(P.vp[0] * x.x + P.vp[1] * x.y + P.vp[2] * x.z - P.cvp);
        };
        for (int t = 0; t < T; ++t) {
            int32_t& G = H->tri_grp[t];
            G = -2 - t;   // unique, never equal to an origin's -1
            if (!pl[t].ok) continue;   // degenerate
            const TriD& E = H->trid[t];
            double k[4] = {E.vp[0], E.vp[1], E.vp[2], E.cvp};
            // canonical sign: first significant normal component positive
            const int lead = fabs(k[0]) > 1e-3 ? 0 : (fabs(k[1]) > 1e-3 ? 1 : 2);
            if (k[lead] < 0) for (double& x : k) x = -x;
            uint64_t key = 1469598103934665603ull;
            for (int i = 0; i < 4; ++i) {
                const int64_t qv = (int64_t)llround(k[i] * (i < 3 ? 1e5 : 1e3));
                key = (key ^ (uint64_t)qv) * 1099511628211ull;
            }
            std::vector<int>& reps = buckets[key];
            for (int r : reps) {
                bool ok = true;
                for (int v = 0; v < 3 && ok; ++v)
                    ok = plane_dist(r, tri_vertex(d, t, v)) <= 1e-12 &&
                         plane_dist(t, tri_vertex(d, r, v)) <= 1e-12;
                if (ok) { G = H->tri_grp[r]; break; }
            }
            if (G < 0) {
                G = n_groups++;
                reps.push_back(t);
            }
        }
    }
    // plane units: consecutive triangles of one object in one coplanar group
    // share a unit (at most 2).  The unit's plane is its first triangle's; the
    // members' planes agree to 1e-12 over the box, covered by +1e-9 slack.
    // Objects with at least kBvhMinTris triangles ("meshes") go to the BVH;
    // the others stay in the uniform list every lane walks in scene order.
    std::vector<int32_t> obj_ntri(d->n_obj, 0);
    for (int t = 0; t < d->n_obj_tri; ++t) obj_ntri[d->tri_obj[t]]++;
    auto in_bvh = [&](int t) { return t < d->n_obj_tri && obj_ntri[d->tri_obj[t]] >= kBvhMinTris; };
    H->unit.clear();
    H->unit_eye.clear();
    H->bunit.clear();
    // Parallelogram pairs ("quads", e.g. the reference's rectangles split
    // along a diagonal): triangles t, t + 1 share two vertices i1, i2 (the
    // diagonal), t's third vertex k and t + 1's third vertex D satisfy
    // D = i1 + i2 - k.  Then t + 1's weights at (i1, i2, D) are
    // (1 - l_i2, 1 - l_i1, -l_k) in t's weights l, so with t's forms taken
    // from vertex rot on (tri_forms: the order i2, k, i1, so alpha = l_i2,
    // beta = l_k, gamma = l_i1) they are (beta + gamma, 1 - gamma, -beta): the
    // render loop tests both members from one pair of forms (pt_path.h
    // quad_m).  Returns rot, or -1 when the
    // pair is no parallelogram; *dev = |i1 + i2 - k - D|_1 (f64).
    auto quad_rot = [&](int t, double* dev) {
        D3 a[3], b[3];
        for (int v = 0; v < 3; ++v) a[v] = tri_vertex(d, t, v), b[v] = tri_vertex(d, t + 1, v);
        auto same = [](D3 p, D3 q) { return p.x == q.x && p.y == q.y && p.z == q.z; };
        int k = -1, ns = 0;
        bool used[3] = {false, false, false};
        for (int i = 0; i < 3; ++i) {
            bool sh = false;
            for (int j = 0; j < 3 && !sh; ++j)
                if (!used[j] && same(a[i], b[j])) { used[j] = sh = true; ++ns; }
            if (!sh) k = i;
        }
        if (ns != 2 || k < 0) return -1;
        int jd = 0;
        while (used[jd]) ++jd;
        const D3 i1 = a[(k + 1) % 3], i2 = a[(k + 2) % 3];
        const D3 e = ((i1 + i2) - a[k]) - b[jd];
        double sc = 0.0;
        for (const D3& q : {i1, i2, a[k], b[jd]}) sc = std::max(sc, l1(q.x, q.y, q.z));
        *dev = l1(e.x, e.y, e.z) + 8e-16 * sc;   // + the rounding of the check itself
        if (!(*dev <= 1e-12 * (sc + 1.0))) return -1;
        return (k + 2) % 3;   // rotated order (v[rot], v[rot+1], v[rot+2]): v[k] second
    };
    // one unit record in frame f (0: all, 1: surface) for triangles t (, t + 1)
    auto make_unit = [&](int t, bool pair, int f, int rot = -1, double dev = 0.0) {
        const std::vector<PlaneD>& PL = f ? pls : pl;
        const std::vector<TriB>& TB = f ? tbs : tb;
        const std::vector<TriE>& TE = f ? tes : te;
        UnitF U{};
        const PlaneD& P = PL[t];
        U.count = pair ? 2 : 1;
        U.grp = H->tri_grp[t];
        U.obj = d->tri_obj[t];
        U.tri[0] = TB[t];
        U.tri[1] = pair ? TB[t + 1] : TriB{};
        U.t[0] = t;
        U.t[1] = pair ? t + 1 : t;
        U.quad = pair ? -1 : 0;   // a pair that is no parallelogram / a single
        U.eo = TE[t].eo;
        U.ed = TE[t].ed;
        U.g = TE[t].g;
        if (!P.ok) {   // degenerate: dt = -inf -> certain miss, never a candidate
            U.eh = -INFINITY;
            U.eq = 0.f;
            U.qhi = INFINITY;
        } else {
            double eh = P.eh, eq = P.eq;
            if (pair) {
                eh = std::max(eh, PL[t + 1].eh) + 1e-9;
                eq = std::max(eq, PL[t + 1].eq) + 1e-9;
                // one bound for both members (the kernel evaluates del once per
                // ray and unit)
                U.eo = f32_up(std::max(TE[t].eo, TE[t + 1].eo) + 2e-9);
                U.ed = std::max(TE[t].ed, TE[t + 1].ed);
                U.g = std::max(TE[t].g, TE[t + 1].g);
            }
            if (rot >= 0) {   // a quad: the first member's forms from vertex rot on
                TriB B0;
                TriE E0;
                tri_forms(t, rot, f, &B0, &E0);
                U.tri[0] = B0;
                U.quad = 1;
                // + the quad relation's own mismatch: moving the second
                // member's vertex D by dev changes its weights at x by at most
                // dev |grad l|_1 |l_D(x)| <= dev (g / 2) (3 (g / 2) X + 1) in
                // the frame's box (x2: eo's convention)
                const double gm = std::max(E0.g, TE[t + 1].g), Xf = f ? Xs : X;
                U.eo = f32_up(std::max((double)E0.eo, (double)TE[t + 1].eo) + 2e-9 +
                              dev * gm * (1.5 * gm * Xf + 1.0));
                U.ed = std::max(E0.ed, TE[t + 1].ed);
                U.g = std::max(E0.g, TE[t + 1].g);
            }
            for (int i = 0; i < 3; ++i) U.n[i] = (float)P.n[i];
            U.cn = (float)P.cn;
            U.eh = f32_up(eh);
            U.eq = f32_up(eq);
            U.qhi = f32_up((1e-5 + eq) * (1 + 1e-4));
        }
        return U;
    };
    for (int part = 0; part < 2; ++part) {
        const int t_begin = part == 0 ? 0 : d->n_obj_tri, t_end = part == 0 ? d->n_obj_tri : T;
        for (int t = t_begin; t < t_end;) {
            bool pair = (t + 1 < t_end) && pl[t].ok && pl[t + 1].ok &&
                        H->tri_grp[t] >= 0 && H->tri_grp[t + 1] == H->tri_grp[t] &&
                        d->tri_obj[t + 1] == d->tri_obj[t];
            if (in_bvh(t)) {
                H->bunit.push_back(make_unit(t, pair, 0));
            } else {
                double dev = 0.0;
                const int rot = pair ? quad_rot(t, &dev) : -1;
                H->unit.push_back(make_unit(t, pair, 1, rot, dev));
                H->unit_eye.push_back(make_unit(t, pair, 0, rot, dev));
            }
            t += pair ? 2 : 1;
        }
        if (part == 0) H->k.n_obj_unit = (int32_t)H->unit.size();
    }
    H->k.n_unit = (int32_t)H->unit.size();
    // materials
    H->mat.assign(d->n_obj, Mat{});
    for (int o = 0; o < d->n_obj; ++o) {
        const double* m = d->mat + 8 * o;
        Mat& M = H->mat[o];
        M.rgb[0] = m[0]; M.rgb[1] = m[1]; M.rgb[2] = m[2];
        M.ka = m[3]; M.kd = m[4]; M.ks = m[5];
        M.kdks = m[4] + m[5];
        M.nexp = m[7];
        for (int c = 0; c < 3; ++c) {
            M.amb[c] = m[c] * m[3] * d->ambient;
            M.lrgb[c] = d->light_rgb[c] * m[c];
        }
        M.nint = (m[7] >= 0 && m[7] <= 16 && m[7] == floor(m[7])) ? (int32_t)m[7] : -1;
    }
    // light CDF: running sums from 0, utils.py:30-35
    H->light_tri.clear();
    H->light_cum.assign(1, 0.0);
    double acc = 0.0;
    for (int t = d->n_obj_tri; t < T; ++t) {
        H->light_tri.push_back(t);
        acc += d->tri_area[t];
        H->light_cum.push_back(acc);
    }
    SceneK& K = H->k;
    K.n_tri = T;
    K.n_obj_tri = d->n_obj_tri;
    K.n_obj = d->n_obj;
    K.n_light = (int32_t)H->light_tri.size();
    K.light_sum = acc;
    for (int i = 0; i < 3; ++i) {
        K.eye[i] = d->eye[i];
        K.light_rgb[i] = d->light_rgb[i];
        K.center[i] = C[i];
        K.center_s[i] = Cs[i];
    }
    for (int i = 0; i < 4; ++i) K.ortho[i] = d->ortho[i];
    K.ambient = d->ambient;
    H->kd.assign(kKdCount, 0.0);
    for (int i = 0; i < 3; ++i) {
        H->kd[kKdEye + i] = K.eye[i];
        H->kd[kKdCenterS + i] = K.center_s[i];
        H->kd[kKdCenter + i] = K.center[i];
        H->kd[kKdLightRgb + i] = K.light_rgb[i];
    }
    H->kd[kKdLightSum] = K.light_sum;
    // leaf codes (unit offset << 3 | count) travel in stack entries as
    // (~code << 3 | ray mask) in 32 bits
    if (H->bunit.size() >= (size_t(1) << 24)) return "mesh too large: at most 2^24 BVH units";
    build_bvh(H, X);   // needs K.center and K.n_tri
    build_unitc(H);
    return "";
}

// host pointers (for the host-side check build)
inline void bind_host(HostScene* H) {
    H->k.unit = H->unit.data();
    H->k.unit_eye = H->unit_eye.data();
    H->k.bnode = H->bnode.data();
    H->k.cnode = H->cnode.data();
    H->k.qnode = H->qnode.data();
    H->k.bunit = H->bunit.data();
    H->k.bunitc = H->bunitc.empty() ? nullptr : H->bunitc.data();
    H->k.tri_grp = H->tri_grp.data();
    H->k.trid = H->trid.data();
    H->k.tris = H->tris.data();
    H->k.tri_obj = H->tri_obj.data();
    H->k.mat = H->mat.data();
    H->k.light_tri = H->light_tri.data();
    H->k.light_cum = H->light_cum.data();
    H->k.kd = H->kd.data();
}

// first band row >= row_begin with iy % step == phase, and the band's row count
inline bool band_layout(const pt_render_params* p, int32_t* first, int32_t* rows) {
    if (p->row_step <= 0 || p->row_phase < 0 || p->row_phase >= p->row_step) return false;
    const int32_t b = std::max(0, p->row_begin), e = std::min(p->height, p->row_end);
    int32_t f = b + ((p->row_phase - b % p->row_step) + p->row_step) % p->row_step;
    *first = f;
    *rows = (f < e) ? (e - f + p->row_step - 1) / p->row_step : 0;
    return true;
}

}  // namespace pt
