// Dev experiment (host only): wave-coherent ("packet") shadow walks over the
// sorted shadow query list, counted against the shipped one-ray walks
// (VERDICT r05 #2).  The K5 wavefront is run on the host with the GPU's slot
// layout (split slots per pixel), each step's shadow list is ordered by the
// origin's cell as the device counting sort orders it (stable by key), cut
// into waves of 64 consecutive entries, and every wave walks the 4-wide
// QNode tree as ONE traversal: a node is visited when some lane of the wave
// meets its box within its range, children in the order of the smallest lane
// distance, a leaf's units tested by the lanes that reached it.  Each lane's
// result must equal its one-ray walk's (checked).  Counts: node visits and
// leaf-unit tests per wave (packet) and per lane (one-ray walks).
//   driven by scripts/micro/packet_count.py
#include "../../tests/hostcheck/pt_hostcheck.cpp"

#include <vector>

namespace {
struct PCount {
    int64_t rays = 0, lane_visits = 0, lane_units = 0;         // one-ray walks
    int64_t waves = 0, wave_visits = 0, wave_units = 0;        // packet walks
    int64_t active_at_visit = 0, active_at_unit = 0;           // lanes in the mask at each
    int64_t mismatches = 0, max_stack = 0;
};
constexpr int kLRNG = PT_WF_LRNG != 0;

void packet_wave(const SceneK& S, std::vector<Shadow1>& r, const std::vector<F3>& o32,
                 const std::vector<int>& ogrp, const std::vector<Spill>& sp, int order, PCount* c) {
    const int n = (int)r.size();
    std::vector<F3> inv(n);
    uint64_t start = 0;
    const BNode R0 = S.bnode[0];
    for (int i = 0; i < n; ++i) {
        inv[i] = rcp_dir(r[i].d32);
        const F3 l = {R0.lo[0] - o32[i].x, R0.lo[1] - o32[i].y, R0.lo[2] - o32[i].z};
        const F3 h = {R0.hi[0] - o32[i].x, R0.hi[1] - o32[i].y, R0.hi[2] - o32[i].z};
        if (shadow1_open(S, r[i]) && box_hit(l, h, inv[i], r[i].hhi)) start |= 1ull << i;
    }
    ++c->waves;
    std::vector<std::pair<int, uint64_t>> st;
    if (start) st.push_back({S.qroot, start});
    while (!st.empty()) {
        auto [ref, m] = st.back();
        st.pop_back();
        uint64_t open = 0;
        for (int i = 0; i < n; ++i) if (shadow1_open(S, r[i])) open |= 1ull << i;
        m &= open;
        if (!m) continue;
        if (ref >= 0) {
            ++c->wave_visits;
            c->active_at_visit += __builtin_popcountll(m);
            const QNode& Q = S.qnode[ref];
            uint64_t cm[4] = {0, 0, 0, 0};
            float key[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
            for (int i = 0; i < n; ++i) {
                if (!((m >> i) & 1u)) continue;
                const QLine L = q_line_ex(Q, o32[i], inv[i]);
                const QSlabs SL = q_slabs(Q, L);
                for (int ch = 0; ch < 4; ++ch) {
                    const float d = q_child_dist_s(SL, ch, L, r[i].hhi);
                    if (d < INFINITY) {
                        cm[ch] |= 1ull << i;
                        const bool first = key[ch] == INFINITY;
                        if (order == 0) key[ch] = fminf(key[ch], d);          // nearest any lane
                        else if (first) key[ch] = d;                          // the first lane's
                    }
                }
            }
            int idx[4] = {0, 1, 2, 3};
            std::sort(idx, idx + 4, [&](int a, int b) { return key[a] < key[b]; });
            for (int j = 3; j >= 0; --j)
                if (cm[idx[j]]) st.push_back({Q.ref[idx[j]], cm[idx[j]]});
            c->max_stack = std::max<int64_t>(c->max_stack, (int64_t)st.size());
        } else {
            const int code = ~ref, u0 = code >> 3, nu = code & 7;
            for (int u = 0; u < nu; ++u) {
                uint64_t mm = 0;
                for (int i = 0; i < n; ++i) if (((m >> i) & 1u) && shadow1_open(S, r[i])) mm |= 1ull << i;
                if (!mm) break;
                ++c->wave_units;
                c->active_at_unit += __builtin_popcountll(mm);
                for (int i = 0; i < n; ++i) {
                    if (!((mm >> i) & 1u)) continue;
                    ShadowTrav1 T;
                    T.o32 = o32[i]; T.ogrp = ogrp[i];
                    if (S.bunitc) shadow1_unit<kLRNG>(S, bvh_unit<true>(S, u0 + u), o32[i], ogrp[i], &r[i], sp[i]);
                    else shadow1_unit<kLRNG>(S, bvh_unit<false>(S, u0 + u), o32[i], ogrp[i], &r[i], sp[i]);
                }
            }
        }
    }
}
}  // namespace

extern "C" {
// slots = pixels x split (the GPU's slot layout), steps: how many shade
// steps to walk; out[10] = PCount fields in order
int pk_count(const pt_scene_desc* d, int size, int spp, int split, int bounces, int max_steps, int order,
             int wave, int64_t* out) {
    HostScene H;
    if (!prepare_scene(d, &H).empty()) return -1;
    bind_host(&H);
    if (H.k.n_bnode == 0 || H.k.n_qnode == 0 || H.k.qstack > kBvhStack) return -3;
    const size_t npix = (size_t)size * size, n = npix * split;
    std::vector<WfPath> W(n);
    std::vector<WfShadowQ> SQ(n);
    std::vector<WfClosestQ> CQ(n);
    std::vector<LaneJob> J(n);
    std::vector<D3> D0(n);
    for (size_t i = 0; i < n; ++i) {
        const size_t px = i / split;
        const int ix = (int)(px % size), iy = (int)(px / size);
        const D3 eye = ld3(H.k.eye);
        const double x = linspace_at(H.k.ortho[0], H.k.ortho[2], size, ix);
        const double y = linspace_at(H.k.ortho[1], H.k.ortho[3], size, iy);
        D0[i] = d3(x - eye.x, y - eye.y, 0.0 - eye.z);
        J[i].seed = 9;
        J[i].pixel = (uint32_t)ix * (uint32_t)size + (uint32_t)iy;
        J[i].sample0 = (int32_t)(i % split);
        J[i].sample_stride = split;
        J[i].n_samples = spp / split;
        J[i].bounces = bounces;
        J[i].rr_depth = -1;
    }
    PCount c;
    std::vector<uint32_t> want(n);
    for (int step = 0; step < max_steps; ++step) {
        bool any = false;
        for (size_t i = 0; i < n; ++i) {
            want[i] = 0;
            if (step == 0) {
                W[i].put_rkey(J[i]);
                want[i] = wf_start(H.k, J[i], D0[i], &W[i], &CQ[i]);
            } else if (W[i].state() != kWfDone) {
                want[i] = wf_shade<true>(H.k, J[i], D0[i], &W[i], &SQ[i], &CQ[i], &CQ[i]);
                any = true;
            }
        }
        if (step > 0 && !any) break;
        // the shadow list: (slot, ray) in slot order, stable-sorted by the cell key
        struct E { uint32_t key; uint32_t slot; int k; };
        std::vector<E> list;
        for (size_t i = 0; i < n; ++i)
            for (int k = 0; k < kLightSamples; ++k)
                if ((want[i] >> k) & 1u) list.push_back(E{want[i] >> 16, (uint32_t)i, k});
        std::stable_sort(list.begin(), list.end(), [](const E& a, const E& b) { return a.key < b.key; });
        // one-ray walks (the shipped result) and their counts
        std::vector<Shadow1> res(list.size()), init(list.size());
        std::vector<F3> o(list.size());
        std::vector<int> g(list.size());
        for (size_t e = 0; e < list.size(); ++e) {
            const size_t i = list[e].slot;
            const Spill sp{W[i].sp, 1};
            Shadow1 r;
            wf_get_shadow1(SQ[i], list[e].k, &o[e], &g[e], &r);
            init[e] = r;
            ShadowTrav1 T;
            int buf[kBvhStackLocal];
            const ShadowStack K{buf, 1};
            s1_init(T, H.k, o[e], g[e], r, H.k.qroot);
            ++c.rays;
            while (T.ref != kNoRef) {
                while (T.ref >= 0) { s1_qnode(T, K, H.k, r); ++c.lane_visits; }
                if (T.ref != kNoRef) {
                    c.lane_units += (~T.ref) & 7;
                    if (H.k.bunitc) s1_units<true, kLRNG>(T, H.k, &r, sp, T.ref);
                    else s1_units<false, kLRNG>(T, H.k, &r, sp, T.ref);
                    T.ref = s1_pop(T, K, H.k, r);
                }
            }
            res[e] = r;
        }
        // packet walks over waves of `wave` consecutive entries
        for (size_t e0 = 0; e0 < list.size(); e0 += wave) {
            const size_t e1 = std::min(list.size(), e0 + wave);
            std::vector<Shadow1> r(init.begin() + e0, init.begin() + e1);
            std::vector<F3> oo(o.begin() + e0, o.begin() + e1);
            std::vector<int> gg(g.begin() + e0, g.begin() + e1);
            std::vector<Spill> sps;
            for (size_t e = e0; e < e1; ++e) sps.push_back(Spill{W[list[e].slot].sp, 1});
            packet_wave(H.k, r, oo, gg, sps, order, &c);
            for (size_t e = e0; e < e1; ++e) {
                const Shadow1& a = r[e - e0];
                const Shadow1& b = res[e];
                if (a.occ != b.occ || a.key2 != b.key2 || a.leak != b.leak) ++c.mismatches;
            }
        }
        for (size_t e = 0; e < list.size(); ++e) wf_put_shadow1(&SQ[list[e].slot], res[e]);
        // closest walks (exact, per lane) so the next shade step can run
        for (size_t i = 0; i < n; ++i) {
            if (!(want[i] & kWfWantClosest)) continue;
            const Spill sp{W[i].sp, 1};
            ClosestAcc ca = wf_get_acc(CQ[i]);
            ClosestTrav T;
            ClosestStackLocal L;
            const ClosestStack K = L.view();
            const WfClosestQ q = CQ[i];
            ctrav_init(T, H.k, F3{q.o[0], q.o[1], q.o[2]}, q.ogrp, F3{q.d[0], q.d[1], q.d[2]}, ca.b1, H.k.qroot);
            while (T.ref != kNoRef) {
                while (T.ref >= 0) ctrav_qnode(T, K, H.k, &ca);
                if (T.ref != kNoRef) {
                    if (H.k.bunitc) ctrav_leaf<false, true>(T, K, H.k, &ca, sp, nullptr);
                    else ctrav_leaf<false>(T, K, H.k, &ca, sp, nullptr);
                }
            }
            CQ[i].a1 = ca.a1; CQ[i].a2 = ca.a2; CQ[i].b1 = ca.b1; CQ[i].i1 = ca.i1;
        }
        fprintf(stderr, "step %d: %zu shadow rays, lane visits %lld, wave visits %lld\n", step, list.size(),
                (long long)c.lane_visits, (long long)c.wave_visits);
    }
    const int64_t v[10] = {c.rays, c.lane_visits, c.lane_units, c.waves, c.wave_visits, c.wave_units,
                           c.active_at_visit, c.active_at_unit, c.mismatches, c.max_stack};
    memcpy(out, v, sizeof v);
    return 0;
}
}
