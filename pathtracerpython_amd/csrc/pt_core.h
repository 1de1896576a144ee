// pt_core.h — numerics of the hot path, shared by the gfx950 kernels and the
// host-side self-test (compiled as __host__ __device__).
//
// Reference semantics reproduced here (thiagoald/pathtracerpython):
//   intersect(ray, triangle)        utils.py:98-147   -> eval64()
//   in_triangle(pt, triangle)       utils.py:72-91    -> eval64()
//   intersect_objects               main.py:83-122    -> closest_* (pt_hip.hip)
//   compute_shadow_rays             main.py:23-73     -> nee() (pt_hip.hip)
//   pick_random_triangle            utils.py:28-39    -> pick_light()
//   sample_random_pt / bary coords  utils.py:21-46    -> light_point()
//   rotate(axis=(0,1,0), ...)       main.py:148-162   -> TriS::R (host precompute)
//   uniform(a, b)                   main.py:16        -> keyed Philox (philox())
//
// Precision design: every test is first run in f32 through a
// *filter* that returns a decision only when it is certain under a rigorous
// per-triangle error bound; otherwise the test is re-evaluated in f64 with
// the reference's own formula.  All path state (origins, directions,
// throughput, colours) is f64.  Hence results track the f64 reference to
// ~1e-15 instead of inheriting f32 hit/miss flips.
#pragma once
#include <math.h>
#include <stdint.h>

#define PT_HD __host__ __device__ __forceinline__

#include "pt_math.h"

namespace pt {

constexpr double kZero = 1e-5;        // main.py:20, utils.py:18
constexpr double kTau = 6.28;         // main.py:19
constexpr int kLightSamples = 3;      // main.py:23
constexpr float kU = 5.9604645e-08f;  // 2^-24, f32 unit roundoff

// |t| thresholds equivalent to squared distance 1e-5, with slack
constexpr float kTzLo = 0.0031622745f;   // sqrt(1e-5) * (1 - 1e-6)
constexpr float kTzHi = 0.0031622809f;   // sqrt(1e-5) * (1 + 1e-6)

// ------------------------------------------------------------- records --
// f32 filter records.  Triangles are grouped into plane UNITS: 1 or 2
// consecutive triangles (scene order, same object) lying in one plane — the
// reference's quads are such pairs.  Per (ray, unit) the plane part of a test
// (q = n.d, 1/q, t, the error bound of t, the range checks) is computed once;
// per triangle only the barycentric part.  Coordinates are relative to
// SceneK::center.  Forms (x = origin, d = unit direction):
//   h(x) = n.x + cn      signed distance to the plane (n = reference v_plane
//                        of the unit's first triangle)
//   b(x) = gb.x + cb     barycentric weight of v2   (affine, plane-invariant)
//   c(x) = gc.x + cc     barycentric weight of v3
// Error constants (host prepare, pt_prepare.h):
//   eh, eq : abs error of h(o) and of q = n.d (eq also covers the rounding of
//            1/q and t, and the unit's plane mismatch between its triangles)
//   eo, ed : twice the abs error of b(o)/c(o) (+ 8u for the weights' own
//            rounding) and of b(d)/c(d) (max of the two forms); the factor 2
//            makes one bound cover alpha = 1 - b - c as well
//   g      : 2 max(|gb|_1, |gc|_1)
//   qhi    : |q| above qhi is certainly > 1e-5 (the reference's parallel test)
//   grp    : coplanar group (host-verified in f64).  A line whose origin lies
//            on a triangle of the same group meets this plane at |t| < 1e-4,
//            i.e. squared distance < 1e-5: certainly not a usable hit.
struct TriB {            // 8 words
    float gb[3], cb;
    float gc[3], cc;
};
struct alignas(16) UnitF {   // 128 B: two s_load_dwordx16
    float n[3], cn;
    float eh, eq, qhi;
    float eo, ed, g;         // the members' barycentric bound (max over members)
    int32_t grp, count;
    int32_t obj;             // the members' object (one per unit)
    int32_t t[2];            // member triangle indices in scene order
    int32_t quad;            // 1: a parallelogram pair (tri[0] labelled for quad_m,
                             // pt_path.h), 0: a single triangle, -1: another pair
    TriB tri[2];
};
static_assert(sizeof(UnitF) == 128, "UnitF is two scalar x16 loads");

// The BVH's single-triangle units in 64 B (two per cache line: the walks'
// leaf working set halves).  eo and eh are bfloat16 rounded up, the direction
// bounds (eq, qhi) the maxima over the BVH's units (SceneK::bvh_eq ...), ed is
// derived from g (ed <= g * kEdPerG, see pt_prepare.h), the object comes from
// tri_obj.  Wider bounds only widen the undecided band, which is decided in
// f64, so verdicts stay exact.
struct alignas(16) UnitC {
    float n[3], cn;
    TriB tri;
    int32_t t, grp;
    float g;
    uint32_t eoeh;   // bf16 of eo (low half) and of eh (high half), rounded up
};
PT_HD float bf16_lo(uint32_t w) { const uint32_t b = w << 16; float f; memcpy(&f, &b, 4); return f; }
PT_HD float bf16_hi(uint32_t w) { const uint32_t b = w & 0xffff0000u; float f; memcpy(&f, &b, 4); return f; }
// bf16 of a finite x >= 0, rounded up
inline uint32_t bf16_up(float x) {
    uint32_t b;
    __builtin_memcpy(&b, &x, 4);
    return (b >> 16) + ((b & 0xffffu) ? 1u : 0u);
}
static_assert(sizeof(UnitC) == 64, "UnitC is 64 B");
constexpr float kEdPerG = 1.25f * 0x1p-21f;   // s * 8u (pt_prepare.h: ed = 2 s 8u M, g >= 2 M (1 + 1e-3))

// f64 exact record: the reference's plane normal and edges (utils.py:109-111,
// :78-80).  cvp = dot(vp, v1).
struct alignas(16) TriD {
    double vp[3], cvp;
    double v1[3], v2[3], v3[3];
    double e12[3], e23[3], e31[3];   // v1-v2, v2-v3, v3-v1
    double pad;
};

// shading record: Obj.normals (scene_reader.py:5-8) and the rotate() matrix
// for angle arccos(n_y) about +y (main.py:248-249); other entries are +-0.
struct alignas(16) TriS {
    double n[3];
    double r00, r02, r11, r20, r22;
};

struct alignas(16) Mat {
    double rgb[3], ka;
    double kd, ks, kdks, nexp;   // kdks = kd + ks (main.py:240)
    int32_t nint;                // nexp as an integer when it is one, else -1
    int32_t pad[3];
    // the colour factors of shadow_color, products taken on the host in the
    // reference's order (bit-identical): the render loop then holds neither
    // Scene.ambient nor light_color in registers (K2 5.58 vs 5.62 ms)
    double amb[3];               // rgb * ka * ambient (compute_ambient_color, main.py:76-80)
    double lrgb[3];              // light_rgb * rgb (the leaked object's factor, main.py:65-73)
};

// BVH node over the plane units of large meshes (pt_prepare.h): boxes in
// centred f32 coordinates, inflated by a rigorous margin so that pruning with
// the f32 line never drops a test the reference's f64 line would pass.
// Depth-first layout with skip links (stackless traversal): an internal
// node's first child is the next node; `skip` is the node after its subtree
// (-1: done).  leaf >= 0: units [leaf >> 3, + (leaf & 7)) of SceneK::bunit.
struct alignas(16) BNode {
    float lo[3];
    int32_t skip;
    float hi[3];
    int32_t leaf;
};

// The same hierarchy for the ordered (nearest-first, per-lane stack)
// traversals: internal nodes only, each holding both children's boxes, so a
// step is one dependent 64-B load.  Child reference c >= 0: internal node
// cnode[c]; c <= -2: leaf, c = ~code with code as in BNode::leaf.
struct alignas(16) CNode {
    float lo0[3];
    int32_t c0;
    float hi0[3];
    int32_t c1;
    float lo1[3];
    int32_t pad0;
    float hi1[3];
    int32_t pad1;
};
constexpr int32_t kNoRef = -1;

// The wavefront walks' node form: 4 children per 64-B node, child boxes
// quantised to 8 bits on a per-node grid (after Ylitie, Karras & Laine 2017,
// "Efficient incoherent ray traversal on GPUs through compressed wide BVHs").
// Grid steps are powers of two and the host checks that every decoded bound
// org + q * step is an f32 value (pt_prepare.h build_qnodes), so the kernel's
// fmaf decode is exact and the decoded box contains the child's (already
// conservatively inflated) box: pruning stays conservative.
struct alignas(16) QNode {
    float org[3];
    uint32_t ex;               // byte a: biased f32 exponent of axis a's grid step
    uint32_t qlo[3], qhi[3];   // axis a, byte c: child c's bounds in grid steps (no child:
                               // lo 255, hi 0 — an empty box every line misses)
    int32_t ref[4];            // >= 0 QNode, <= -2 leaf (~code), kNoRef: no child
    int32_t pad[2];
};
static_assert(sizeof(QNode) == 64, "QNode is 64 B");

struct SceneK {
    const UnitF* unit;          // [n_unit] uniform plane units: object units (small objects, scene
                                // order), then the light's; large meshes go to the BVH
    const TriD* trid;
    const TriS* tris;
    const int32_t* tri_obj;
    const Mat* mat;
    const int32_t* light_tri;   // [n_light] global triangle index
    const double* light_cum;    // [n_light+1] running area sums (utils.py:31-35)
    const int32_t* tri_grp;     // [n_tri] coplanar group of each triangle
    int32_t n_tri, n_obj_tri, n_obj, n_light;
    int32_t n_unit, n_obj_unit, pad0, pad1;
    double light_sum;
    double eye[3];
    double ortho[4];
    double ambient;
    double light_rgb[3];
    double center[3];           // centre of the box of the triangles and the eye: the
                                // coordinates of unit_eye and of the BVH records
    double center_s[3];         // centre of the triangles' box: the coordinates of `unit`
                                // (origins on scene surfaces)
    const UnitF* unit_eye;      // [n_unit] the uniform units relative to `center`, with
                                // error bounds valid out to the eye (primary rays)
    const BNode* bnode;         // [n_bnode] BVH of the mesh objects' units (none: n_bnode = 0)
    const UnitF* bunit;         // [n_bunit] those units in leaf order
    int32_t n_bnode, n_bunit, bvh_min_tri, bvh_min_obj;   // lowest triangle / object in it
    int32_t bvh_depth;           // levels below the root (the ordered traversal's stack need)
    int32_t bvh_root;            // the root as a CNode reference (0, or ~code for a leaf root)
    int32_t pad3[2];
    const CNode* cnode;          // [n_bnode - leaves] the two-child form of bnode
    const QNode* qnode;          // [n_qnode] the 4-wide quantised form (wavefront walks)
    int32_t n_qnode, qroot;      // qroot: a QNode, or ~code for a leaf root
    int32_t qstack, pad4;        // stack entries a 4-wide walk can need
    const UnitC* bunitc;         // [n_bunit] bunit in 64-B form, or null (some unit is a
                                 // coplanar pair or degenerate: the walks read bunit)
    float bvh_eh, bvh_eq, bvh_qhi;   // maxima over bunit
    int32_t bvh_obj1;            // the BVH's one object, or -1 (several: from tri_obj)
    // The f64 constants the bounce loop reads (eye, the frame centres,
    // light_sum, light_rgb),
    // also in device memory, where the loop reads them: as kernel-argument
    // fields they sit next to `ortho` and came in one 16-dword scalar load
    // whose register tuple was spilled to VGPR lanes and restored whole at
    // each use (336 v_readlane in k_render; 99 -> 73 SGPR spills, 499 -> 109
    // readlanes with this table)
    const double* kd;            // [kKd*] below
};
enum : int { kKdEye = 0, kKdCenterS = 3, kKdLightSum = 6, kKdCenter = 7, kKdLightRgb = 10, kKdCount = 13 };

// ------------------------------------------------------------------ RNG --
// Philox4x32-10 (Salmon et al., SC'11), key = seed, counter =
// (pixel, sample, bounce, slot>>2); see tests/golden/philox_ref.py.
// The 4 blocks of one (pixel, sample, bounce) — slots 0..15 — in lockstep:
// four independent 10-round chains interleaved, instead of one chain at a time
PT_HD void rng_blocks4(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t bounce,
                       uint32_t w[16]) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        w[4 * b] = pixel; w[4 * b + 1] = sample; w[4 * b + 2] = bounce; w[4 * b + 3] = (uint32_t)b;
    }
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            uint32_t* c = w + 4 * b;
            const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
            const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
            const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
            const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
            c[1] = (uint32_t)p1;
            c[3] = (uint32_t)p0;
            c[0] = n0;
            c[2] = n2;
        }
    }
}

// One Philox4x32-10 block: slots 4 blk .. 4 blk + 3 of (pixel, sample, bounce)
#ifndef PT_RNG_KEY_OPQ
#define PT_RNG_KEY_OPQ 1
#endif
PT_HD void rng_block(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t bounce, uint32_t blk,
                     uint32_t c[4]) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#if PT_RNG_KEY_OPQ && defined(__HIP_DEVICE_COMPILE__)
    // The round keys from the seed at each call (two scalar adds per round)
    // instead of 20 keys the compiler precomputes and holds in SGPRs across
    // the bounce loop (K2: SGPR spills 65 -> 43, no scratch): an
    // empty pure asm with the loop-variant bounce index as an input cannot
    // be hoisted out of the loop.  (A volatile asm would count as a memory
    // side effect and turn the unit records' scalar loads into vector loads.)
    asm("" : "+s"(k0), "+s"(k1) : "v"(bounce));
#endif
    c[0] = pixel; c[1] = sample; c[2] = bounce; c[3] = blk;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[1] = (uint32_t)p1;
        c[3] = (uint32_t)p0;
        c[0] = n0;
        c[2] = n2;
    }
}

PT_HD double u_of(uint32_t w) { return (double)(w >> 8) * (1.0 / 16777216.0); }

// ------------------------------------------------------------- vectors --
struct D3 { double x, y, z; };
struct F3 { float x, y, z; };

PT_HD D3 d3(double x, double y, double z) { D3 r; r.x = x; r.y = y; r.z = z; return r; }
PT_HD D3 ld3(const double* p) { return d3(p[0], p[1], p[2]); }
PT_HD D3 operator+(D3 a, D3 b) { return d3(a.x + b.x, a.y + b.y, a.z + b.z); }
PT_HD D3 operator-(D3 a, D3 b) { return d3(a.x - b.x, a.y - b.y, a.z - b.z); }
PT_HD D3 operator*(D3 a, double s) { return d3(a.x * s, a.y * s, a.z * s); }
PT_HD double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PT_HD D3 cross(D3 a, D3 b) {   // np.cross component formulas
    return d3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// squared_dist(pt1, pt2), utils.py:48-49 (sum from 0, component order)
PT_HD double squared_dist(D3 a, D3 b) {
    const double dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
    return ((0.0 + dx * dx) + dy * dy) + dz * dz;
}
PT_HD D3 unit(D3 a) {   // v / np.linalg.norm(v), as v * rsqrt(v.v)
    return a * rsqrt_d(dot(a, a));
}
PT_HD F3 to_f3(D3 a) { F3 r; r.x = (float)a.x; r.y = (float)a.y; r.z = (float)a.z; return r; }

// -------------------------------------------------------- exact (f64) --
// intersect(ray, triangle) of utils.py:98-147 + squared_dist to the origin.
// dn: normalised direction (utils.py:110).  Returns hit, P, sqd = |P - o|^2.
// in_triangle's normalisations are skipped: only the signs of c1.c2 and
// c1.c3 matter, and a zero cross product gives 0 -> "outside", as the
// reference's NaN does.
// the intersection point P = o + dn t of utils.py:118-120 (no range test)
PT_HD D3 plane_point(const TriD& T, D3 o, D3 dn) {
    const D3 vp = ld3(T.vp);
    const double t = (T.cvp - dot(vp, o)) * rcp_d(dot(vp, dn));
    return o + dn * t;
}
PT_HD bool eval64(const TriD& T, D3 o, D3 dn, D3* P, double* sqd) {
    const D3 vp = ld3(T.vp);
    const double den = dot(dn, vp);
    if (!(fabs(den) > kZero)) return false;
    const D3 p = plane_point(T, o, dn);
    const D3 c1 = cross(ld3(T.e12), p - ld3(T.v2));
    const D3 c2 = cross(ld3(T.e23), p - ld3(T.v3));
    const D3 c3 = cross(ld3(T.e31), p - ld3(T.v1));
    *P = p;
    *sqd = squared_dist(p, o);
    return dot(c1, c2) > 0.0 && dot(c1, c3) > 0.0;
}

// --------------------------------------------------------- f32 filter --
PT_HD float aff3(const float g[3], float c, F3 x) {
    return fmaf(g[0], x.x, fmaf(g[1], x.y, fmaf(g[2], x.z, c)));
}
PT_HD float lin3(const float g[3], F3 x) {
    return fmaf(g[0], x.x, fmaf(g[1], x.y, g[2] * x.z));
}
PT_HD float min3f(float a, float b, float c) { return fminf(a, fminf(b, c)); }

PT_HD float rcpf(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);   // v_rcp_f32, 1 ulp; covered by eq/eh slack
#else
    return 1.0f / x;
#endif
}

// Filter verdicts
enum : int { kMiss = 0, kCand = 1, kAmb = 2 };

// Plane part of a test (per ray and unit).  Range semantics:
//   closest: valid iff sqd > 1e-5                 -> hi = inf
//   shadow : occluder iff 1e-5 <= sqd < |L - P|^2 -> hi_lo/hi_hi bracket tL
struct RayPlane {
    float q;       // n . d
    float t, at, dt;
    float del;     // barycentric bound, shared by the unit's triangles (see classify_tri)
    bool rmiss;    // |t| certainly out of range: the test is a certain miss
    bool rcand;    // |t| certainly in range and |q| certainly > 1e-5
};
// eh, eo: U.eh, U.eo (the render loop passes VGPR copies made once per unit:
// a VOP3 reads one SGPR, so two record constants in one fma cost a v_mov per
// ray otherwise, PT_VCONST)
PT_HD RayPlane ray_plane_e(const UnitF& U, float h, F3 d, float hi_lo, float hi_hi, float eh, float eo) {
    RayPlane p;
    const float q = lin3(U.n, d);
    p.q = q;
    const float r = rcpf(q);
    p.t = -h * r;
    p.at = fabsf(p.t);
    // |t_ref - t| <= (eh + |t| eq) / |q|  (eq absorbs the 3u|t| of 1/q and t)
    p.dt = fabsf(r) * fmaf(p.at, U.eq, eh);
    // the unit's bound coefficients are the max over its triangles, so one
    // del serves both
    p.del = fmaf(U.g, p.dt, fmaf(p.at, U.ed, eo));
    p.rmiss = (p.at + p.dt < kTzLo) | (p.at - p.dt >= hi_hi);
    p.rcand = (fabsf(q) > U.qhi) & (p.at - p.dt > kTzHi) & (p.at + p.dt < hi_lo);
    return p;
}
PT_HD RayPlane ray_plane(const UnitF& U, float h, F3 d, float hi_lo, float hi_hi) {
    return ray_plane_e(U, h, d, hi_lo, hi_hi, U.eh, U.eo);
}

// Barycentric part (per ray and triangle), branch-free.  With
// del = g dt + |t| ed + eo (unit-wide coefficients), the host constants already carry the factor 2:
// |beta_ref - beta|, |gamma_ref - gamma| <= del/2 and |alpha_ref - alpha|
// <= del (alpha = 1 - beta - gamma), so with m = min(beta, gamma, alpha):
//   m < -del  -> some true weight < 0: certainly outside
//   m >  del  -> every true weight > 0: certainly inside
struct Verdict {
    bool cand;   // the reference certainly reports a usable intersection
    bool amb;    // undecided: evaluate in f64
};
// the verdict of a test from its weight minimum m
PT_HD Verdict verdict_m(float m, const RayPlane& p) {
    const float del = p.del;
    Verdict v;
    v.cand = p.rcand & (m > del);
    v.amb = !(p.rmiss | (m < -del)) & !v.cand;
    return v;
}
PT_HD Verdict classify_tri(const TriB& B, const RayPlane& p, float bo, float co, F3 d) {
    const float beta = fmaf(p.t, lin3(B.gb, d), bo);
    const float gam = fmaf(p.t, lin3(B.gc, d), co);
    return verdict_m(min3f(beta, gam, (1.0f - beta) - gam), p);
}
PT_HD int verdict_code(Verdict v) { return v.cand ? kCand : (v.amb ? kAmb : kMiss); }

// ------------------------------------------------------ light sampling --
// pick_random_triangle, utils.py:28-39: first i with cum[i] <= n < cum[i+1]
PT_HD int pick_light(const SceneK& S, double u) {
    const double n = 0.0 + (S.kd[kKdLightSum] - 0.0) * u;
    for (int i = 0; i < S.n_light; ++i)
        if (S.light_cum[i] <= n && n < S.light_cum[i + 1]) return i;
    return 0;   // unreachable for u < 1 (the reference would fail here)
}

// sample_random_pt with sample_bary_coords, utils.py:21-25, :42-46
PT_HD D3 light_point(const TriD& T, double u1, double u2, double u3) {
    const double inv = rcp_d(((0.0 + u1) + u2) + u3);
    const double a = u1 * inv, b = u2 * inv, c = u3 * inv;
    return d3(a * T.v1[0] + b * T.v2[0] + c * T.v3[0],
              a * T.v1[1] + b * T.v2[1] + c * T.v3[1],
              a * T.v1[2] + b * T.v2[2] + c * T.v3[2]);
}

// ------------------------------------------------------------- bounce --
PT_HD D3 rotate_y(const TriS& R, D3 v) {   // np.dot(rotation_matrix, v)
    return d3(R.r00 * v.x + R.r02 * v.z, R.r11 * v.y, R.r20 * v.x + R.r22 * v.z);
}

// x ** n for a non-integer exponent: the general f64 pow, kept out of line —
// inlined it costs the kernel ~40 VGPRs for a path the Cornell materials
// (n = 5) never take.  `const`: no memory effects, so the call does not stop
// the compiler from using scalar loads for the uniform scene reads.
__host__ __device__ __attribute__((noinline, const)) inline double pow_general(double x, double n) {
    return pow(x, n);
}

PT_HD double pow_ref(double x, const Mat& m) {   // x ** n (numpy float power)
    if (m.nint >= 0) {
        double r = 1.0;
#pragma unroll 1
        for (int i = 0; i < m.nint; ++i) r *= x;
        return r;
    }
    return pow_general(x, m.nexp);
}
}  // namespace pt
