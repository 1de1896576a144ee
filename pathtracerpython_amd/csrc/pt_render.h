// pt_render.h — the single render kernel (k_render) and its launch records,
// shared by pt_hip.hip (the library, every other instantiation) and pt_k2.hip
// (k_render<false, false, false>, the K2 kernel, in a translation unit of its
// own so that it gets its own code-generation flags, build.py K2_FLAGS).
#pragma once
#include <hip/hip_runtime.h>

#include "pt_path.h"

using namespace pt;

// PT_K2_OWN_TU: k_render<false, false, false> is compiled in pt_k2.hip
// (pt_hip.hip declares the instantiation extern).  The phase-clock dev build
// keeps it in pt_hip.hip: its device-side counters live in that unit.
#ifndef PT_K2_OWN_TU
#if defined(PT_PHASE_CLOCKS)
#define PT_K2_OWN_TU 0
#else
#define PT_K2_OWN_TU 1
#endif
#endif

// ------------------------------------------------------------- kernels --
struct RenderK {
    int32_t W, H, spp, bounces;
    uint64_t seed;
    int32_t rr_depth;   // -1: off
    int32_t first_row, row_step, n_rows;
    int32_t sample_begin;
    uint32_t split, split_log2;
    uint32_t npix;
    int32_t out_f64;
    uint32_t out_stride;   // elements between output rows (pt_render_params.out_row_stride)
    // single kernel, launch drain: the pixels from tail_pix on (the image's
    // top rows, dispatched last) get 2^tail_log2 lanes each, from lane
    // tail_lane (a multiple of 64) on; tail_pix = npix: none
    uint32_t tail_pix, tail_lane, tail_log2;
};

struct StatsDev { unsigned long long v[8]; };

template <bool COUNT>
__device__ __forceinline__ void flush_counters(const Counters& c, StatsDev* st) {
    if (!COUNT) return;
    uint32_t v[8] = {c.closest_tests, c.shadow_tests, c.ray_bounces, c.shading_points,
                     c.light_hits, c.escapes, c.fallbacks, c.rescans};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t x = v[i];
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m);
        if ((threadIdx.x & 63) == 0 && x) atomicAdd(&st->v[i], (unsigned long long)x);
    }
}

// Work-item -> (pixel, sample slice) of a launch: `split` adjacent work-items
// share a pixel and stride its samples; the primary ray of main.py:191
// (make_screen_pts / make_rays, utils.py:55-69).
struct SlotJob {
    LaneJob J;
    D3 d0;
    int32_t row_local, ix;
    uint32_t c;
    bool valid;
};
__device__ __forceinline__ SlotJob slot_job(const SceneK& S, const RenderK& R, uint32_t tid) {
    SlotJob j;
    const uint32_t pl = tid >> R.split_log2;
    j.c = tid & (R.split - 1u);
    j.valid = pl < R.npix;
    j.row_local = 0;
    j.ix = 0;
    j.d0 = d3(0, 0, 0);
    j.J = LaneJob{};
    if (j.valid) {
        j.row_local = (int32_t)(pl / (uint32_t)R.W);
        j.ix = (int32_t)pl - j.row_local * R.W;
        const int32_t iy = R.first_row + j.row_local * R.row_step;
        const D3 eye = ld3(S.eye);
        const double x = linspace_at(S.ortho[0], S.ortho[2], R.W, j.ix);
        const double y = linspace_at(S.ortho[1], S.ortho[3], R.H, iy);
        j.d0 = d3(x - eye.x, y - eye.y, 0.0 - eye.z);
        const int32_t c = (int32_t)j.c, sp = (int32_t)R.split;
        j.J.seed = R.seed;
        j.J.pixel = (uint32_t)j.ix * (uint32_t)R.H + (uint32_t)iy;
        j.J.sample0 = R.sample_begin + c;
        j.J.sample_stride = sp;
        j.J.n_samples = (c < R.spp) ? (R.spp - c + sp - 1) / sp : 0;
        j.J.bounces = R.bounces;
        j.J.rr_depth = R.rr_depth;
    }
    return j;
}

// Sum of a pixel's sample colours over its `split` work-items (fixed xor
// order: deterministic), / spp (main.py:277), into the framebuffer.
__device__ __forceinline__ void store_pixel(const RenderK& R, const SlotJob& j, D3 acc, void* out,
                                            uint32_t split) {
    for (uint32_t m = 1; m < split; m <<= 1) {
        acc.x += __shfl_xor(acc.x, (int)m);
        acc.y += __shfl_xor(acc.y, (int)m);
        acc.z += __shfl_xor(acc.z, (int)m);
    }
    if (j.valid && j.c == 0) {   // pixel_color_list[i] / how_many_rays, main.py:277
        const double inv = (double)R.spp;
        const size_t e = (size_t)(R.n_rows - 1 - j.row_local) * (size_t)R.out_stride + (size_t)j.ix * 3;
        if (R.out_f64) {
            double* o = (double*)out + e;
            o[0] = acc.x / inv; o[1] = acc.y / inv; o[2] = acc.z / inv;
        } else {
            float* o = (float*)out + e;
            o[0] = (float)(acc.x / inv); o[1] = (float)(acc.y / inv); o[2] = (float)(acc.z / inv);
        }
    }
}

// The primary ray's closest hit (main.py:191, :197-205), shared by the
// `split` lanes of a pixel (scenes without a BVH): lane c tests the
// eye-frame units c, c + split, ... (a per-lane unit index: vector loads of
// the 128-B records), the group merges its candidate intervals with xor
// shuffles, and every lane finishes the query as closest() does.  The merge
// keeps closest_add's result except for the order among equal lower bounds,
// and those never decide: closest_finish sends them to its f64 rescan (its
// interval test b1 < a2 fails), so the hit is closest()'s bit for bit.  A
// lane traces 1/split of the primary ray instead of all of it (K2 frame:
// 32 lanes per pixel in one rank's band at N = 8, 64 in the tail rows).
__device__ __forceinline__ ClosestAcc closest_merge(const ClosestAcc& x, const ClosestAcc& y) {
    const bool yw = y.a1 < x.a1;   // (ties: x's, as closest_add keeps the first)
    ClosestAcc r;
    r.a1 = yw ? y.a1 : x.a1;
    r.b1 = yw ? y.b1 : x.b1;
    r.i1 = yw ? y.i1 : x.i1;
    r.a2 = fminf(fminf(x.a2, y.a2), yw ? x.a1 : y.a1);
    return r;
}
__device__ __forceinline__ int primary_shared(const SceneK& S, D3 eye, D3 d0, uint32_t c, uint32_t split,
                                              const Spill& sp, D3* P0) {
    const D3 dn = unit(d0);
    sp.put3(kSpP, eye);
    sp.put3(kSpNd, d0);
    const F3 o32 = to_f3(eye - ld3(S.center));
    const F3 d32 = to_f3(dn);
    ClosestAcc acc = closest_init();
    for (int u = (int)c; u < S.n_unit; u += (int)split) {
        const UnitF U = S.unit_eye[u];
        closest_unit<false>(S, U, origin_u(U, o32), d32, U.grp == -1, sp, kSpP, kSpNd, &acc, nullptr);
    }
    for (uint32_t m = 1; m < split; m <<= 1) {   // the pixel's lanes: one wave
        ClosestAcc y;
        y.a1 = __shfl_xor(acc.a1, (int)m);
        y.a2 = __shfl_xor(acc.a2, (int)m);
        y.b1 = __shfl_xor(acc.b1, (int)m);
        y.i1 = __shfl_xor(acc.i1, (int)m);
        acc = closest_merge(acc, y);
    }
    return closest_finish<false, false, false>(S, acc, eye, dn, P0, nullptr);
}
// from this many lanes per pixel on (wave-uniform): N = 8 band of the K2
// frame (32 lanes) 0.765 -> 0.750 ms; at 8 lanes (N = 1) the vector loads
// and the merge cost more than the 7/8 of the trace they save (+0.5%)
#ifndef PT_PRIMARY_SHARED
#define PT_PRIMARY_SHARED 16
#endif

// Work-items per k_render block: one wave.  Nothing in the kernel is shared
// beyond a wave (a pixel's lanes reduce with shuffles), and the spill home
// is LDS allocated per block: with 4-wave blocks a wave's slot stayed idle
// until the block's slowest wave ended (its 40 KB held), with 1-wave blocks
// it is refilled as soon as the wave ends.
#ifndef PT_RENDER_BLOCK
#define PT_RENDER_BLOCK 64
#endif
constexpr uint32_t kRenderBlock = PT_RENDER_BLOCK;
template <bool FORCE64, bool COUNT, bool BVH>
// 4 waves/SIMD (<= 128 VGPRs, a little scratch spill outside the triangle
// loops): 9.5 ms vs 10.8 ms at 3 waves and 15.3 ms at 2 on the 512^2 x 64spp
// bench (MI355X), see DESIGN.md §5.
#ifndef PT_RENDER_WAVES
#define PT_RENDER_WAVES 4
#endif
__global__ __launch_bounds__(kRenderBlock, PT_RENDER_WAVES) void k_render(SceneK S, RenderK R, void* __restrict__ out,
                                                         StatsDev* __restrict__ st) {
    __shared__ double spill[kSpillSlots][kRenderBlock];
    const Spill sp{&spill[0][threadIdx.x], (int)kRenderBlock};
    PT_STAMP(k0);
    // (slot_job's mapping written out: the register allocation of this kernel
    // is sensitive to what stays live across the render loop)
    const uint32_t tid = blockIdx.x * kRenderBlock + threadIdx.x;
    const bool tail = tid >= R.tail_lane;   // wave-uniform
    const uint32_t slog = tail ? R.tail_log2 : R.split_log2, split = 1u << slog;
    const uint32_t lt = tail ? tid - R.tail_lane : tid;
    const uint32_t pl = (tail ? R.tail_pix : 0u) + (lt >> slog);
    const uint32_t c = lt & (split - 1u);
    const bool valid = pl < (tail ? R.npix : R.tail_pix);
    Counters cnt = {};
    D3 acc = d3(0, 0, 0);
    int32_t row_local = 0, ix = 0;
    if (valid) {
        row_local = (int32_t)(pl / (uint32_t)R.W);
        ix = (int32_t)pl - row_local * R.W;
        const int32_t iy = R.first_row + row_local * R.row_step;
        const D3 eye = ld3(S.eye);
        const double x = linspace_at(S.ortho[0], S.ortho[2], R.W, ix);
        const double y = linspace_at(S.ortho[1], S.ortho[3], R.H, iy);
        const D3 d0 = d3(x - eye.x, y - eye.y, 0.0 - eye.z);
        const int32_t ns = ((int32_t)c < R.spp) ? (R.spp - (int32_t)c + (int32_t)split - 1) / (int32_t)split : 0;
        LaneJob J;
        J.seed = R.seed;
        J.pixel = (uint32_t)ix * (uint32_t)R.H + (uint32_t)iy;
        J.sample0 = R.sample_begin + (int32_t)c;
        J.sample_stride = (int32_t)split;
        J.n_samples = ns;
        J.bounces = R.bounces;
        J.rr_depth = R.rr_depth;
        D3 P0 = d3(0, 0, 0);
        int tri0 = -1;
        // (a pixel's lanes are all valid or all invalid, and split <= spp
        // gives every lane samples: the whole group takes this branch)
        if (PT_PRIMARY_SHARED && !FORCE64 && !COUNT && !BVH && split >= PT_PRIMARY_SHARED) {
            if (R.bounces > 0) tri0 = primary_shared(S, eye, d0, c, split, sp, &P0);
        } else if (ns > 0 && R.bounces > 0) {
            tri0 = closest<FORCE64, false, BVH>(S, eye, d0, -1, sp, &P0, &cnt, true);
        }
#if defined(PT_PHASE_CLOCKS)
        {
            PT_STAMP(k1);
            PT_PHASE_FLUSH_AT(5, k1 - k0);
        }
#endif
        acc = render_lane<FORCE64, COUNT, BVH>(S, J, d0, tri0, P0, sp, &cnt);
    }
#if defined(PT_PHASE_CLOCKS)
    {
        PT_STAMP(k2);
        PT_PHASE_FLUSH_AT(6, k2 - k0);
    }
#endif
    SlotJob j;
    j.valid = valid;
    j.c = c;
    j.row_local = row_local;
    j.ix = ix;
    store_pixel(R, j, acc, out, split);
    flush_counters<COUNT>(cnt, st);
}
