// pt_shade.h — the wavefront path's list appends and its shade step
// (k_wf_shade), shared by pt_hip.hip and pt_shade.hip: k_wf_shade is compiled
// in a translation unit of its own (pt_shade.hip) so that it gets its own
// code-generation flags (build.py UNITS), as the K2 kernel does (pt_k2.hip).
#pragma once
#include "pt_render.h"
#include "pt_wavefront.h"

// PT_WF_BIN: the shadow walks' query list sorted by the origin's cell
// (wf_cell, 12 Morton bits; a counting sort on the device, k_bin_hist /
// k_bin_scatter) before each walk step (render_wavefront): lanes of a wave
// then walk from nearby origins toward the light, and the shadow walks run
// 10% faster.  The closest list stays unsorted
// (random directions: its walks did not gain).
#ifndef PT_WF_BIN
#define PT_WF_BIN 1
#endif
// PT_SHADE_OWN_TU: k_wf_shade is defined in pt_shade.hip (pt_hip.hip sees
// its declaration); 0: in pt_hip.hip
#ifndef PT_SHADE_OWN_TU
#define PT_SHADE_OWN_TU 1
#endif

// ------------------------------------------------- wavefront (BVH scenes) --
// pt_wavefront.h.  Queue counters: [0] shadow count, [1] shadow head,
// [2] closest count, [3] closest head; lists[0..3 slots) the shadow rays
// ((slot << 2) | ray), then [3 slots, 4 slots) closest.
// A walk kernel gets its list and its [count, head] pair.
__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {   // set bits of m below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// wave-aggregated append: one atomic per wave
__device__ __forceinline__ void wf_append(bool want, int32_t* counter, int32_t* list, int32_t v) {
    const uint64_t m = __ballot(want);
    if (m == 0) return;
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1u;
    int32_t base = 0;
    if (lane_id() == leader) base = atomicAdd(counter, (int32_t)__popcll(m));
    base = __shfl(base, (int)leader);
    if (want) list[base + (int32_t)lanes_below(m)] = v;
}
// the same for the shadow rays (bits 0..2 of want): one atomic per wave for
// all three (a single counter takes every wave's appends: three atomics made
// the shade step 6 -> 11.6 ms), entries (slot << 2) | ray, a slot's rays next
// to each other (they share the query record and the origin: 94.1 vs 96.5 ms
// ray-major on K5 512^2 x 64)
__device__ __forceinline__ void wf_append3(uint32_t want, int32_t* counter, int32_t* list, int32_t slot) {
    uint64_t m[kLightSamples];
    int32_t n = 0;
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) {
        m[k] = __ballot(((want >> k) & 1u) != 0);
        n += (int32_t)__popcll(m[k]);
    }
    if (n == 0) return;
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)__ballot(true)) - 1u;
    int32_t base = 0;
    if (lane_id() == leader) base = atomicAdd(counter, n);
    base = __shfl(base, (int)leader);
    int32_t pos = base;
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) pos += (int32_t)lanes_below(m[k]);
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k)
        if ((want >> k) & 1u) list[pos++] = wf_shadow_entry(slot, k);
}
// Both lists' appends of a 256-work-item block with one atomic per list and
// block: every block's appends land on the same two counters, whose atomics
// serialise (~10 ns each: three per wave on one counter made the shade step
// 6 -> 11.6 ms at 262k waves).  Entries as wf_append3 / wf_append, the
// block's waves in order.
#ifndef PT_WF_BLOCK_APPEND
#define PT_WF_BLOCK_APPEND 1
#endif
// work-items per shade block (one append atomic per list and block): 256 /
// 512 / 1024 -> K5 1248 / 1255 / 1284 ms (512: two waves/SIMD at 135 VGPRs;
// 1024: 127 VGPRs with a spill)
#ifndef PT_SHADE_BLOCK
#define PT_SHADE_BLOCK 256
#endif
constexpr int kShadeBlock = PT_SHADE_BLOCK;
// (>= 128: wf_append_block issues its two list atomics from waves 0 and 1)
static_assert(kShadeBlock % 64 == 0 && kShadeBlock >= 128 && kShadeBlock <= 1024, "whole waves, >= 2");
__device__ __forceinline__ void wf_append_block(uint32_t want, int32_t* counters, int32_t* shadow_list,
                                                int32_t* closest_list, int32_t slot,
                                                uint16_t* skeys = nullptr, uint32_t skey = 0) {
    constexpr int kWaves = kShadeBlock / 64;
    __shared__ int32_t cnt[2][kWaves], base[2];
    uint64_t m[kLightSamples];
    int32_t n = 0;
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) {
        m[k] = __ballot(((want >> k) & 1u) != 0);
        n += (int32_t)__popcll(m[k]);
    }
    const uint64_t mc = __ballot((want & kWfWantClosest) != 0);
    const int wv = (int)(threadIdx.x >> 6);
    if ((threadIdx.x & 63u) == 0) {
        cnt[0][wv] = n;
        cnt[1][wv] = (int32_t)__popcll(mc);
    }
    __syncthreads();
    if (threadIdx.x == 0 || threadIdx.x == 64) {   // the two atomics from two waves
        const int l = threadIdx.x == 0 ? 0 : 1;
        int32_t tot = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) tot += cnt[l][w];
        base[l] = tot ? atomicAdd(&counters[2 * l], tot) : 0;
    }
    __syncthreads();
    int32_t bs = base[0], bc = base[1];
    for (int w = 0; w < wv; ++w) {
        bs += cnt[0][w];
        bc += cnt[1][w];
    }
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k) bs += (int32_t)lanes_below(m[k]);
#pragma unroll
    for (int k = 0; k < kLightSamples; ++k)
        if ((want >> k) & 1u) {
            if (skeys) skeys[bs] = (uint16_t)skey;
            shadow_list[bs++] = wf_shadow_entry(slot, k);
        }
    if (want & kWfWantClosest) closest_list[bc + (int32_t)lanes_below(mc)] = slot;
}
#if defined(PT_SHADE_UNIT) ? PT_SHADE_OWN_TU : !PT_SHADE_OWN_TU
__global__ __launch_bounds__(kShadeBlock) void k_wf_shade(SceneK S, RenderK R, int32_t step,
                                                  WfPath* __restrict__ W, WfShadowQ* __restrict__ SQ,
                                                  WfClosestQ* __restrict__ CQ, const WfClosestQ* __restrict__ CQP,
                                                  int32_t* __restrict__ lists, int32_t* counters,
                                                  uint32_t slots, uint16_t* __restrict__ keys) {
    const uint32_t tid = blockIdx.x * (uint32_t)kShadeBlock + threadIdx.x;
    uint32_t want = 0;
#if PT_WF_BIN
    uint32_t skey = 0;
#endif
    if (tid >= slots) {   // (the last block of a kShadeBlock grid over 256-slot blocks)
    } else if (step == 0) {   // the primary queries are k_wf_primary's (one per pixel)
        const SlotJob j = slot_job(S, R, tid);
        W[tid].acc[0] = W[tid].acc[1] = W[tid].acc[2] = 0.0;
        W[tid].put_rkey(j.J);
        W[tid].set(j.valid && j.J.n_samples > 0 && j.J.bounces > 0 ? kWfPrimary : kWfDone, false, 0);
    } else if ((tid >> R.split_log2) < R.npix && W[tid].state() != kWfDone) {
        // (a finished slot costs one load: its job is only built when it runs)
        const SlotJob j = slot_job(S, R, tid);
#if PT_WF_BIN
        want = wf_shade<true>(S, j.J, j.d0, &W[tid], &SQ[tid], &CQ[tid], &CQP[tid >> R.split_log2]);
        skey = want >> 16;
        want &= 0xffffu;
#else
        want = wf_shade(S, j.J, j.d0, &W[tid], &SQ[tid], &CQ[tid], &CQP[tid >> R.split_log2]);
#endif
    }
#if PT_WF_BIN
    wf_append_block(want, counters, lists, lists + 3 * (size_t)slots, (int32_t)tid, keys, skey);
#elif PT_WF_BLOCK_APPEND
    wf_append_block(want, counters, lists, lists + 3 * (size_t)slots, (int32_t)tid);
#else
    wf_append3(want, &counters[0], lists, (int32_t)tid);   // one shadow walk per open ray
    wf_append((want & kWfWantClosest) != 0, &counters[2], lists + 3 * (size_t)slots, (int32_t)tid);
#endif
}
#elif !defined(PT_SHADE_UNIT)
__global__ __launch_bounds__(kShadeBlock) void k_wf_shade(SceneK S, RenderK R, int32_t step,
                                                  WfPath* __restrict__ W, WfShadowQ* __restrict__ SQ,
                                                  WfClosestQ* __restrict__ CQ, const WfClosestQ* __restrict__ CQP,
                                                  int32_t* __restrict__ lists, int32_t* counters,
                                                  uint32_t slots, uint16_t* __restrict__ keys);
#endif
