// pt_hip.hip — gfx950 kernels + C-ABI (include/pt_capi.h) of the MI355X path
// tracer.  Replaces the reference's spp x bounce loop (main.py:186-280) and its
// two Pool callables (intersect_objects main.py:83, compute_color main.py:142).
//
// Kernel geometry: one work-item per (pixel, sample-slice);
// `split` adjacent lanes share a pixel and stride its samples, so the whole
// pixel lives in one wave and is reduced with DPP/shuffles in a fixed order
// (deterministic).  Triangles are read with uniform indices -> scalar loads
// (s_load_dwordx16) from the 80-B f32 filter records; only rare ambiguous
// tests touch the f64 records.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <vector>

#include "pt_path.h"
#include "pt_wavefront.h"
#include "pt_prepare.h"
#include "pt_image.h"
#include "pt_ingest.h"

using namespace pt;

// ------------------------------------------------------------- errors --
static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
#define HIPCHK(expr)                                                              \
    do {                                                                          \
        hipError_t e_ = (expr);                                                   \
        if (e_ != hipSuccess)                                                     \
            return fail(PT_EHIP, std::string(#expr " failed: ") + hipGetErrorString(e_)); \
    } while (0)

// ------------------------------------------------------------- kernels --
// k_render and its launch records: pt_render.h
#include "pt_render.h"
#if PT_K2_OWN_TU
extern template __global__ void k_render<false, false, false>(SceneK, RenderK, void*, StatsDev*);
#endif

// ------------------------------------------------- wavefront (BVH scenes) --
// the list appends and the shade step (k_wf_shade): pt_shade.h
#include "pt_shade.h"

// PT_WF_BIN: the shadow list's counting sort on the 12-bit cell key without
// the host: the list's length n is read on the device.  nb = bin_cols(n)
// blocks (at most kBinBlocks, at least kBinMinChunk entries each, so a short
// list pays a small count matrix) each take a contiguous chunk of the list;
// k_bin_hist counts its keys per cell (LDS) into the cell-major count matrix
// (kBins x nb), k_bin_rows turns each cell's row into its exclusive prefix
// sums in place (one wave per row) and writes the row's total, k_bin_base
// scans the kBins totals (one block), and k_bin_scatter places the chunk's
// entries at base[cell] + row prefix (LDS cursors): every entry lands exactly
// once, in (cell, block, position-in-block) order.  Hand-written two-level
// scan, no decoupled lookback: a lookback scan's blocks can wait behind the
// persistent closest-walk blocks that share the GPU (DESIGN.md §11, 13.7 ms
// per call for hipCUB's).
constexpr int kBinBits = 12, kBins = 1 << kBinBits, kBinBlocks = 1024, kBinMinChunk = 2048;
static_assert(kBinBlocks <= 64 * 16, "k_bin_rows: a row is at most 16 entries per lane");
static_assert(kBins % 4 == 0 && kBins == 4 * 1024, "k_bin_rows: 4 rows per block; k_bin_base: 4 per thread");
__device__ __forceinline__ int32_t bin_cols(int32_t n) {
    const int32_t c = (n + kBinMinChunk - 1) / kBinMinChunk;
    return c < 1 ? 1 : (c > kBinBlocks ? kBinBlocks : c);
}
__device__ __forceinline__ void bin_chunk(int32_t n, int32_t nb, int32_t* b0, int32_t* b1) {
    const int32_t chunk = (n + nb - 1) / nb;
    *b0 = min(n, (int32_t)blockIdx.x * chunk);
    *b1 = min(n, *b0 + chunk);
}
// inclusive prefix sum over the 64 lanes of a wave
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const int lane = (int)(threadIdx.x & 63u);
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}
__global__ __launch_bounds__(256) void k_bin_hist(const uint16_t* __restrict__ keys, const int32_t* count,
                                                  uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[kBins];
    const int32_t n = *count, nb = bin_cols(n);
    if ((int32_t)blockIdx.x >= nb) return;   // (block-uniform, before any barrier)
    for (int i = threadIdx.x; i < kBins; i += 256) h[i] = 0u;
    __syncthreads();
    int32_t b0, b1;
    bin_chunk(n, nb, &b0, &b1);
    for (int32_t i = b0 + (int32_t)threadIdx.x; i < b1; i += 256) atomicAdd(&h[keys[i] & (kBins - 1)], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < kBins; i += 256) hist[(size_t)i * nb + blockIdx.x] = h[i];
}
// kBins / 4 blocks: one row of the count matrix per wave, lane l holding the
// row's entries [l per, (l + 1) per); the row becomes its exclusive prefix
// sums, its total goes to rowsum
__global__ __launch_bounds__(256) void k_bin_rows(uint32_t* __restrict__ hist, const int32_t* count,
                                                  uint32_t* __restrict__ rowsum) {
    const int32_t nb = bin_cols(*count);
    const int row = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63u);
    uint32_t* r = hist + (size_t)row * nb;
    const int per = (nb + 63) >> 6;
    uint32_t v[16], s = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int i = lane * per + j;
        v[j] = (j < per && i < nb) ? r[i] : 0u;
        s += v[j];
    }
    const uint32_t incl = wave_incl_scan(s);
    uint32_t x = incl - s;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int i = lane * per + j;
        if (j < per && i < nb) r[i] = x;
        x += v[j];
    }
    if (lane == 63) rowsum[row] = incl;
}
// one block of 1024: the exclusive prefix sums of the kBins row totals
__global__ __launch_bounds__(1024) void k_bin_base(const uint32_t* __restrict__ rowsum,
                                                   uint32_t* __restrict__ base) {
    __shared__ uint32_t wsum[16];
    const int t = (int)threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t v[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = rowsum[4 * t + j]; s += v[j]; }
    const uint32_t incl = wave_incl_scan(s);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t x = incl - s;
    for (int i = 0; i < w; ++i) x += wsum[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) { base[4 * t + j] = x; x += v[j]; }
}
__global__ __launch_bounds__(256) void k_bin_scatter(const uint16_t* __restrict__ keys,
                                                     const int32_t* __restrict__ vals, const int32_t* count,
                                                     const uint32_t* __restrict__ off,
                                                     const uint32_t* __restrict__ base,
                                                     int32_t* __restrict__ out) {
    __shared__ uint32_t cur[kBins];
    const int32_t n = *count, nb = bin_cols(n);
    if ((int32_t)blockIdx.x >= nb) return;   // (block-uniform, before any barrier)
    for (int i = threadIdx.x; i < kBins; i += 256) cur[i] = base[i] + off[(size_t)i * nb + blockIdx.x];
    __syncthreads();
    int32_t b0, b1;
    bin_chunk(n, nb, &b0, &b1);
    for (int32_t i = b0 + (int32_t)threadIdx.x; i < b1; i += 256)
        out[atomicAdd(&cur[keys[i] & (kBins - 1)], 1u)] = vals[i];
}

// Next list positions for the lanes that need one.  A wave claims a chunk of
// kWfChunk consecutive positions with one atomic on the list head and hands
// them out to its lanes as they need work; it claims the next chunk only when
// this one runs out (one global atomic per ~kWfChunk queries instead of one
// per refill turn).  [cb, ce): the wave's unclaimed rest (wave-uniform).
#ifndef PT_WF_CHUNK
#define PT_WF_CHUNK 64
#endif
constexpr int32_t kWfChunk = PT_WF_CHUNK;
static_assert(kWfChunk >= 64, "a refill turn can need a position for every lane of a wave");
__device__ __forceinline__ int32_t wf_fetch(bool need, int32_t* head, int32_t& cb, int32_t& ce) {
    const uint64_t m = __ballot(need);
    const int32_t n = (int32_t)__popcll(m);
    const int32_t idx = (int32_t)lanes_below(m);   // rank among the needing lanes
    const int32_t avail = ce - cb;
    int32_t pos = cb + idx;
    if (n > avail) {   // wave-uniform: claim the next chunk
        const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1u;
        int32_t base = 0;
        if (lane_id() == leader) base = atomicAdd(head, kWfChunk);
        base = __shfl(base, (int)leader);
        if (idx >= avail) pos = base + (idx - avail);
        cb = base + (n - avail);
        ce = base + kWfChunk;
    } else {
        cb += n;
    }
    return pos;
}

// The primary rays: one work-item per pixel (a pixel's `split` slots share
// it, main.py:191): the uniform part of the eye ray into CQP[pixel], whose
// BVH part is a closest query (list entry = pixel; spill home = the pixel's
// first slot).  Every slot of the pixel finishes it in its first shade step.
__global__ __launch_bounds__(256) void k_wf_primary(SceneK S, RenderK R, WfPath* __restrict__ W,
                                                    WfClosestQ* __restrict__ CQP,
                                                    int32_t* __restrict__ list, int32_t* counters) {
    const uint32_t pix = blockIdx.x * 256u + threadIdx.x;
    uint32_t want = 0;
    if (pix < R.npix) {
        const uint32_t slot = pix << R.split_log2;
        const SlotJob j = slot_job(S, R, slot);
        if (j.valid) want = wf_start(S, j.J, j.d0, &W[slot], &CQP[pix]);
    }
    wf_append((want & kWfWantClosest) != 0, counters, list, (int32_t)pix);
}
// Persistent walk kernels over the 4-wide quantised BVH (QNode): a
// work-item holds one query at a time and takes the next one from the list
// as soon as its walk ends.  A loop turn is one
// "while-while" round, except that the node phase ends for the whole wave
// once at most `thr` of its lanes are still descending and some lane has a
// leaf to test (the others carry on in the next turn): the wave does not wait
// for its longest node run, and lanes whose walk ended are refilled every
// turn.  Every turn makes progress (a node step, a leaf or a fetch), and a
// lane whose list is exhausted stays idle, so the loop drains.
// Walk stacks: kWalkStack entries per work-item, the first kWalkStackLds in
// shared memory (the top of a stack, where nearly all pushes and pops land),
// the rest in global memory.  Smaller shared-memory stacks let more
// work-groups share a CU (the walks wait on dependent node loads: occupancy
// is their latency hiding).
#ifndef PT_SHADOW_WAVES   // one-ray shadow walk: 5 waves/SIMD (90 VGPRs, no spills; 6: spills)
#define PT_SHADOW_WAVES 5
#endif
#ifndef PT_CLOSEST_WAVES
#define PT_CLOSEST_WAVES 5
#endif
#ifndef PT_WALK_STACK_LDS
#define PT_WALK_STACK_LDS 16
#endif
constexpr int kWalkStack = 48;                   // entries of a walk kernel's stack (= kBvhStack)
constexpr int kWalkStackLds = PT_WALK_STACK_LDS;  // of them in shared memory
constexpr int kWalkStackGlobal = kWalkStack - kWalkStackLds;
// COUNT (PT_FLAG_WALK_COUNT launches only): per-query work of the walk —
// queries, 4-wide node visits, leaf-unit tests — summed into wc[0..2]
// (the walks' algorithmic bytes).
template <bool COUNT>
__device__ __forceinline__ void flush_walk_counts(uint32_t q, uint32_t nodes, uint32_t units,
                                                  unsigned long long* wc) {
    if (!COUNT) return;
    uint32_t v[3] = {q, nodes, units};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        uint32_t x = v[i];
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m);
        if ((threadIdx.x & 63) == 0 && x) atomicAdd(&wc[i], (unsigned long long)x);
    }
}
__device__ __forceinline__ uint32_t leaf_units(int ref) { return (uint32_t)(~ref) & 7u; }

// The shadow walks: one work-item per open shadow ray (list entries
// (slot << 2) | ray, pt_path.h "one-ray shadow walks").
template <bool UC, bool COUNT>
__global__ __launch_bounds__(256, PT_SHADOW_WAVES) void k_wf_shadow(SceneK S, WfPath* __restrict__ W,
                                                   WfShadowQ* __restrict__ SQ,
                                                   const int32_t* __restrict__ list, int32_t* counters,
                                                   int32_t thr, unsigned long long* wc,
                                                   int* __restrict__ ovf) {
    uint32_t c_q = 0, c_nodes = 0, c_units = 0;
    const int32_t count = counters[0];
    int32_t cb = 0, ce = 0;   // this wave's claimed list positions (wf_fetch)
    int32_t slot = -1;
    bool exhausted = false;
    // the walk stack: its top kWalkStackLds entries in shared memory
    // (4 B each per lane), the rest in global memory
    __shared__ int stack[kWalkStackLds][256];
    const int lanes = (int)gridDim.x * 256, gl = (int)(blockIdx.x * 256u + threadIdx.x);
    const ShadowStackLds K{(PT_LDS int*)&stack[0][threadIdx.x], 256, ovf + gl, lanes, kWalkStackLds};
    Shadow1 r;
    ShadowTrav1 T;
    T.ref = kNoRef;
    int pl = kNoRef, pl2 = kNoRef;   // postponed leaves
    while (true) {
        const bool need = slot < 0 && !exhausted;
        if (__any(need)) {
            const int32_t i = wf_fetch(need, &counters[1], cb, ce);
            if (need) {
                if (i < count) {
                    const int32_t e = list[i];
                    slot = e >> 2;
                    if (COUNT) ++c_q;
                    F3 o32;
                    int ogrp;
                    wf_get_shadow1(SQ[slot], e & 3, &o32, &ogrp, &r);
                    s1_init(T, S, o32, ogrp, r, S.qroot);
                } else {
                    exhausted = true;
                }
            }
        }
        if (__all(slot < 0)) break;
        // node phase (wave-uniform loop).  Speculative: a lane that reaches a
        // leaf postpones it (pl) and keeps walking, so a turn can test two
        // leaves per lane and fewer lanes idle in this loop.
        while (true) {
            if (slot >= 0 && T.ref <= -2 && pl2 == kNoRef) {
                if (pl == kNoRef) pl = T.ref;
                else pl2 = T.ref;
                T.ref = s1_pop(T, K, S, r);
            }
            const bool desc = slot >= 0 && T.ref >= 0;
            const int32_t nd = (int32_t)__popcll(__ballot(desc));
            // end it early only when some lane has a leaf to test (progress)
            if (nd == 0 || (nd <= thr && __any(slot >= 0 && (pl != kNoRef || T.ref <= -2)))) break;
            if (desc) {
                if (COUNT) ++c_nodes;
                s1_qnode(T, K, S, r);
            }
        }
        if (slot >= 0) {
            const Spill sp{W[slot].sp, 1};
            if (COUNT)
                c_units += (pl != kNoRef ? leaf_units(pl) : 0u) + (pl2 != kNoRef ? leaf_units(pl2) : 0u) +
                           (T.ref <= -2 ? leaf_units(T.ref) : 0u);
            if (pl != kNoRef) s1_units<UC, PT_WF_LRNG != 0>(T, S, &r, sp, pl);
            if (pl2 != kNoRef) s1_units<UC, PT_WF_LRNG != 0>(T, S, &r, sp, pl2);
            pl = pl2 = kNoRef;
            if (T.ref <= -2) {
                s1_units<UC, PT_WF_LRNG != 0>(T, S, &r, sp, T.ref);
                T.ref = s1_pop(T, K, S, r);
            }
            // a ray closed meanwhile drops what is left (entries, a node)
            if (!shadow1_open(S, r)) T.ref = kNoRef;
        }
        if (slot >= 0 && T.ref == kNoRef) {
            wf_put_shadow1(&SQ[slot], r);
            slot = -1;
        }
    }
    flush_walk_counts<COUNT>(c_q, c_nodes, c_units, wc);
}

template <bool UC, bool COUNT>
__global__ __launch_bounds__(256, PT_CLOSEST_WAVES) void k_wf_closest(SceneK S, WfPath* __restrict__ W,
                                                    WfClosestQ* __restrict__ CQ,
                                                    const int32_t* __restrict__ list, int32_t* counters,
                                                    int32_t thr, unsigned long long* wc,
                                                    int* __restrict__ ovf_ref,
                                                    uint16_t* __restrict__ ovf_dist,
                                                    uint32_t wshift) {
    // wshift: list entries index CQ; the spill home of entry e is
    // W[e << wshift] (the primary queries: one per pixel, its first slot's home)
    uint32_t c_q = 0, c_nodes = 0, c_units = 0;
    const int32_t count = counters[0];   // [count, head]
    int32_t cb = 0, ce = 0;   // this wave's claimed list positions (wf_fetch)
    int32_t slot = -1;
    bool exhausted = false;
    ClosestAcc ca = closest_init();
    ClosestTrav T;
    // the walk stack: its top kWalkStackLds entries in shared memory (6 B
    // each per lane), the rest in global memory
    __shared__ int sref[kWalkStackLds][256];
    __shared__ uint16_t sdist[kWalkStackLds][256];
    const int lanes = (int)gridDim.x * 256, gl = (int)(blockIdx.x * 256u + threadIdx.x);
    const ClosestStackLds K{(PT_LDS int*)&sref[0][threadIdx.x], (PT_LDS uint16_t*)&sdist[0][threadIdx.x], 256,
                            ovf_ref + gl,
                         ovf_dist + gl, lanes, kWalkStackLds};
    T.ref = kNoRef;
    int pl = kNoRef, pl2 = kNoRef;   // postponed leaves
    while (true) {
        const bool need = slot < 0 && !exhausted;
        if (__any(need)) {
            const int32_t i = wf_fetch(need, &counters[1], cb, ce);
            if (need) {
                if (i < count) {
                    slot = list[i];
                    if (COUNT) ++c_q;
                    const WfClosestQ q = CQ[slot];
                    ca = wf_get_acc(q);
                    ctrav_init(T, S, F3{q.o[0], q.o[1], q.o[2]}, q.ogrp, F3{q.d[0], q.d[1], q.d[2]},
                               ca.b1, S.qroot);
                } else {
                    exhausted = true;
                }
            }
        }
        if (__all(slot < 0)) break;
        while (true) {   // node phase, speculative as in k_wf_shadow
            if (slot >= 0 && T.ref <= -2 && pl2 == kNoRef) {
                if (pl == kNoRef) pl = T.ref;
                else pl2 = T.ref;
                T.ref = ctrav_pop(T, K, ca.b1);
            }
            const bool desc = slot >= 0 && T.ref >= 0;
            const int32_t nd = (int32_t)__popcll(__ballot(desc));
            if (nd == 0 || (nd <= thr && __any(slot >= 0 && (pl != kNoRef || T.ref <= -2)))) break;
            if (desc) {
                if (COUNT) ++c_nodes;
                ctrav_qnode(T, K, S, &ca);
            }
        }
        if (slot >= 0) {
            const Spill sp{W[(size_t)slot << wshift].sp, 1};
            if (COUNT)
                c_units += (pl != kNoRef ? leaf_units(pl) : 0u) + (pl2 != kNoRef ? leaf_units(pl2) : 0u) +
                           (T.ref <= -2 ? leaf_units(T.ref) : 0u);
            if (pl != kNoRef) ctrav_units<false, UC>(T, S, &ca, sp, nullptr, pl);
            if (pl2 != kNoRef) ctrav_units<false, UC>(T, S, &ca, sp, nullptr, pl2);
            pl = pl2 = kNoRef;
            if (T.ref <= -2) ctrav_leaf<false, UC>(T, K, S, &ca, sp, nullptr);
        }
        if (slot >= 0 && T.ref == kNoRef) {
            CQ[slot].a1 = ca.a1;
            CQ[slot].a2 = ca.a2;
            CQ[slot].b1 = ca.b1;
            CQ[slot].i1 = ca.i1;
            slot = -1;
        }
    }
    flush_walk_counts<COUNT>(c_q, c_nodes, c_units, wc);
}

__global__ __launch_bounds__(256) void k_wf_final(SceneK S, RenderK R, const WfPath* __restrict__ W,
                                                  void* __restrict__ out) {
    const uint32_t tid = blockIdx.x * 256u + threadIdx.x;
    const SlotJob j = slot_job(S, R, tid);
    const D3 acc = j.valid ? ld3(W[tid].acc) : d3(0, 0, 0);
    store_pixel(R, j, acc, out, R.split);
}

// the origins the filter's bounds cover: within the surface frame's box
// (xs), within the box with the eye (xa); outside both -> forced f64
__device__ __forceinline__ bool in_box(F3 o, float x) {
    return fabsf(o.x) <= x && fabsf(o.y) <= x && fabsf(o.z) <= x;
}

// pt_signal: one 64-bit flag store after the stream's earlier work, released
// at system scope (a vector store; the host or a peer polls the flag)
__global__ __launch_bounds__(64) void k_signal(uint64_t* flag, uint64_t v) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void k_intersect(SceneK S, const double* __restrict__ rays,
                                                   int64_t n, float xs, float xa,
                                                   int32_t* __restrict__ out_tri,
                                                   double* __restrict__ out_p) {
    __shared__ double spill[kSpillSlots][256];
    const Spill sp{&spill[0][threadIdx.x], 256};
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const D3 o = ld3(rays + 6 * i), d = ld3(rays + 6 * i + 3);
    const bool in_s = in_box(to_f3(o - ld3(S.center_s)), xs);
    const bool in_a = in_box(to_f3(o - ld3(S.center)), xa);
    D3 P = d3(0, 0, 0);
    Counters c;
    // the uniform units take either frame (eye = !in_s), but the BVH walk
    // always runs in the frame with the eye (its boxes' inflation assumes
    // |o - center| <= xa): scenes with a BVH need in_a for the filter
    const bool fast = S.n_bnode > 0 ? in_a : (in_s || in_a);
    const int t = fast ? closest<false, false>(S, o, d, -1, sp, &P, &c, !in_s)
                       : closest<true, false>(S, o, d, -1, sp, &P, &c, true);
    out_tri[i] = t;
    out_p[3 * i] = P.x; out_p[3 * i + 1] = P.y; out_p[3 * i + 2] = P.z;
}

__global__ __launch_bounds__(256) void k_color(SceneK S, const int32_t* __restrict__ obj,
                                               const double* __restrict__ point,
                                               const double* __restrict__ normal,
                                               const double* __restrict__ u, int64_t n, float xs,
                                               float xa, double* __restrict__ out) {
    __shared__ double spill[kSpillSlots][256];
    const Spill sp{&spill[0][threadIdx.x], 256};
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const D3 P = ld3(point + 3 * i);
    double uu[12];
    for (int j = 0; j < 12; ++j) uu[j] = u[12 * i + j];
    // nee() tests the uniform units in the surface frame and the BVH in the
    // frame with the eye: the filter needs the point inside both boxes
    const bool ok = in_box(to_f3(P - ld3(S.center_s)), xs) && in_box(to_f3(P - ld3(S.center)), xa);
    Counters c;
    const D3 col = ok ? nee<false, false>(S, P, ld3(normal + 3 * i), obj[i], -1, uu, sp, &c)
                          : nee<true, false>(S, P, ld3(normal + 3 * i), obj[i], -1, uu, sp, &c);
    out[3 * i] = col.x; out[3 * i + 1] = col.y; out[3 * i + 2] = col.z;
}

// ---------------------------------------------------------------- API --
struct pt_scene {
    int device = 0;
    uint64_t fingerprint = 0;   // of the scene descriptor (pt_render_multi: one scene on every handle)
    int n_cu = 256;   // compute units of the device (MI355X: 256 in 8 XCDs)
    HostScene host;
    SceneK dev{};
    float xb_surf = 0.f, xb_all = 0.f;   // origin boxes of the two filter frames
    void* blob = nullptr;          // all scene tables, one allocation
    StatsDev* stats = nullptr;
    void* out_dev = nullptr;       // pt_render's staging buffer
    size_t out_cap = 0;
    hipStream_t stream = nullptr;  // pt_render's own stream
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    // wavefront path (BVH scenes): path records, query records, query lists
    // and counters, one allocation grown on demand
    void* wf = nullptr;
    size_t wf_bytes = 0;
    hipStream_t wf_side = nullptr;             // the closest walks run beside the shadow walks
    hipEvent_t wf_ev_shade = nullptr, wf_ev_walk = nullptr;
    std::vector<hipEvent_t> prof_ev;           // PT_FLAG_KERNEL_TIMES
};

namespace {
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// Origins handed to the filter must lie in the box its bounds assume: the
// largest centred coordinate of the triangles (surface frame), or of the
// triangles and the eye (frame with the eye), as prepare_scene's X.
float box_bound(const HostScene& H, bool with_eye) {
    double X = 0.0;
    const SceneK& K = H.k;
    const double* c = with_eye ? K.center : K.center_s;
    for (const TriD& T : H.trid) {
        const double* vs[3] = {T.v1, T.v2, T.v3};
        for (int v = 0; v < 3; ++v)
            for (int i = 0; i < 3; ++i) X = std::max(X, fabs(vs[v][i] - c[i]));
    }
    if (with_eye)
        for (int i = 0; i < 3; ++i) X = std::max(X, fabs(K.eye[i] - c[i]));
    return (float)X;
}
}  // namespace

template <typename T>
static int dev_alloc_copy(T** d, const T* h, size_t n) {
    HIPCHK(hipMalloc((void**)d, n * sizeof(T) + 16));
    if (h) HIPCHK(hipMemcpy(*d, h, n * sizeof(T), hipMemcpyHostToDevice));
    return PT_OK;
}

#if defined(PT_PHASE_CLOCKS)
// dev builds only (scripts/phase_clocks.py): the phase clocks of pt_path.h
extern "C" int pt_debug_phase_clocks(unsigned long long* out, int reset) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(pt_phase_clk), 8 * sizeof(unsigned long long)));
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(pt_phase_clk), z, sizeof(z)));
    }
    return PT_OK;
}
#endif

extern "C" {

int pt_api_version(void) { return PT_API_VERSION; }

// The content hash of the sources this library was compiled from
// (pathtracerpython_amd/build.py passes it as PT_BUILD_ID; the marker lets the
// build read it back from the file without loading it).
#ifndef PT_BUILD_ID
#error "PT_BUILD_ID (the sources' content hash) must be defined: build with pathtracerpython_amd/build.py"
#endif
static const char pt_build_id_str[] = "PT_BUILD_ID=" PT_BUILD_ID;
const char* pt_build_id(void) { return pt_build_id_str + 12; }

// test hook (tests/test_gpu.py): pt_render_multi fails while dealing band i
static std::atomic<int32_t> g_fault_multi{-1};
int pt_test_fault_inject(int32_t multi_band) {
    g_fault_multi.store(multi_band);
    return PT_OK;
}

const char* pt_last_error(void) { return g_err.c_str(); }

int pt_device_count(int32_t* count) {
    if (!count) return fail(PT_EINVAL, "null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return PT_OK;
}

void pt_scene_destroy(pt_scene* s) {
    if (!s) return;
    {
        DeviceGuard g(s->device);
        if (s->blob) (void)hipFree(s->blob);
        if (s->stats) (void)hipFree(s->stats);
        if (s->out_dev) (void)hipFree(s->out_dev);
        if (s->wf) (void)hipFree(s->wf);
        if (s->wf_ev_shade) (void)hipEventDestroy(s->wf_ev_shade);
        if (s->wf_ev_walk) (void)hipEventDestroy(s->wf_ev_walk);
        if (s->wf_side) (void)hipStreamDestroy(s->wf_side);
        for (hipEvent_t e : s->prof_ev) (void)hipEventDestroy(e);
        if (s->ev0) (void)hipEventDestroy(s->ev0);
        if (s->ev1) (void)hipEventDestroy(s->ev1);
        if (s->stream) (void)hipStreamDestroy(s->stream);
    }
    delete s;
}

int pt_scene_create_on(const pt_scene_desc* desc, int32_t device, pt_scene** out) {
    if (!out) return fail(PT_EINVAL, "null output handle");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(PT_ENODEV, "no HIP device visible (the MI355X path needs a gfx950 GPU)");
    if (device < 0 || device >= ndev)
        return fail(PT_EINVAL, "device " + std::to_string(device) + " out of range (" +
                                   std::to_string(ndev) + " visible)");
    DeviceGuard g(device);
    return pt_scene_create(desc, out);
}

// FNV-1a over the descriptor's arrays and constants
static void fnv(uint64_t* h, const void* p, size_t n) {
    const unsigned char* b = (const unsigned char*)p;
    for (size_t i = 0; i < n; ++i) *h = (*h ^ b[i]) * 0x100000001b3ull;
}
static uint64_t scene_fingerprint(const pt_scene_desc* d) {
    uint64_t h = 0xcbf29ce484222325ull;
    const size_t T = (size_t)d->n_tri;
    fnv(&h, &d->n_tri, 3 * sizeof(int32_t));
    fnv(&h, d->tri_v, 9 * T * sizeof(double));
    fnv(&h, d->tri_n, 3 * T * sizeof(double));
    fnv(&h, d->tri_area, T * sizeof(double));
    fnv(&h, d->tri_obj, T * sizeof(int32_t));
    fnv(&h, d->mat, 8 * (size_t)d->n_obj * sizeof(double));
    fnv(&h, d->eye, sizeof(d->eye) + sizeof(d->ortho) + sizeof(d->ambient) + sizeof(d->light_rgb));
    return h;
}

int pt_scene_create(const pt_scene_desc* desc, pt_scene** out) {
    if (!out) return fail(PT_EINVAL, "null output handle");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(PT_ENODEV, "no HIP device visible (the MI355X path needs a gfx950 GPU)");
    pt_scene* s = new pt_scene();
    std::string err = prepare_scene(desc, &s->host);
    if (!err.empty()) { delete s; return fail(PT_EINVAL, err); }
    if (hipGetDevice(&s->device) != hipSuccess) { delete s; return fail(PT_EHIP, "hipGetDevice failed"); }
    s->fingerprint = scene_fingerprint(desc);   // (prepare_scene checked the arrays)
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, s->device) == hipSuccess) {
        if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos) {
            std::string arch = prop.gcnArchName;
            delete s;
            return fail(PT_ENODEV, "device is " + arch + ", this build targets gfx950 only");
        }
        if (prop.multiProcessorCount > 0) s->n_cu = prop.multiProcessorCount;
    }
    HostScene& H = s->host;
    constexpr int kArrays = 15;
    const size_t sz[kArrays] = {H.unit.size() * sizeof(UnitF), H.trid.size() * sizeof(TriD),
                                H.tris.size() * sizeof(TriS), H.tri_obj.size() * sizeof(int32_t),
                                H.mat.size() * sizeof(Mat), H.light_tri.size() * sizeof(int32_t),
                                H.light_cum.size() * sizeof(double),
                                H.tri_grp.size() * sizeof(int32_t),
                                H.bnode.size() * sizeof(BNode), H.bunit.size() * sizeof(UnitF),
                                H.cnode.size() * sizeof(CNode), H.qnode.size() * sizeof(QNode),
                                H.bunitc.size() * sizeof(UnitC), H.unit_eye.size() * sizeof(UnitF),
                                H.kd.size() * sizeof(double)};
    const void* src[kArrays] = {H.unit.data(), H.trid.data(), H.tris.data(), H.tri_obj.data(),
                                H.mat.data(), H.light_tri.data(), H.light_cum.data(),
                                H.tri_grp.data(), H.bnode.data(), H.bunit.data(), H.cnode.data(),
                                H.qnode.data(), H.bunitc.data(), H.unit_eye.data(), H.kd.data()};
    size_t off[kArrays], total = 0;
    for (int i = 0; i < kArrays; ++i) { off[i] = total; total += align_up(sz[i]); }
    int rc = PT_OK;
    auto cleanup = [&](int code, const std::string& m) { pt_scene_destroy(s); return fail(code, m); };
    if (hipMalloc(&s->blob, total) != hipSuccess) return cleanup(PT_ENOMEM, "hipMalloc scene tables");
    for (int i = 0; i < kArrays; ++i)
        if (sz[i] && hipMemcpy((char*)s->blob + off[i], src[i], sz[i], hipMemcpyHostToDevice) != hipSuccess)
            return cleanup(PT_EHIP, "hipMemcpy scene tables");
    if (hipMalloc((void**)&s->stats, sizeof(StatsDev)) != hipSuccess) return cleanup(PT_ENOMEM, "hipMalloc stats");
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&s->ev0) != hipSuccess || hipEventCreate(&s->ev1) != hipSuccess)
        return cleanup(PT_EHIP, "stream/event creation");
    s->dev = H.k;
    char* b = (char*)s->blob;
    s->dev.unit = (const UnitF*)(b + off[0]);
    s->dev.trid = (const TriD*)(b + off[1]);
    s->dev.tris = (const TriS*)(b + off[2]);
    s->dev.tri_obj = (const int32_t*)(b + off[3]);
    s->dev.mat = (const Mat*)(b + off[4]);
    s->dev.light_tri = (const int32_t*)(b + off[5]);
    s->dev.light_cum = (const double*)(b + off[6]);
    s->dev.tri_grp = (const int32_t*)(b + off[7]);
    s->dev.bnode = (const BNode*)(b + off[8]);
    s->dev.bunit = (const UnitF*)(b + off[9]);
    s->dev.cnode = (const CNode*)(b + off[10]);
    s->dev.qnode = (const QNode*)(b + off[11]);
    s->dev.bunitc = H.bunitc.empty() ? nullptr : (const UnitC*)(b + off[12]);
    s->dev.unit_eye = (const UnitF*)(b + off[13]);
    s->dev.kd = (const double*)(b + off[14]);
    s->xb_surf = box_bound(H, false);
    s->xb_all = box_bound(H, true);
    *out = s;
    return rc;
}

int pt_band_rows(const pt_render_params* p, int32_t* rows) {
    if (!p || !rows) return fail(PT_EINVAL, "null argument");
    int32_t first;
    if (!band_layout(p, &first, rows)) return fail(PT_EINVAL, "bad row_step/row_phase");
    return PT_OK;
}

constexpr uint32_t kKnownFlags = PT_FLAG_RR | PT_FLAG_FORCE_F64 | PT_FLAG_COUNT | PT_FLAG_OUT_F64 |
                                 PT_FLAG_MEGAKERNEL | PT_FLAG_WALK_COUNT | PT_FLAG_KERNEL_TIMES;
static int validate(const pt_render_params* p) {
    if (!p) return fail(PT_EINVAL, "null params");
    if (p->width <= 0 || p->height <= 0) return fail(PT_EINVAL, "width/height must be > 0");
    // pixel keys k = ix*H + iy and the launch's pixel counts are 32-bit
    if ((int64_t)p->width * p->height >= (int64_t)1 << 32) return fail(PT_EINVAL, "image too large for 32-bit pixel keys");
    if (p->spp <= 0) return fail(PT_EINVAL, "spp must be > 0");
    if (p->bounces < 0) return fail(PT_EINVAL, "bounces must be >= 0");
    if (p->sample_begin < 0) return fail(PT_EINVAL, "sample_begin must be >= 0");
    if (p->row_step <= 0 || p->row_phase < 0 || p->row_phase >= p->row_step)
        return fail(PT_EINVAL, "need row_step > 0 and 0 <= row_phase < row_step");
    if (p->flags & ~kKnownFlags)
        return fail(PT_EINVAL, "unknown flag bits (bit 7, v4's PT_FLAG_TREE_WALK, is retired)");
    if (p->out_row_stride != 0 && (int64_t)p->out_row_stride < (int64_t)p->width * 3)
        return fail(PT_EINVAL, "out_row_stride must be 0 or >= width*3");
    if (p->lanes_per_pixel != 0) {
        uint32_t cap = 64;
        while (cap > 1 && (int32_t)cap > p->spp) cap >>= 1;
        const int32_t l = p->lanes_per_pixel;
        if (l < 0 || (l & (l - 1)) != 0 || l > (int32_t)cap)
            return fail(PT_EINVAL, "lanes_per_pixel must be 0 or a power of two <= min(64, spp)");
    }
    return PT_OK;
}

// Lanes (wavefront: path slots) per pixel: a power of two <= min(64, spp).
//
// Single kernel (scenes without a BVH): >= 8 samples per lane where the
// launch is large (K2 512^2 x 64 spp: 8 lanes per pixel; K3 and K4: 64), at
// most 2^30 lanes over the full image — but at least `min_lanes` lanes in the
// launch, i.e. ~4 dispatch rounds of the device's resident waves (n_cu x 4
// SIMDs x 4 waves x 64 lanes x 4 rounds = 2^20 on MI355X).  A launch of one
// round is as long as its slowest wave (~0.7 ms at K2) however little work
// the band holds: one rank's band of an N-GPU strong-scaling split of the K2
// frame, per-band kernel ms at 8 / 16 / 32 / 64 lanes per
// pixel: N=4 1.592 / 1.450 / 1.480 / 1.566, N=8 0.882 / 0.816 / 0.767 / 0.809
// (N=1 5.584 / 5.674 / 5.792 / 6.136: each lane traces its pixel's primary
// ray once).  A pixel's samples are summed in an order that depends on its
// lane count, so bands of different sizes round differently in the last
// bits (all within 1e-12 of the oracle); bands of equal launch size agree bit
// for bit.
// Wavefront (BVH scenes): path slots hold ~420 B of state each, so at most
// 64M slots (28 GB) over the full image (K5 512^2 x 64 spp: 2M slots 161.6
// ms, 4M 147.1, 8M 140.5, 16M 139.3 (round 1); 1024^2 x 256 spp with the
// one-ray walks: 16M 1419 ms, 32M 1392, 64M 1378 — fewer shade / walk steps,
// each with its drain); an N-way band gets 1/N of them.  The single kernel
// uses the same split on BVH scenes (min_lanes does not apply), so its
// framebuffer stays bitwise equal to the wavefront one.
//
// PT_SPLIT_FIXED (compile-time, tuning builds only) pins the split.
// PT_MIN_SPL: samples per lane the whole-image split keeps at least (round 6:
// 4, i.e. 16 lanes per pixel at K2 — 4.669-4.693 vs 4.741-4.744 ms at 8 samples
// per lane; round 5's kernel was flat between 8 and 16 lanes)
#ifndef PT_MIN_SPL
#define PT_MIN_SPL 4
#endif
static uint32_t choose_split(uint64_t image_pixels, uint64_t launch_pixels, int32_t spp, bool bvh,
                             uint64_t min_lanes) {
    uint32_t cap = 64;
    while (cap > 1 && (int32_t)cap > spp) cap >>= 1;
#ifdef PT_SPLIT_FIXED
    uint32_t f = 1;
    while (f * 2 <= (uint32_t)PT_SPLIT_FIXED && f * 2 <= cap) f *= 2;
    (void)image_pixels; (void)launch_pixels; (void)bvh; (void)min_lanes;
    return f;
#else
    uint32_t s = 1;
    const uint64_t target = (uint64_t)1 << (bvh ? 26 : 30);
    while (s < cap && image_pixels * s * 2 <= target && (bvh || spp / (int32_t)(s * 2) >= PT_MIN_SPL)) s *= 2;
    if (!bvh)
        while (s < cap && launch_pixels * s < min_lanes) s *= 2;
    return s;
#endif
}
// lanes of a single-kernel launch below which it gets more lanes per pixel:
// PT_MIN_ROUNDS dispatch rounds of the device's resident waves (4 per SIMD,
// k_render's __launch_bounds__)
#ifndef PT_MIN_ROUNDS
#define PT_MIN_ROUNDS 4
#endif
static uint64_t min_lanes_of(int n_cu) {
    return (uint64_t)n_cu * 4u * (uint64_t)PT_RENDER_WAVES * 64u * (uint64_t)PT_MIN_ROUNDS;
}

// Walk kernels: node-phase exit threshold (lanes still descending) and
// persistent grid size.  At 16M slots (K5 512^2 x 64 spp) the threshold
// 4 / 8 / 12 / 16 / 20 / 24 / 32 / 48 -> 149 / 140 / 134 / 131 / 129 / 128 /
// 130 / 174 ms; grids of 1 / 2 / 3 / 4 / 16 blocks per CU -> 271 / 174 / 169
// / 178 / 188 ms.  Compile-time (-D) so tuning builds can sweep them; the
// shipped library has no run-time knobs.
// Round 2 re-sweep (512^2 x 64 spp render, both walks): 16 / 24 / 32 / 40 /
// 48 -> 114.3 / 110.5 / 108.0 / 107.8 / 109.5 ms; the one-ray shadow walk's
// threshold 16 / 24 / 32 / 40 / 48 -> 100.7 / 98.8 / 97.4 / 96.9 / 96.9 ms.
// At the K5 bench size with 64M slots (1024^2 x 256 spp, ms): shadow / closest
// 40/32 1372-1382, 32/32 1407, 48/32 1366, 40/40 1370, 48/40 1349, 48/48
// 1351, 56/48 1359, 64/56 1885 (64: the node phase never ends early).
#ifndef PT_WF_THR_SHADOW
#define PT_WF_THR_SHADOW 48
#endif
#ifndef PT_WF_THR_CLOSEST
#define PT_WF_THR_CLOSEST 40
#endif
#ifndef PT_WF_SHADOW_BLOCKS_PER_CU
#define PT_WF_SHADOW_BLOCKS_PER_CU 5
#endif
#ifndef PT_WF_CLOSEST_BLOCKS_PER_CU
#define PT_WF_CLOSEST_BLOCKS_PER_CU 5
#endif
#ifndef PT_WF_CONCURRENT   // the two walks of a step on two streams
#define PT_WF_CONCURRENT 1
#endif

// The wavefront render of a BVH scene (pt_wavefront.h): per step one shade
// launch over the path slots, then the two persistent walk launches over the
// queries it appended.  A slot runs at most n_samples x bounces bounces plus
// the primary ray, so that many steps (+1 to finish the last bounce) drain
// every slot; steps after that would find no work.
static int render_wavefront(pt_scene* s, const RenderK& R, dim3 grid, void* out_dev, hipStream_t st,
                            uint32_t flags, pt_stats* stats) {
    const size_t slots = (size_t)grid.x * 256;
    const size_t sz_w = slots * sizeof(WfPath), sz_s = slots * sizeof(WfShadowQ),
                 sz_c = slots * sizeof(WfClosestQ), sz_l = 4 * slots * sizeof(int32_t);
    const unsigned sh_blocks =
        std::max(1u, std::min<unsigned>(grid.x, (unsigned)PT_WF_SHADOW_BLOCKS_PER_CU * (unsigned)s->n_cu));
    const unsigned cl_blocks =
        std::max(1u, std::min<unsigned>(grid.x, (unsigned)PT_WF_CLOSEST_BLOCKS_PER_CU * (unsigned)s->n_cu));
    // walk-stack overflow (entries below the shared-memory part): 4 B per
    // entry and shadow lane, 4 + 2 B per entry and closest lane
    const size_t ovf_n = (size_t)kWalkStackGlobal;
    const size_t sz_os = ovf_n * sh_blocks * 256 * 4, sz_ocr = ovf_n * cl_blocks * 256 * 4,
                 sz_ocd = ovf_n * cl_blocks * 256 * 2;
    const size_t off_s = sz_w, off_c = off_s + sz_s, off_l = off_c + sz_c, off_n = off_l + sz_l;
    const size_t off_os = off_n + 256, off_ocr = off_os + sz_os, off_ocd = off_ocr + sz_ocr;
    const size_t sz_p = (size_t)R.npix * sizeof(WfClosestQ);   // the primary queries, per pixel
    const size_t off_p = (off_ocd + sz_ocd + 255) / 256 * 256;
    // PT_WF_BIN: the shadow list's keys (3 slots x u16), the sorted list
    // (3 slots x i32), the sort's count matrix, its scan and scan storage
    size_t sz_tmp = 0;
#if PT_WF_BIN
    // the count matrix (its rows' prefix sums in place), the row totals and their scan
    sz_tmp = ((size_t)kBins * kBinBlocks + 2 * (size_t)kBins) * sizeof(uint32_t);
#endif
    const size_t sz_k = PT_WF_BIN ? 3 * slots * sizeof(uint16_t) : 0,
                 sz_lo = PT_WF_BIN ? 3 * slots * sizeof(int32_t) : 0;
    const size_t off_k = (off_p + sz_p + 255) / 256 * 256, off_lo = (off_k + sz_k + 255) / 256 * 256,
                 off_t = (off_lo + sz_lo + 255) / 256 * 256;
    const size_t need = off_t + sz_tmp + 256;
    if (need > s->wf_bytes) {
        if (s->wf) (void)hipFree(s->wf);
        s->wf = nullptr;
        s->wf_bytes = 0;
        if (hipMalloc(&s->wf, need) != hipSuccess) return fail(PT_ENOMEM, "hipMalloc wavefront buffers");
        s->wf_bytes = need;
    }
    if (!s->wf_side) {
        HIPCHK(hipStreamCreateWithFlags(&s->wf_side, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&s->wf_ev_shade, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&s->wf_ev_walk, hipEventDisableTiming));
    }
    char* b = (char*)s->wf;
    WfPath* W = (WfPath*)b;
    WfShadowQ* SQ = (WfShadowQ*)(b + off_s);
    WfClosestQ* CQ = (WfClosestQ*)(b + off_c);
    int32_t* lists = (int32_t*)(b + off_l);
    int32_t* counters = (int32_t*)(b + off_n);
    int* ovf_s = (int*)(b + off_os);
    int* ovf_cr = (int*)(b + off_ocr);
    uint16_t* ovf_cd = (uint16_t*)(b + off_ocd);
    WfClosestQ* CQP = (WfClosestQ*)(b + off_p);
    uint16_t* keys = PT_WF_BIN ? (uint16_t*)(b + off_k) : nullptr;
    int32_t* lists_o = (int32_t*)(b + off_lo);
#if PT_WF_BIN
    uint32_t* bin_hist = (uint32_t*)(b + off_t);
    uint32_t* bin_rowsum = bin_hist + (size_t)kBins * kBinBlocks;
    uint32_t* bin_base = bin_rowsum + kBins;
#endif
    bool sorted = false;   // this step's lists are in lists_o
#if PT_WF_BIN
    auto bin_sort = [&]() -> hipError_t {   // (the device reads the list's length: no host wait)
        hipLaunchKernelGGL(k_bin_hist, dim3(kBinBlocks), dim3(256), 0, st, (const uint16_t*)keys,
                           (const int32_t*)counters, bin_hist);
        hipLaunchKernelGGL(k_bin_rows, dim3(kBins / 4), dim3(256), 0, st, bin_hist, (const int32_t*)counters,
                           bin_rowsum);
        hipLaunchKernelGGL(k_bin_base, dim3(1), dim3(1024), 0, st, (const uint32_t*)bin_rowsum, bin_base);
        hipLaunchKernelGGL(k_bin_scatter, dim3(kBinBlocks), dim3(256), 0, st, (const uint16_t*)keys,
                           (const int32_t*)lists, (const int32_t*)counters, (const uint32_t*)bin_hist,
                           (const uint32_t*)bin_base, lists_o);
        sorted = true;
        return hipGetLastError();
    };
#endif
    const int32_t per_slot = (R.spp + (int32_t)R.split - 1) / (int32_t)R.split;
    const int32_t steps = per_slot * R.bounces + 2;
    const bool wcount = (flags & PT_FLAG_WALK_COUNT) != 0 && stats;
    const bool times = (flags & PT_FLAG_KERNEL_TIMES) != 0 && stats;
    unsigned long long* wc = (unsigned long long*)s->stats;   // [0..2] shadow, [3..5] closest
    if (wcount) HIPCHK(hipMemsetAsync(s->stats, 0, sizeof(StatsDev), st));
    // per-kernel HIP events (PT_FLAG_KERNEL_TIMES): shade, shadow, closest, the
    // shadow list's sort x (start, end) per step
    constexpr int kEv = 8;
    if (times) {
        const size_t ne = (size_t)steps * kEv;
        while (s->prof_ev.size() < ne) {
            hipEvent_t e;
            HIPCHK(hipEventCreate(&e));
            s->prof_ev.push_back(e);
        }
    }
    auto mark = [&](int32_t step, int k, int end, hipStream_t on) -> hipError_t {
        return times ? hipEventRecord(s->prof_ev[(size_t)step * kEv + k * 2 + end], on) : hipSuccess;
    };
    // step 0 walks the primary queries (CQP, one per pixel), later steps the slots' (CQ)
    auto closest_walk = [&](hipStream_t on, int32_t step) {
        const int32_t* l = lists + 3 * slots;
        WfClosestQ* q = step == 0 ? CQP : CQ;
        const uint32_t ws = step == 0 ? R.split_log2 : 0u;
        if (s->dev.bunitc) {
            if (wcount) hipLaunchKernelGGL((k_wf_closest<true, true>), dim3(cl_blocks), dim3(256), 0, on, s->dev, W, q, l, counters + 2, PT_WF_THR_CLOSEST, wc + 3, ovf_cr, ovf_cd, ws);
            else hipLaunchKernelGGL((k_wf_closest<true, false>), dim3(cl_blocks), dim3(256), 0, on, s->dev, W, q, l, counters + 2, PT_WF_THR_CLOSEST, wc + 3, ovf_cr, ovf_cd, ws);
        } else {
            if (wcount) hipLaunchKernelGGL((k_wf_closest<false, true>), dim3(cl_blocks), dim3(256), 0, on, s->dev, W, q, l, counters + 2, PT_WF_THR_CLOSEST, wc + 3, ovf_cr, ovf_cd, ws);
            else hipLaunchKernelGGL((k_wf_closest<false, false>), dim3(cl_blocks), dim3(256), 0, on, s->dev, W, q, l, counters + 2, PT_WF_THR_CLOSEST, wc + 3, ovf_cr, ovf_cd, ws);
        }
    };
    auto shadow_walk = [&](hipStream_t on) {
        const int32_t* l = sorted ? lists_o : lists;
        if (s->dev.bunitc) {
            if (wcount) hipLaunchKernelGGL((k_wf_shadow<true, true>), dim3(sh_blocks), dim3(256), 0, on, s->dev, W, SQ, l, counters, PT_WF_THR_SHADOW, wc, ovf_s);
            else hipLaunchKernelGGL((k_wf_shadow<true, false>), dim3(sh_blocks), dim3(256), 0, on, s->dev, W, SQ, l, counters, PT_WF_THR_SHADOW, wc, ovf_s);
        } else {
            if (wcount) hipLaunchKernelGGL((k_wf_shadow<false, true>), dim3(sh_blocks), dim3(256), 0, on, s->dev, W, SQ, l, counters, PT_WF_THR_SHADOW, wc, ovf_s);
            else hipLaunchKernelGGL((k_wf_shadow<false, false>), dim3(sh_blocks), dim3(256), 0, on, s->dev, W, SQ, l, counters, PT_WF_THR_SHADOW, wc, ovf_s);
        }
    };
    HIPCHK(hipEventRecord(s->ev0, st));
    for (int32_t step = 0; step < steps; ++step) {
        HIPCHK(hipMemsetAsync(counters, 0, 4 * sizeof(int32_t), st));
        HIPCHK(mark(step, 0, 0, st));
        hipLaunchKernelGGL(k_wf_shade, dim3((unsigned)((slots + kShadeBlock - 1) / kShadeBlock)),
                           dim3(kShadeBlock), 0, st, s->dev, R, step, W, SQ, CQ,
                           (const WfClosestQ*)CQP, lists, counters, (uint32_t)slots, keys);
        if (step == 0)
            hipLaunchKernelGGL(k_wf_primary, dim3((R.npix + 255) / 256), dim3(256), 0, st, s->dev, R, W,
                               CQP, lists + 3 * slots, counters + 2);
        HIPCHK(mark(step, 0, 1, st));
        sorted = false;
        if (step + 1 < steps) {
            // the two walks only read the shade step's output and write
            // disjoint records: the closest walks run on a side stream
            // (PT_FLAG_KERNEL_TIMES launches run them one after the other on
            // one stream, so each walk's HIP-event time is its own time on
            // the whole chip, not the stretches it waits for the other's CUs)
            const bool side = PT_WF_CONCURRENT && !times;
            hipStream_t cs = side ? s->wf_side : st;
            if (side) {
                HIPCHK(hipEventRecord(s->wf_ev_shade, st));
                HIPCHK(hipStreamWaitEvent(s->wf_side, s->wf_ev_shade, 0));
            }
            HIPCHK(mark(step, 2, 0, cs));
            closest_walk(cs, step);
            HIPCHK(mark(step, 2, 1, cs));
            if (side) HIPCHK(hipEventRecord(s->wf_ev_walk, s->wf_side));
#if PT_WF_BIN
            // the shadow list sorted by the origin's cell (the device reads
            // its length) while the closest walks, unsorted, already run
            if (step > 0) {   // (step 0: the primary rays)
                HIPCHK(mark(step, 3, 0, st));
                HIPCHK(bin_sort());
                HIPCHK(mark(step, 3, 1, st));
            }
#endif
            HIPCHK(mark(step, 1, 0, st));
            shadow_walk(st);
            HIPCHK(mark(step, 1, 1, st));
            if (side) HIPCHK(hipStreamWaitEvent(st, s->wf_ev_walk, 0));
        }
    }
    hipLaunchKernelGGL(k_wf_final, grid, dim3(256), 0, st, s->dev, R, (const WfPath*)W, out_dev);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(s->ev1, st));
    s->timed = true;
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        if (wcount || times) HIPCHK(hipStreamSynchronize(st));
        if (wcount) {
            StatsDev h;
            HIPCHK(hipMemcpy(&h, s->stats, sizeof(h), hipMemcpyDeviceToHost));
            stats->shadow_queries = h.v[0];
            stats->shadow_node_visits = h.v[1];
            stats->shadow_leaf_units = h.v[2];
            stats->closest_queries = h.v[3];
            stats->closest_node_visits = h.v[4];
            stats->closest_leaf_units = h.v[5];
        }
        if (times) {
            double t[4] = {0, 0, 0, 0};
            uint64_t n[4] = {0, 0, 0, 0};
            for (int32_t step = 0; step < steps; ++step)
                for (int k = 0; k < 4; ++k) {
                    if (k > 0 && step + 1 >= steps) continue;
                    if (k == 3 && (!PT_WF_BIN || step == 0)) continue;
                    float ms = 0.f;
                    HIPCHK(hipEventElapsedTime(&ms, s->prof_ev[(size_t)step * kEv + k * 2],
                                               s->prof_ev[(size_t)step * kEv + k * 2 + 1]));
                    t[k] += ms;
                    ++n[k];
                }
            stats->shade_ms = t[0]; stats->shadow_ms = t[1]; stats->closest_ms = t[2];
            stats->shade_launches = n[0]; stats->shadow_launches = n[1]; stats->closest_launches = n[2];
            stats->sort_ms = t[3]; stats->sort_launches = n[3];
        }
    }
    return PT_OK;
}

int pt_render_device(pt_scene* s, const pt_render_params* p, void* out_dev, void* stream,
                     pt_stats* stats) {
    int rc = validate(p);
    if (rc) return rc;
    if (!s) return fail(PT_EINVAL, "null scene");
    int32_t first = 0, rows = 0;
    band_layout(p, &first, &rows);
    if (rows == 0) return PT_OK;
    if (!out_dev) return fail(PT_EINVAL, "null output");
    DeviceGuard g(s->device);
    hipStream_t st = (hipStream_t)stream;
    RenderK R;
    R.W = p->width; R.H = p->height; R.spp = p->spp; R.bounces = p->bounces;
    R.seed = p->seed;
    R.rr_depth = (p->flags & PT_FLAG_RR) ? std::max(0, p->rr_depth) : -1;
    R.first_row = first; R.row_step = p->row_step; R.n_rows = rows;
    R.sample_begin = p->sample_begin;
    R.out_f64 = (p->flags & PT_FLAG_OUT_F64) ? 1 : 0;
    R.npix = (uint32_t)rows * (uint32_t)p->width;
    R.out_stride = p->out_row_stride ? (uint32_t)p->out_row_stride : (uint32_t)p->width * 3u;
    R.split = p->lanes_per_pixel > 0
                  ? (uint32_t)p->lanes_per_pixel
                  : choose_split((uint64_t)p->width * (uint64_t)p->height, (uint64_t)R.npix, p->spp,
                                 s->dev.n_bnode > 0, min_lanes_of(s->n_cu));
    R.split_log2 = 0;
    while ((1u << R.split_log2) < R.split) ++R.split_log2;
    R.tail_pix = R.npix;
    R.tail_lane = R.npix * R.split;
    R.tail_log2 = R.split_log2;
    if (s->dev.n_bnode == 0) {
        // The launch drains for about one wave lifetime (~1 ms at K2: 7% of
        // its wave-slots idle).  The image's top sixteenth of
        // rows (iy >= H - ceil(H/16), dispatched last, also in every
        // interleaved band) gets 8x the lanes per pixel, so the last dispatch
        // round is short waves.  K2 6.70 -> 6.49 ms; sixteenth / eighth /
        // quarter of the rows at 2x / 4x / 8x lanes all land within 6.49-6.54.
#ifndef PT_TAIL_FRAC
#define PT_TAIL_FRAC 16
#endif
#ifndef PT_TAIL_MUL
#define PT_TAIL_MUL 3
#endif
        constexpr int kTailFrac = PT_TAIL_FRAC;
        constexpr uint32_t kTailMul = PT_TAIL_MUL;   // log2 of the lane multiplier
        uint32_t cap = 64;
        while (cap > 1 && (int32_t)cap > p->spp) cap >>= 1;
        const uint32_t tl = std::min(R.split_log2 + kTailMul, (uint32_t)__builtin_ctz(cap));
        const int32_t thresh = p->height - (p->height + kTailFrac - 1) / kTailFrac;
        int32_t ra = 0;   // band rows below the threshold (a prefix: rows ascend)
        while (ra < rows && first + ra * p->row_step < thresh) ++ra;
        // (no tail when this launch's lanes would overflow the 32-bit lane index)
        const uint64_t lanes = (uint64_t)ra * p->width * R.split + 64 +
                               (((uint64_t)(rows - ra) * (uint64_t)p->width) << tl);
        if (tl > R.split_log2 && ra < rows && lanes < ((uint64_t)1 << 32)) {
            R.tail_pix = (uint32_t)ra * (uint32_t)p->width;
            R.tail_lane = (R.tail_pix * R.split + 63u) & ~63u;
            R.tail_log2 = tl;
        }
    }
    const uint64_t threads = (uint64_t)R.tail_lane + ((uint64_t)(R.npix - R.tail_pix) << R.tail_log2);
    if ((uint64_t)R.npix * R.split >= ((uint64_t)1 << 32) || threads >= ((uint64_t)1 << 32))
        return fail(PT_EINVAL, "launch needs 2^32 or more work-items (32-bit lane index)");
    // launches on one handle share its scratch (wavefront state, counters,
    // events): order this one after the previous launch, whatever stream
    // that one ran on
    if (s->timed) HIPCHK(hipStreamWaitEvent(st, s->ev1, 0));
    const dim3 grid((unsigned)((threads + 255) / 256));   // (the wavefront's slots)
    const dim3 rgrid((unsigned)((threads + kRenderBlock - 1) / kRenderBlock)), rblock(kRenderBlock);
    const bool count = (p->flags & PT_FLAG_COUNT) != 0;
    const bool f64 = (p->flags & PT_FLAG_FORCE_F64) != 0;
    // BVH scenes render through the wavefront kernels unless the caller asks
    // for the single kernel (and for counting / forced-f64 launches, which
    // only the single kernel implements; and for launches of 2^29 or more
    // path slots, beyond the shadow lists' (slot << 2) | ray entries — the
    // single kernel's framebuffer is the same bit for bit)
    const bool wavefront = s->dev.n_bnode > 0 && !count && !f64 &&
                           !(p->flags & PT_FLAG_MEGAKERNEL) && s->dev.n_qnode > 0 &&
                           s->dev.qstack <= kWalkStack && (uint64_t)grid.x * 256u < ((uint64_t)1 << 29);
    if (wavefront) return render_wavefront(s, R, grid, out_dev, st, p->flags, stats);
    if (count) HIPCHK(hipMemsetAsync(s->stats, 0, sizeof(StatsDev), st));
    HIPCHK(hipEventRecord(s->ev0, st));
    if (f64) {
        if (count) hipLaunchKernelGGL((k_render<true, true, true>), rgrid, rblock, 0, st, s->dev, R, out_dev, s->stats);
        else hipLaunchKernelGGL((k_render<true, false, true>), rgrid, rblock, 0, st, s->dev, R, out_dev, s->stats);
    } else if (s->dev.n_bnode > 0) {   // scenes with meshes: the BVH instantiation
        if (count) hipLaunchKernelGGL((k_render<false, true, true>), rgrid, rblock, 0, st, s->dev, R, out_dev, s->stats);
        else hipLaunchKernelGGL((k_render<false, false, true>), rgrid, rblock, 0, st, s->dev, R, out_dev, s->stats);
    } else {
        if (count) hipLaunchKernelGGL((k_render<false, true, false>), rgrid, rblock, 0, st, s->dev, R, out_dev, s->stats);
        else hipLaunchKernelGGL((k_render<false, false, false>), rgrid, rblock, 0, st, s->dev, R, out_dev, s->stats);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(s->ev1, st));
    s->timed = true;
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        if (count) {
            StatsDev h;
            HIPCHK(hipMemcpyAsync(&h, s->stats, sizeof(h), hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            stats->closest_tests = h.v[0];
            stats->shadow_tests = h.v[1];
            stats->ray_bounces = h.v[2];
            stats->shading_points = h.v[3];
            stats->light_hits = h.v[4];
            stats->escapes = h.v[5];
            stats->f64_fallbacks = h.v[6];
            stats->f64_rescans = h.v[7];
        }
    }
    return PT_OK;
}

int pt_render(pt_scene* s, const pt_render_params* p, void* out_host, pt_stats* stats) {
    int rc = validate(p);
    if (rc) return rc;
    if (!s) return fail(PT_EINVAL, "null scene");
    int32_t first = 0, rows = 0;
    band_layout(p, &first, &rows);
    if (rows == 0) return PT_OK;
    if (!out_host) return fail(PT_EINVAL, "null output");
    DeviceGuard g(s->device);
    const size_t elem = (p->flags & PT_FLAG_OUT_F64) ? sizeof(double) : sizeof(float);
    const size_t row_bytes = (size_t)p->width * 3 * elem;
    const size_t bytes = (size_t)rows * row_bytes;
    if (bytes > s->out_cap) {
        if (s->out_dev) (void)hipFree(s->out_dev);
        s->out_dev = nullptr;
        s->out_cap = 0;
        HIPCHK(hipMalloc(&s->out_dev, bytes));
        s->out_cap = bytes;
    }
    pt_render_params q = *p;   // packed in the staging buffer, strided on the host
    q.out_row_stride = 0;
    rc = pt_render_device(s, &q, s->out_dev, s->stream, stats);
    if (rc) return rc;
    if (p->out_row_stride == 0 || (size_t)p->out_row_stride * elem == row_bytes)
        HIPCHK(hipMemcpyAsync(out_host, s->out_dev, bytes, hipMemcpyDeviceToHost, s->stream));
    else
        HIPCHK(hipMemcpy2DAsync(out_host, (size_t)p->out_row_stride * elem, s->out_dev, row_bytes,
                                row_bytes, (size_t)rows, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return PT_OK;
}

}  // extern "C"

static void add_stats(pt_stats* d, const pt_stats& s) {
    d->closest_tests += s.closest_tests; d->shadow_tests += s.shadow_tests;
    d->ray_bounces += s.ray_bounces; d->shading_points += s.shading_points;
    d->light_hits += s.light_hits; d->escapes += s.escapes;
    d->f64_fallbacks += s.f64_fallbacks; d->f64_rescans += s.f64_rescans;
    d->shadow_queries += s.shadow_queries; d->shadow_node_visits += s.shadow_node_visits;
    d->shadow_leaf_units += s.shadow_leaf_units; d->closest_queries += s.closest_queries;
    d->closest_node_visits += s.closest_node_visits; d->closest_leaf_units += s.closest_leaf_units;
    d->shade_ms += s.shade_ms; d->shadow_ms += s.shadow_ms; d->closest_ms += s.closest_ms;
    d->shade_launches += s.shade_launches; d->shadow_launches += s.shadow_launches;
    d->closest_launches += s.closest_launches;
    d->sort_ms += s.sort_ms; d->sort_launches += s.sort_launches;
}
static_assert(sizeof(pt_stats) == 19 * 8 + 3 * 8, "add_stats covers every pt_stats field");

extern "C" {

// Waits for the work already queued on the first n handles' streams (the
// error path of pt_render_multi: asynchronous band renders and copies of
// devices launched before the failing one must not outlive the call).
static void drain(pt_scene* const* scenes, int32_t n) {
    for (int32_t i = 0; i < n; ++i) {
        DeviceGuard g(scenes[i]->device);
        (void)hipStreamSynchronize(scenes[i]->stream);
    }
}

int pt_render_multi(pt_scene* const* scenes, int32_t n, const pt_render_params* p, void* out_host,
                    pt_stats* stats) {
    if (!scenes || n <= 0) return fail(PT_EINVAL, "need n >= 1 scene handles");
    for (int32_t i = 0; i < n; ++i) {
        if (!scenes[i]) return fail(PT_EINVAL, "null scene handle");
        if (scenes[i]->fingerprint != scenes[0]->fingerprint)
            return fail(PT_EINVAL, "handle " + std::to_string(i) + " holds another scene than handle 0");
    }
    int rc = validate(p);
    if (rc) return rc;
    // fault injection for the tests of the error path (pt_test_fault_inject):
    // dealing band i fails after bands 0..i-1 were launched
    const int32_t fail_at = g_fault_multi.load();
    if (p->row_step != 1) return fail(PT_EINVAL, "pt_render_multi deals out the rows itself: row_step must be 1");
    if (p->out_row_stride != 0) return fail(PT_EINVAL, "pt_render_multi writes the packed layout: out_row_stride must be 0");
    int32_t first = 0, total = 0;
    band_layout(p, &first, &total);
    if (total == 0) return PT_OK;
    if (!out_host) return fail(PT_EINVAL, "null output");
    const int32_t rb = first, re = first + total;   // the rows, clamped to the image
    const size_t elem = (p->flags & PT_FLAG_OUT_F64) ? sizeof(double) : sizeof(float);
    const size_t row_bytes = (size_t)p->width * 3 * elem;
    // any stats-producing flag: every device's pt_stats is summed field by
    // field (counts and the kernel-time sums alike)
    const bool count = (p->flags & (PT_FLAG_COUNT | PT_FLAG_WALK_COUNT | PT_FLAG_KERNEL_TIMES)) != 0;
    if (stats) memset(stats, 0, sizeof(*stats));
    std::vector<pt_render_params> bp(n);
    std::vector<int32_t> rows(n, 0);
    // 1. every device renders its band into its staging buffer (asynchronous);
    // a failure drains the devices launched so far (and this one) first
    for (int32_t i = 0; i < n; ++i) {
        pt_scene* s = scenes[i];
        bp[i] = *p;
        bp[i].row_begin = rb;
        bp[i].row_end = re;
        bp[i].row_step = n;
        bp[i].row_phase = (rb + i) % n;
        int32_t f = 0;
        band_layout(&bp[i], &f, &rows[i]);
        if (rows[i] == 0) continue;
        int rci = PT_OK;
        {
            DeviceGuard g(s->device);
            const size_t bytes = (size_t)rows[i] * row_bytes;
            if (bytes > s->out_cap) {
                // (the handle's previous work may still read or write it)
                if (hipStreamSynchronize(s->stream) != hipSuccess) {
                    rci = fail(PT_EHIP, "hipStreamSynchronize before growing a staging buffer failed");
                } else {
                    if (s->out_dev) (void)hipFree(s->out_dev);
                    s->out_dev = nullptr;
                    s->out_cap = 0;
                    if (hipMalloc(&s->out_dev, bytes) != hipSuccess)
                        rci = fail(PT_ENOMEM, "hipMalloc band staging buffer");
                    else
                        s->out_cap = bytes;
                }
            }
            if (rci == PT_OK && i == fail_at) rci = fail(PT_EHIP, "fault injected (pt_test_fault_inject)");
            if (rci == PT_OK) {
                pt_stats st;
                rci = pt_render_device(s, &bp[i], s->out_dev, s->stream, (count && stats) ? &st : nullptr);
                if (rci == PT_OK && count && stats) add_stats(stats, st);
            }
        }
        if (rci != PT_OK) {
            const std::string msg = g_err;
            drain(scenes, i + 1);
            g_err = "device " + std::to_string(i) + ": " + msg;
            return rci;
        }
    }
    // 2. each band lands in its rows of the host frame: band row j (launch
    // order, highest iy first) is frame row (re-1-iy) = (re-1-iy_top) + j*n
    for (int32_t i = 0; i < n; ++i) {
        if (rows[i] == 0) continue;
        pt_scene* s = scenes[i];
        DeviceGuard g(s->device);
        const int32_t phase = bp[i].row_phase;
        int32_t iy_top = re - 1;
        while (((iy_top % n) + n) % n != phase) --iy_top;
        char* dst = (char*)out_host + (size_t)(re - 1 - iy_top) * row_bytes;
        if (hipMemcpy2DAsync(dst, (size_t)n * row_bytes, s->out_dev, row_bytes, row_bytes, (size_t)rows[i],
                             hipMemcpyDeviceToHost, s->stream) != hipSuccess) {
            drain(scenes, n);
            return fail(PT_EHIP, "hipMemcpy2DAsync of device " + std::to_string(i) + "'s band failed");
        }
    }
    int rc_sync = PT_OK;
    for (int32_t i = 0; i < n; ++i) {
        DeviceGuard g(scenes[i]->device);
        if (hipStreamSynchronize(scenes[i]->stream) != hipSuccess && rc_sync == PT_OK)
            rc_sync = fail(PT_EHIP, "hipStreamSynchronize of device " + std::to_string(i) + " failed");
    }
    return rc_sync;
}

int pt_host_map(void* host, uint64_t bytes, void** dev_ptr) {
    if (!host || !dev_ptr || bytes == 0) return fail(PT_EINVAL, "need host, bytes > 0 and dev_ptr");
    *dev_ptr = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(PT_ENODEV, "no HIP device visible (the MI355X path needs a gfx950 GPU)");
    HIPCHK(hipHostRegister(host, (size_t)bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    void* d = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&d, host, 0);
    if (e != hipSuccess) {
        (void)hipHostUnregister(host);
        return fail(PT_EHIP, std::string("hipHostGetDevicePointer failed: ") + hipGetErrorString(e));
    }
    *dev_ptr = d;
    return PT_OK;
}

int pt_host_unmap(void* host) {
    if (!host) return fail(PT_EINVAL, "null host pointer");
    HIPCHK(hipHostUnregister(host));
    return PT_OK;
}

int pt_signal(uint64_t* flag_dev, uint64_t value, void* stream) {
    if (!flag_dev || ((uintptr_t)flag_dev & 7u)) return fail(PT_EINVAL, "need an 8-byte aligned flag");
    hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, (hipStream_t)stream, flag_dev, value);
    HIPCHK(hipGetLastError());
    return PT_OK;
}

int pt_wait_flags(const uint64_t* flags, int32_t n, int32_t stride, uint64_t value, double timeout_s) {
    if (!flags || n < 0 || stride <= 0) return fail(PT_EINVAL, "need flags, n >= 0, stride > 0");
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
        int32_t i = 0;
        while (i < n && __atomic_load_n(&flags[(size_t)i * stride], __ATOMIC_RELAXED) >= value) ++i;
        if (i == n) break;
        if ((spin & 1023u) == 1023u &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
            return fail(PT_ETIMEOUT, "pt_wait_flags: flag " + std::to_string(i) + " below " +
                                         std::to_string(value) + " after " + std::to_string(timeout_s) + " s");
        __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return PT_OK;
}

int pt_last_kernel_ms(pt_scene* s, float* ms) {
    if (!s || !ms) return fail(PT_EINVAL, "null argument");
    if (!s->timed) return fail(PT_EINVAL, "no launch recorded yet");
    DeviceGuard g(s->device);
    HIPCHK(hipEventSynchronize(s->ev1));
    HIPCHK(hipEventElapsedTime(ms, s->ev0, s->ev1));
    return PT_OK;
}

int pt_image_u8_device(const void* fb_dev, int32_t width, int32_t height, uint32_t flags,
                       void* out_u8_dev, void* stream) {
    if (!fb_dev || !out_u8_dev) return fail(PT_EINVAL, "null buffer");
    if (width <= 0 || height <= 0) return fail(PT_EINVAL, "need width, height > 0");
    const int64_t n = (int64_t)width * height * 3;
    hipStream_t st = (hipStream_t)stream;
#ifndef PT_IMAGE_V2
#define PT_IMAGE_V2 1
#endif
    if (PT_IMAGE_V2) {   // pt_image.h: per-block partials, no atomics and no fills
        const int vec = ((uintptr_t)fb_dev % 16 == 0) && ((uintptr_t)out_u8_dev % 4 == 0);
        const int pblocks = (int)std::max<int64_t>(1, std::min<int64_t>((n / 4 + 255) / 256, kImgBlocks));
#ifndef PT_IMG_U8_BLOCKS
#define PT_IMG_U8_BLOCKS 2048
#endif
        const int ublocks = (int)std::max<int64_t>(1, std::min<int64_t>((n / 16 + 255) / 256, PT_IMG_U8_BLOCKS));
        double* part = nullptr;
        HIPCHK(hipMallocAsync((void**)&part, 2 * sizeof(double) * (size_t)pblocks, st));
        if (flags & PT_FLAG_OUT_F64) {
            hipLaunchKernelGGL(k_minmax2<double>, dim3(pblocks), dim3(256), 0, st, (const double*)fb_dev, n, vec,
                               part);
            hipLaunchKernelGGL(k_to_u8_2<double>, dim3(ublocks), dim3(256), 0, st, (const double*)fb_dev, n, vec,
                               part, pblocks, (uint8_t*)out_u8_dev);
        } else {
            hipLaunchKernelGGL(k_minmax2<float>, dim3(pblocks), dim3(256), 0, st, (const float*)fb_dev, n, vec,
                               part);
            hipLaunchKernelGGL(k_to_u8_2<float>, dim3(ublocks), dim3(256), 0, st, (const float*)fb_dev, n, vec,
                               part, pblocks, (uint8_t*)out_u8_dev);
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipFreeAsync(part, st));
        return PT_OK;
    }
    unsigned long long* keys = nullptr;
    HIPCHK(hipMallocAsync((void**)&keys, 2 * sizeof(unsigned long long), st));
    HIPCHK(hipMemsetAsync(keys, 0xff, sizeof(unsigned long long), st));
    HIPCHK(hipMemsetAsync(keys + 1, 0, sizeof(unsigned long long), st));
    // 4 elements per thread step when the buffers allow 16-byte loads and
    // 4-byte stores; ~8 blocks per CU of grid-stride work
    const int vec = ((uintptr_t)fb_dev % 16 == 0) && ((uintptr_t)out_u8_dev % 4 == 0);
    const int blocks = (int)std::min<int64_t>((n / 4 + 255) / 256 + 1, 2048);
    if (flags & PT_FLAG_OUT_F64) {
        hipLaunchKernelGGL(k_minmax<double>, dim3(blocks), dim3(256), 0, st, (const double*)fb_dev, n, vec, keys);
        hipLaunchKernelGGL(k_to_u8<double>, dim3(blocks), dim3(256), 0, st, (const double*)fb_dev, n, vec, keys,
                           (uint8_t*)out_u8_dev);
    } else {
        hipLaunchKernelGGL(k_minmax<float>, dim3(blocks), dim3(256), 0, st, (const float*)fb_dev, n, vec, keys);
        hipLaunchKernelGGL(k_to_u8<float>, dim3(blocks), dim3(256), 0, st, (const float*)fb_dev, n, vec, keys,
                           (uint8_t*)out_u8_dev);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipFreeAsync(keys, st));
    return PT_OK;
}

int pt_assemble_bands_device(const void* tiles_dev, int32_t world, int32_t max_rows, int32_t width,
                             int32_t height, uint32_t flags, void* out_dev, void* stream) {
    if (!tiles_dev || !out_dev) return fail(PT_EINVAL, "null buffer");
    if (world <= 0 || width <= 0 || height <= 0) return fail(PT_EINVAL, "need world, width, height > 0");
    if (max_rows < (height + world - 1) / world)
        return fail(PT_EINVAL, "max_rows is smaller than the largest band (ceil(height / world))");
    const int64_t row_bytes = (int64_t)width * 3 * ((flags & PT_FLAG_OUT_F64) ? 8 : 4);
    const bool v16 = row_bytes % 16 == 0 && (uintptr_t)tiles_dev % 16 == 0 && (uintptr_t)out_dev % 16 == 0;
    const int64_t units = row_bytes / (v16 ? 16 : 4);
    const int64_t n = (int64_t)height * units;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    if (v16)
        hipLaunchKernelGGL(k_assemble_bands<uint4>, grid, block, 0, st, (const uint4*)tiles_dev, world, max_rows,
                           height, units, (uint4*)out_dev);
    else
        hipLaunchKernelGGL(k_assemble_bands<uint32_t>, grid, block, 0, st, (const uint32_t*)tiles_dev, world,
                           max_rows, height, units, (uint32_t*)out_dev);
    HIPCHK(hipGetLastError());
    return PT_OK;
}

int pt_image_u8(const void* fb_host, int32_t width, int32_t height, uint32_t flags,
                uint8_t* out_u8_host) {
    if (!fb_host || !out_u8_host) return fail(PT_EINVAL, "null buffer");
    if (width <= 0 || height <= 0) return fail(PT_EINVAL, "need width, height > 0");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(PT_ENODEV, "no HIP device");
    const size_t n = (size_t)width * height * 3;
    const size_t in_bytes = n * ((flags & PT_FLAG_OUT_F64) ? sizeof(double) : sizeof(float));
    void *d_in = nullptr, *d_out = nullptr;
    HIPCHK(hipMalloc(&d_in, in_bytes));
    if (hipMalloc(&d_out, n) != hipSuccess) {
        (void)hipFree(d_in);
        return fail(PT_ENOMEM, "hipMalloc failed");
    }
    int rc = PT_OK;
    if (hipMemcpy(d_in, fb_host, in_bytes, hipMemcpyHostToDevice) != hipSuccess)
        rc = fail(PT_EHIP, "hipMemcpy to device failed");
    if (!rc) rc = pt_image_u8_device(d_in, width, height, flags, d_out, nullptr);
    if (!rc && hipMemcpy(out_u8_host, d_out, n, hipMemcpyDeviceToHost) != hipSuccess)
        rc = fail(PT_EHIP, "hipMemcpy to host failed");
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return rc;
}

struct pt_mesh_impl {
    pt_mesh pub;
    MeshOut data;
};

int pt_obj_load(const char* path, pt_mesh** out) {
    if (!path || !out) return fail(PT_EINVAL, "null argument");
    *out = nullptr;
    pt_mesh_impl* m = new (std::nothrow) pt_mesh_impl();
    if (!m) return fail(PT_ENOMEM, "out of host memory");
    int rc;
    try {
        rc = parse_obj_file(path, &m->data);
    } catch (const std::bad_alloc&) {
        delete m;
        return fail(PT_ENOMEM, "out of host memory");
    }
    if (rc != kIngestOk) {
        delete m;
        if (rc == kIngestIo) return fail(PT_EINVAL, std::string("cannot read ") + path);
        return fail(PT_EUNSUPPORTED, rc == kIngestDivZero
                                         ? "zero-area triangle (the reference divides by zero)"
                                         : "input outside the fast reader's subset");
    }
    const MeshOut& d = m->data;
    m->pub.n_vert = (int64_t)(d.vert.size() / 3);
    m->pub.n_tri = (int64_t)d.tri_area.size();
    m->pub.n_skip = (int64_t)d.skip_off.size();
    m->pub.vert = d.vert.data();
    m->pub.face = d.face.data();
    m->pub.tri_v = d.tri_v.data();
    m->pub.tri_n = d.tri_n.data();
    m->pub.tri_area = d.tri_area.data();
    m->pub.skip_off = d.skip_off.data();
    m->pub.skip_len = d.skip_len.data();
    *out = &m->pub;
    return PT_OK;
}

void pt_mesh_free(pt_mesh* m) {
    delete reinterpret_cast<pt_mesh_impl*>(m);   // pub is the first member
}

int pt_intersect_objects(pt_scene* s, const double* rays, int64_t n, int32_t* out_tri,
                         double* out_p) {
    if (!s || (n > 0 && (!rays || !out_tri || !out_p))) return fail(PT_EINVAL, "null argument");
    if (n <= 0) return PT_OK;
    DeviceGuard g(s->device);
    double *d_rays = nullptr, *d_p = nullptr;
    int32_t* d_tri = nullptr;
    int rc = dev_alloc_copy(&d_rays, rays, (size_t)n * 6);
    if (!rc) rc = dev_alloc_copy(&d_p, (const double*)nullptr, (size_t)n * 3);
    if (!rc) rc = dev_alloc_copy(&d_tri, (const int32_t*)nullptr, (size_t)n);
    if (!rc) {
        hipLaunchKernelGGL(k_intersect, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s->stream,
                           s->dev, d_rays, n, s->xb_surf, s->xb_all, d_tri, d_p);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
        if (e == hipSuccess) e = hipMemcpy(out_tri, d_tri, n * sizeof(int32_t), hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(out_p, d_p, n * 3 * sizeof(double), hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = fail(PT_EHIP, std::string("k_intersect: ") + hipGetErrorString(e));
    }
    if (d_rays) (void)hipFree(d_rays);
    if (d_p) (void)hipFree(d_p);
    if (d_tri) (void)hipFree(d_tri);
    return rc;
}

int pt_compute_color(pt_scene* s, const int32_t* obj, const double* point, const double* normal,
                     const double* u, int64_t n, double* out_rgb) {
    if (!s || (n > 0 && (!obj || !point || !normal || !u || !out_rgb)))
        return fail(PT_EINVAL, "null argument");
    if (n <= 0) return PT_OK;
    for (int64_t i = 0; i < n; ++i)
        if (obj[i] < 0 || obj[i] >= s->host.k.n_obj) return fail(PT_EINVAL, "object index out of range");
    DeviceGuard g(s->device);
    int32_t* d_obj = nullptr;
    double *d_pt = nullptr, *d_n = nullptr, *d_u = nullptr, *d_out = nullptr;
    int rc = dev_alloc_copy(&d_obj, obj, (size_t)n);
    if (!rc) rc = dev_alloc_copy(&d_pt, point, (size_t)n * 3);
    if (!rc) rc = dev_alloc_copy(&d_n, normal, (size_t)n * 3);
    if (!rc) rc = dev_alloc_copy(&d_u, u, (size_t)n * 12);
    if (!rc) rc = dev_alloc_copy(&d_out, (const double*)nullptr, (size_t)n * 3);
    if (!rc) {
        hipLaunchKernelGGL(k_color, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s->stream,
                           s->dev, d_obj, d_pt, d_n, d_u, n, s->xb_surf, s->xb_all, d_out);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
        if (e == hipSuccess) e = hipMemcpy(out_rgb, d_out, n * 3 * sizeof(double), hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = fail(PT_EHIP, std::string("k_color: ") + hipGetErrorString(e));
    }
    for (void* p : {(void*)d_obj, (void*)d_pt, (void*)d_n, (void*)d_u, (void*)d_out})
        if (p) (void)hipFree(p);
    return rc;
}

}  // extern "C"
