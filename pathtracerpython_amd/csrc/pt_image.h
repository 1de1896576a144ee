// pt_image.h — image finalisation of the reference's make_image
// (utils.py:150-161) on the device: global min over the whole H x W x 3
// array, shift, divide by the shifted maximum, x255, truncation to uint8.
//
// Two passes over the framebuffer (HBM-bound: 2 reads of 12 B (f32) or
// 24 B (f64) per pixel + a 3 B write).  Version 1 (PT_IMAGE_V2=0; version 2
// below is the default):
//   k_minmax  grid-stride reduction; each block folds its min/max into two
//             64-bit keys with one atomicMin/atomicMax (an order-preserving
//             map of the doubles, so the result is exact and independent of
//             the order blocks finish in);
//   k_to_u8   elementwise ((x - min) / (max - min)) * 255 -> uint8, in f64
//             as numpy does.
// numpy semantics kept: a NaN anywhere makes every output NaN, which
// astype('uint8') turns into 0 on x86; a constant image (max - min == 0)
// gives 0/0 = NaN -> 0 as well.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pt {

// order-preserving double -> uint64 (for atomicMin/atomicMax on the bits)
__device__ __forceinline__ uint64_t order_key(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double key_value(uint64_t k) {
    const uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double((long long)b);
}

template <typename T>
__device__ __forceinline__ double load_f64(const T* p, int64_t i) { return (double)p[i]; }

// 4 consecutive elements as doubles (one 16-byte load for f32, two for f64);
// the caller guarantees 16-byte alignment of p + 4i
__device__ __forceinline__ void load4(const float* p, int64_t i, double v[4]) {
    const float4 f = reinterpret_cast<const float4*>(p)[i];
    v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
}
__device__ __forceinline__ void load4(const double* p, int64_t i, double v[4]) {
    const double2 a = reinterpret_cast<const double2*>(p)[2 * i];
    const double2 b = reinterpret_cast<const double2*>(p)[2 * i + 1];
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
}

// keys[0] = min key (init ~0), keys[1] = max key (init 0).  Vector body over
// n4 = n/4 groups when `vec` (16-byte aligned input), scalar tail.
template <typename T>
__global__ __launch_bounds__(256) void k_minmax(const T* __restrict__ fb, int64_t n, int vec,
                                                unsigned long long* __restrict__ keys) {
    uint64_t kmin = ~0ull, kmax = 0ull;
    const int64_t stride = (int64_t)gridDim.x * 256;
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n4 = vec ? n / 4 : 0;
    for (int64_t i = gid; i < n4; i += stride) {
        double v[4];
        load4(fb, i, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t k = order_key(v[j]);
            kmin = k < kmin ? k : kmin;
            kmax = k > kmax ? k : kmax;
        }
    }
    for (int64_t i = 4 * n4 + gid; i < n; i += stride) {
        const uint64_t k = order_key(load_f64(fb, i));
        kmin = k < kmin ? k : kmin;
        kmax = k > kmax ? k : kmax;
    }
    for (int m = 32; m >= 1; m >>= 1) {
        const uint64_t a = (uint64_t)__shfl_xor((unsigned long long)kmin, m);
        const uint64_t b = (uint64_t)__shfl_xor((unsigned long long)kmax, m);
        kmin = a < kmin ? a : kmin;
        kmax = b > kmax ? b : kmax;
    }
    __shared__ uint64_t smin[4], smax[4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { smin[w] = kmin; smax[w] = kmax; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int j = 1; j < 4; ++j) {
            kmin = smin[j] < kmin ? smin[j] : kmin;
            kmax = smax[j] > kmax ? smax[j] : kmax;
        }
        atomicMin(&keys[0], (unsigned long long)kmin);
        atomicMax(&keys[1], (unsigned long long)kmax);
    }
}

// NaN keys sit above +inf (positive NaN) or below -inf (negative NaN)
__device__ __forceinline__ bool key_is_nan(uint64_t k) {
    return k > 0xfff0000000000000ull || k < 0x000fffffffffffffull;
}

__device__ __forceinline__ uint32_t to_u8(double x, double mn, double mx, bool nan) {
    const double v = ((x - mn) / mx) * 255.0;
    // astype('uint8'): truncation; NaN (constant image 0/0, or a NaN input)
    // -> 0 as x86's conversion gives
    return (nan || !(v == v)) ? 0u : (uint32_t)(int)v;
}

// `vec`: input 16-byte and output 4-byte aligned -> 4 elements per step,
// one packed 32-bit store
template <typename T>
__global__ __launch_bounds__(256) void k_to_u8(const T* __restrict__ fb, int64_t n, int vec,
                                               const unsigned long long* __restrict__ keys,
                                               uint8_t* __restrict__ out) {
    const uint64_t kmin = keys[0], kmax = keys[1];
    const bool nan = key_is_nan(kmin) || key_is_nan(kmax);
    const double mn = key_value(kmin);
    const double mx = key_value(kmax) - mn;   // np.max(mat - min) = fl(max - min)
    const int64_t stride = (int64_t)gridDim.x * 256;
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n4 = vec ? n / 4 : 0;
    for (int64_t i = gid; i < n4; i += stride) {
        double v[4];
        load4(fb, i, v);
        uint32_t w = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) w |= to_u8(v[j], mn, mx, nan) << (8 * j);
        reinterpret_cast<uint32_t*>(out)[i] = w;
    }
    for (int64_t i = 4 * n4 + gid; i < n; i += stride)
        out[i] = (uint8_t)to_u8(load_f64(fb, i), mn, mx, nan);
}

// ---- version 2 (PT_IMAGE_V2, the default): no atomics, no fills --------
// k_minmax2  per-block min / max in the input type, NaN-propagating
//            (IEEE minimum/maximum: any NaN in the frame reaches the result),
//            four 16-byte loads in flight per lane and step (the one-load
//            loop above ran latency-bound at ~2.9 TB/s), one partial pair per
//            block into `part` (written by every block: no initialisation);
// k_to_u8_2  each block first folds the partials (<= kImgBlocks pairs, from
//            L2), then k_to_u8's element formula, four 4-element groups per
//            lane and step (2 or 4, 512 to 2048 blocks: within 1%; a
//            division-free form of the formula with an exact fallback near
//            integers did not move it either: the pass is memory-bound).
// min / max of f32 values taken in f32 are the f64 min / max of the same
// values (the conversion is exact and monotone).
constexpr int kImgBlocks = 1024;   // k_minmax2's grid at most (4 blocks per CU)

template <typename T>
__device__ __forceinline__ T nmin(T a, T b) { return __builtin_elementwise_minimum(a, b); }
template <typename T>
__device__ __forceinline__ T nmax(T a, T b) { return __builtin_elementwise_maximum(a, b); }

// 4 consecutive elements in their own type (16 B for f32, 32 B for f64)
__device__ __forceinline__ void load4t(const float* p, int64_t i, float v[4]) {
    const float4 f = reinterpret_cast<const float4*>(p)[i];
    v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
}
__device__ __forceinline__ void load4t(const double* p, int64_t i, double v[4]) {
    const double2 a = reinterpret_cast<const double2*>(p)[2 * i];
    const double2 b = reinterpret_cast<const double2*>(p)[2 * i + 1];
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
}

template <typename T>
__device__ __forceinline__ void fold4(const T v[4], T* mn, T* mx) {
    *mn = nmin(*mn, nmin(nmin(v[0], v[1]), nmin(v[2], v[3])));
    *mx = nmax(*mx, nmax(nmax(v[0], v[1]), nmax(v[2], v[3])));
}

// part[2b] = block b's minimum, part[2b + 1] its maximum (as doubles)
template <typename T>
__global__ __launch_bounds__(256) void k_minmax2(const T* __restrict__ fb, int64_t n, int vec,
                                                 double* __restrict__ part) {
    T mn = (T)INFINITY, mx = (T)-INFINITY;
    const int64_t stride = (int64_t)gridDim.x * 256;
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n4 = vec ? n / 4 : 0;
    int64_t i = gid;
    for (; i + 3 * stride < n4; i += 4 * stride) {   // four groups in flight
        T a[4], b[4], c[4], d[4];
        load4t(fb, i, a);
        load4t(fb, i + stride, b);
        load4t(fb, i + 2 * stride, c);
        load4t(fb, i + 3 * stride, d);
        fold4(a, &mn, &mx);
        fold4(b, &mn, &mx);
        fold4(c, &mn, &mx);
        fold4(d, &mn, &mx);
    }
    for (; i < n4; i += stride) {
        T a[4];
        load4t(fb, i, a);
        fold4(a, &mn, &mx);
    }
    for (int64_t j = 4 * n4 + gid; j < n; j += stride) {
        mn = nmin(mn, fb[j]);
        mx = nmax(mx, fb[j]);
    }
    for (int m = 32; m >= 1; m >>= 1) {
        mn = nmin(mn, (T)__shfl_xor(mn, m));
        mx = nmax(mx, (T)__shfl_xor(mx, m));
    }
    __shared__ T smin[4], smax[4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { smin[w] = mn; smax[w] = mx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = (double)nmin(nmin(smin[0], smin[1]), nmin(smin[2], smin[3]));
        part[2 * blockIdx.x + 1] = (double)nmax(nmax(smax[0], smax[1]), nmax(smax[2], smax[3]));
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_to_u8_2(const T* __restrict__ fb, int64_t n, int vec,
                                                 const double* __restrict__ part, int n_part,
                                                 uint8_t* __restrict__ out) {
    __shared__ double smin[4], smax[4];
    double pmn = INFINITY, pmx = -INFINITY;
    for (int j = threadIdx.x; j < n_part; j += 256) {
        pmn = nmin(pmn, part[2 * j]);
        pmx = nmax(pmx, part[2 * j + 1]);
    }
    for (int m = 32; m >= 1; m >>= 1) {
        pmn = nmin(pmn, __shfl_xor(pmn, m));
        pmx = nmax(pmx, __shfl_xor(pmx, m));
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { smin[w] = pmn; smax[w] = pmx; }
    __syncthreads();
    const double vmin = nmin(nmin(smin[0], smin[1]), nmin(smin[2], smin[3]));
    const double vmax = nmax(nmax(smax[0], smax[1]), nmax(smax[2], smax[3]));
    const bool nan = !(vmin == vmin) || !(vmax == vmax);
    const double mn = vmin;
    const double mx = vmax - mn;   // np.max(mat - min) = fl(max - min)
    const int64_t stride = (int64_t)gridDim.x * 256;
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n4 = vec ? n / 4 : 0;
    int64_t i = gid;
#ifndef PT_IMG_U8_DEPTH
#define PT_IMG_U8_DEPTH 4
#endif
    constexpr int D = PT_IMG_U8_DEPTH;   // groups in flight per lane
    for (; i + (D - 1) * stride < n4; i += D * stride) {
        T a[D][4];
#pragma unroll
        for (int g = 0; g < D; ++g) load4t(fb, i + g * stride, a[g]);
#pragma unroll
        for (int g = 0; g < D; ++g) {
            uint32_t wa = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) wa |= to_u8((double)a[g][j], mn, mx, nan) << (8 * j);
            reinterpret_cast<uint32_t*>(out)[i + g * stride] = wa;
        }
    }
    for (; i < n4; i += stride) {
        T a[4];
        load4t(fb, i, a);
        uint32_t wa = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) wa |= to_u8((double)a[j], mn, mx, nan) << (8 * j);
        reinterpret_cast<uint32_t*>(out)[i] = wa;
    }
    for (int64_t j = 4 * n4 + gid; j < n; j += stride)
        out[j] = (uint8_t)to_u8((double)fb[j], mn, mx, nan);
}

// Frame assembly of an interleaved multi-GPU render (the step after the
// RCCL gather): tiles = the gathered (world, max_rows, row)
// array, band r holding the image rows iy % world == r top-first (as
// pt_render_device writes a band); out = the (height, row) frame, row
// height-1-iy holding image row iy.  One work-item per V-sized piece of an
// output row (V = 16 B when every row offset is 16-B aligned, else 4 B):
// HBM-bound, one read and one write of the frame.
template <typename V>
__global__ __launch_bounds__(256) void k_assemble_bands(const V* __restrict__ tiles, int32_t world,
                                                        int32_t max_rows, int32_t height,
                                                        int64_t row_units, V* __restrict__ out) {
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid >= (int64_t)height * row_units) return;
    const int32_t fr = (int32_t)(gid / row_units);
    const int64_t c = gid - (int64_t)fr * row_units;
    const int32_t iy = height - 1 - fr;
    const int32_t r = iy % world, k = iy / world;
    const int32_t rows_r = (height - r + world - 1) / world;
    const int32_t j = rows_r - 1 - k;   // band row, top-first
    out[gid] = tiles[((int64_t)r * max_rows + j) * row_units + c];
}

}  // namespace pt
