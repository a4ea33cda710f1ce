// Shared device helpers for the gfx950 kernels of avse_challenge_amd.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/avse_hip.h"

#define AVSE_LOG2E 1.4426950408889634f
#define AVSE_LN2 0.6931471805599453f

#define AVSE_CHECK_LAUNCH()                                  \
    do {                                                     \
        if (hipGetLastError() != hipSuccess) return AVSE_ELAUNCH; \
    } while (0)

namespace avse {

// ---------------------------------------------------------------- dtype helpers
template <typename T> struct io;
template <> struct io<float> {
    __device__ static inline float ld(const float* p) { return *p; }
    __device__ static inline void st(float* p, float v) { *p = v; }
};
struct bf16_t { uint16_t x; };
template <> struct io<bf16_t> {
    __device__ static inline float ld(const bf16_t* p) {
        uint32_t u = ((uint32_t)p->x) << 16;
        return __uint_as_float(u);
    }
    __device__ static inline void st(bf16_t* p, float v) {
        // round-to-nearest-even, NaN preserved (MI355X_MICROARCH 'Correctness boundaries')
        uint32_t u = __float_as_uint(v);
        if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) {
            p->x = (uint16_t)((u >> 16) | 0x40);
            return;
        }
        u += 0x7fffu + ((u >> 16) & 1u);
        p->x = (uint16_t)(u >> 16);
    }
};

// Raw buffer loads: 32-bit per-lane voffset + wave-uniform soffset (an SGPR), hardware range check
// (out-of-range reads return 0).  Used for the strided row gathers of the scan so that 16 rows
// per tensor cost ONE address VGPR (the row step goes in soffset), not 16 64-bit pointers.
template <typename T> struct bufld;
template <> struct bufld<float> {
    __device__ static inline float ld(__amdgpu_buffer_rsrc_t r, int voff_elems, int soff_elems) {
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff_elems * 4, soff_elems * 4, 0));
    }
};
template <> struct bufld<bf16_t> {
    __device__ static inline float ld(__amdgpu_buffer_rsrc_t r, int voff_elems, int soff_elems) {
        const unsigned short v = __builtin_amdgcn_raw_buffer_load_b16(r, voff_elems * 2, soff_elems * 2, 0);
        return __uint_as_float(((uint32_t)v) << 16);
    }
};
template <> struct bufld<uint8_t> {
    __device__ static inline float ld(__amdgpu_buffer_rsrc_t r, int voff_elems, int soff_elems) {
        return (float)__builtin_amdgcn_raw_buffer_load_b8(r, voff_elems, soff_elems, 0);
    }
};
template <typename T> struct bufst;
template <> struct bufst<float> {
    __device__ static inline void st(__amdgpu_buffer_rsrc_t r, int voff_elems, int soff_elems, float v) {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff_elems * 4, soff_elems * 4, 0);
    }
};
template <> struct bufst<bf16_t> {
    __device__ static inline void st(__amdgpu_buffer_rsrc_t r, int voff_elems, int soff_elems, float v) {
        bf16_t h;
        io<bf16_t>::st(&h, v);
        __builtin_amdgcn_raw_buffer_store_b16(h.x, r, voff_elems * 2, soff_elems * 2, 0);
    }
};
template <typename T>
__device__ inline __amdgpu_buffer_rsrc_t make_rsrc(const T* base, int64_t n_elems) {
    int64_t bytes = n_elems * (int64_t)sizeof(T);
    if (bytes > 0x7FFFFFFFLL) bytes = 0x7FFFFFFFLL;
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

__device__ inline float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// packed fp32 pair: v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32 do two lanes' worth of f32 math per
// issue (MI355X: 64 FLOP/clk/SIMD for v_pk_fma_f32 vs 32 for v_fma_f32)
typedef float f2_t __attribute__((ext_vector_type(2)));
__device__ inline f2_t pkfma(f2_t a, f2_t b, f2_t c) { return __builtin_elementwise_fma(a, b, c); }
__device__ inline f2_t exp2_2(f2_t x) { return f2_t{__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)}; }
__device__ inline float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * AVSE_LOG2E); }

__device__ inline float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// softplus with the threshold mamba's kernels and torch use (x > 20 -> x).  log1p(t) via the
// hardware log2 with Kahan's correction (u = 1 + t; log1p(t) = log(u) * t / (u - 1)), which keeps
// ~1 ulp for tiny t (dt biases sit at softplus^-1 of [1e-3, 1e-1]) without the libm call and its
// branches; exp / rcp are the hardware instructions.
// Branch-free: both sides are computed and selected (v_cndmask), so a loop of softplus calls has no
// exec-mask branches (the unselected side may be inf / NaN for x > 88 or t ~ 0; it is discarded).
__device__ inline float softplus(float x) {
    const float t = fast_exp(x);
    const float u = 1.f + t;
    const float lp = __builtin_amdgcn_logf(u) * AVSE_LN2 * t * fast_rcp(u - 1.f);
    const float r = (u == 1.f) ? t : lp;
    return (x > 20.f) ? x : r;
}
// The same value with two transcendentals instead of three: log1p(t) = log(u + c) with u = fl(1 + t) and
// c = t - (u - 1) the rounding error of that sum (u - 1 is exact for t < 3), so log1p(t) = log(u) + c/u + O(c^2);
// taking c for c/u errs by |c| t / (1 + t) <= 2^-24 t, i.e. below one ulp of log1p(t) ~ t for tiny t (u == 1 gives
// log(u) = 0 and c = t exactly) and far below it for t ~ 1.  No rcp, no u == 1 select.
__device__ inline float softplus2(float x) {
    const float t = fast_exp(x);
    const float u = 1.f + t;
    const float c = t - (u - 1.f);
    const float r = __builtin_fmaf(__builtin_amdgcn_logf(u), AVSE_LN2, c);
    return (x > 20.f) ? x : r;
}
__device__ inline float sigmoidf_(float x) { return fast_rcp(1.f + fast_exp(-x)); }
__device__ inline float siluf_(float x) { return x * sigmoidf_(x); }

// ---------------------------------------------------------------- cross-lane (wave64)
// xor-1 / xor-2 inside a quad via DPP quad_perm (a single VALU op with the add folded in)
__device__ inline float dpp_xor1(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
}
__device__ inline float dpp_xor2(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));
}
// xor 4/8/16 within 32-lane halves: ds_swizzle bitmask mode (and=0x1f, xor=m)
template <int M>
__device__ inline float swz_xor(float v) {
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x1F | (M << 10)));
}
__device__ inline float xor32(float v) { return __shfl_xor(v, 32, 64); }

template <int M>
__device__ inline float lane_xor(float v) {
    if constexpr (M == 1) return dpp_xor1(v);
    else if constexpr (M == 2) return dpp_xor2(v);
    else if constexpr (M == 32) return xor32(v);
    else return swz_xor<M>(v);
}

// sum over the G lanes sharing (lane / G) — G in {1, 2, 4}
template <int G>
__device__ inline float group_sum(float v) {
    if constexpr (G >= 2) v += dpp_xor1(v);
    if constexpr (G >= 4) v += dpp_xor2(v);
    return v;
}

// XCD-aware bijective remap of a 1-D block id (cdna_hip_programming.md §5 'XCD swizzle must be
// bijective'): consecutive logical ids land on the same XCD (speed only, never correctness).
__device__ inline int xcd_remap(int orig, int nwg) {
    const int nx = 8;
    int q = nwg / nx, r = nwg % nx;
    int xcd = orig % nx, k = orig / nx;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

}  // namespace avse
