// Depthwise causal conv1d (width <= 4, optional SiLU) forward / backward for gfx950.
//
// Replaces causal_conv1d_cuda.causal_conv1d_fwd / causal_conv1d_bwd (causal-conv1d
// 1.1.3.post1, un-vendored) called at
// /root/reference/Mamba-TasNet/modules/mamba/selective_scan_interface.py:182,244,286.
// Semantics pinned by the in-tree fallback bimamba.py:278-279:
//   out[b,d,t] = act(bias[d] + sum_k w[d,k] * x[b,d,t-(W-1)+k]),  x[<0] = 0.
// x / out / dout / dx are fp32 or bf16 (T; fp32 arithmetic, weights fp32), as causal-conv1d's
// kernels take the activation dtype under bf16 autocast.  One workgroup per (b, d) row; the row is streamed in TILE-sized pieces through LDS with a
// (W-1)-sample halo so every HBM byte is read once with lane-contiguous accesses (HBM-bound:
// fwd 2*4 B/elem, bwd 3*4 B/elem).  The backward reduces dweight/dbias per row in LDS and a
// second kernel sums the per-row partials over the batch (deterministic).
#include <algorithm>

#include "common.h"

namespace avse {
namespace cconv {

constexpr int THREADS = 256;
constexpr int PER = 8;                     // elements per thread per tile
constexpr int TILE = THREADS * PER;        // 2048
constexpr int MAXW = 4;

template <typename T, int W, bool SILU, bool HAS_BIAS>
__global__ __launch_bounds__(THREADS) void fwd_kernel(int D, int L, const T* __restrict__ x, int64_t x_bs,
                                                      int64_t x_ds, const float* __restrict__ w,
                                                      const float* __restrict__ bias, T* __restrict__ out,
                                                      int64_t o_bs, int64_t o_ds, int rev) {
    __shared__ float s[TILE + MAXW];
    const int row = blockIdx.x;
    const int b = row / D, d = row % D;
    const T* xr = x + b * x_bs + (int64_t)d * x_ds;
    T* orow = out + b * o_bs + (int64_t)d * o_ds;
    float wk[W];
#pragma unroll
    for (int k = 0; k < W; ++k) wk[k] = w[d * W + k];
    const float bv = HAS_BIAS ? bias[d] : 0.f;
    for (int t0 = 0; t0 < L; t0 += TILE) {
        __syncthreads();
        // s[i] holds x[t0 - (W-1) + i]
        for (int i = threadIdx.x; i < TILE + W - 1; i += THREADS) {
            const int t = t0 - (W - 1) + i;
            s[i] = (t >= 0 && t < L) ? io<T>::ld(&xr[rev ? L - 1 - t : t]) : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int p = 0; p < PER; ++p) {
            const int i = threadIdx.x + p * THREADS, t = t0 + i;
            if (t < L) {
                float acc = bv;
#pragma unroll
                for (int k = 0; k < W; ++k) acc += wk[k] * s[i + k];
                io<T>::st(&orow[rev ? L - 1 - t : t], SILU ? siluf_(acc) : acc);
            }
        }
    }
}

// dx_max (round 6): every row's max |dx| goes to the workspace after the rows' dw / db partials (wsmax[row]), and
// rowmax_kernel folds them into *dx_max with one atomic: one same-word atomic per wave of a (b * d)-row grid cost
// ~1.3 ms per C3 launch
__device__ inline float wave_max(float m) {
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    return m;
}

template <typename T, int W, bool SILU, bool HAS_BIAS>
__global__ __launch_bounds__(THREADS) void bwd_kernel(int D, int L, const T* __restrict__ x, int64_t x_bs,
                                                      int64_t x_ds, const float* __restrict__ w,
                                                      const float* __restrict__ bias, const T* __restrict__ dout,
                                                      int64_t g_bs, int64_t g_ds, T* __restrict__ dx,
                                                      int64_t dx_bs, int64_t dx_ds, float* __restrict__ ws, int rev,
                                                      int dx_acc, uint32_t* __restrict__ dx_max) {
    __shared__ float sx[TILE + 2 * MAXW];
    __shared__ float sg[TILE + MAXW];
    __shared__ float sred[THREADS / 64][MAXW + 2];
    const int row = blockIdx.x;
    const int b = row / D, d = row % D;
    const T* xr = x + b * x_bs + (int64_t)d * x_ds;
    const T* gr = dout + b * g_bs + (int64_t)d * g_ds;
    T* dxr = dx + b * dx_bs + (int64_t)d * dx_ds;
    float wk[W];
#pragma unroll
    for (int k = 0; k < W; ++k) wk[k] = w[d * W + k];
    const float bv = HAS_BIAS ? bias[d] : 0.f;
    float dw[W], db = 0.f, dmax = 0.f;
#pragma unroll
    for (int k = 0; k < W; ++k) dw[k] = 0.f;

    for (int t0 = 0; t0 < L; t0 += TILE) {
        __syncthreads();
        // sx[i] = x[t0 - (W-1) + i], i in [0, TILE + 2(W-1)) ; sg[i] = dpre[t0 + i], i in [0, TILE + W - 1)
        for (int i = threadIdx.x; i < TILE + 2 * (W - 1); i += THREADS) {
            const int t = t0 - (W - 1) + i;
            sx[i] = (t >= 0 && t < L) ? io<T>::ld(&xr[rev ? L - 1 - t : t]) : 0.f;
        }
        __syncthreads();
        for (int i = threadIdx.x; i < TILE + W - 1; i += THREADS) {
            const int t = t0 + i;
            float g = 0.f;
            if (t < L) {
                g = io<T>::ld(&gr[rev ? L - 1 - t : t]);
                if (SILU) {
                    float pre = bv;
#pragma unroll
                    for (int k = 0; k < W; ++k) pre += wk[k] * sx[i + k];
                    const float sgm = sigmoidf_(pre);
                    g *= sgm * (1.f + pre * (1.f - sgm));
                }
            }
            sg[i] = g;
        }
        __syncthreads();
#pragma unroll
        for (int p = 0; p < PER; ++p) {
            const int i = threadIdx.x + p * THREADS, t = t0 + i;
            if (t < L) {
                // dx[t] = sum_k w[k] * dpre[t + (W-1) - k]
                float acc = 0.f;
#pragma unroll
                for (int k = 0; k < W; ++k) acc += wk[k] * sg[i + (W - 1) - k];
                T* q = &dxr[rev ? L - 1 - t : t];
                const float v = dx_acc ? acc + io<T>::ld(q) : acc;
                io<T>::st(q, v);
                dmax = fmaxf(dmax, fabsf(v));
                const float g = sg[i];
                db += g;
#pragma unroll
                for (int k = 0; k < W; ++k) dw[k] += g * sx[i + k];
            }
        }
    }
    // block reduce dw, db (and the row's max |dx|)
#pragma unroll
    for (int k = 0; k <= W; ++k) {
        float v = (k < W) ? dw[k] : db;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
        if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6][k] = v;
    }
    if (dx_max) {
        const float m = wave_max(dmax);
        if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6][MAXW + 1] = m;
    }
    __syncthreads();
    if (threadIdx.x <= W) {
        float v = 0.f;
        for (int i = 0; i < THREADS / 64; ++i) v += sred[i][threadIdx.x];
        ws[(int64_t)row * (MAXW + 1) + threadIdx.x] = v;
    }
    if (dx_max && threadIdx.x == MAXW + 1) {
        float m = 0.f;
        for (int i = 0; i < THREADS / 64; ++i) m = fmaxf(m, sred[i][MAXW + 1]);
        ws[(int64_t)gridDim.x * (MAXW + 1) + row] = m;          // wsmax[row]
    }
}

// ---------------------------------------------------------------- vectorised rows (the Mamba layout)
// Rows with a 4-element-aligned stride (the product's 128-B aligned time stride): thread = 4 consecutive
// outputs, operands in registers.  The forward reads its own 4-vector and the neighbouring one (the (W-1)-sample
// halo: the neighbour's own vector, so an L1/L2 hit, not HBM); no LDS, no barriers, one vector load/store per
// 4 elements instead of the scalar LDS staging of fwd_kernel.  REV = the BiMamba backward direction: the conv
// runs in reversed time, i.e. over memory positions m with taps x[m .. m+W-1].
template <typename T> struct v4io;
template <> struct v4io<float> {
    __device__ static inline void ld(const float* p, float* v) {
        const float4 q = *reinterpret_cast<const float4*>(p);
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    }
    __device__ static inline void st(float* p, const float* v) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    }
};
template <> struct v4io<bf16_t> {
    __device__ static inline void ld(const bf16_t* p, float* v) {
        const uint2 q = *reinterpret_cast<const uint2*>(p);
        v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
        v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
    }
    __device__ static inline void st(bf16_t* p, const float* v) {
        bf16_t h[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) io<bf16_t>::st(&h[i], v[i]);
        *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)h[0].x | ((uint32_t)h[1].x << 16),
                                                  (uint32_t)h[2].x | ((uint32_t)h[3].x << 16));
    }
};

template <typename T>
__device__ inline void ld4z(const T* row, int t, int L, float* v) {   // x[t .. t+3], 0 outside [0, L)
    if (t >= 0 && t < L) {
        v4io<T>::ld(row + t, v);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (t + i >= L) v[i] = 0.f;
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = 0.f;
    }
}

template <typename T>
__device__ inline void st4(T* row, int t, int L, const float* v) {
    if (t + 3 < L) {
        v4io<T>::st(row + t, v);
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (t + i < L) io<T>::st(&row[t + i], v[i]);
    }
}

__device__ inline float silu_grad(float pre) {
    const float sgm = sigmoidf_(pre);
    return sgm * (1.f + pre * (1.f - sgm));
}

template <typename T, int W, bool SILU, bool HAS_BIAS, bool REV>
__global__ __launch_bounds__(THREADS) void fwd_vec_kernel(int D, int L, const T* __restrict__ x, int64_t x_bs,
                                                          int64_t x_ds, const float* __restrict__ w,
                                                          const float* __restrict__ bias, T* __restrict__ out,
                                                          int64_t o_bs, int64_t o_ds) {
    const int row = blockIdx.x;
    const int b = row / D, d = row % D;
    const T* xr = x + b * x_bs + (int64_t)d * x_ds;
    T* orow = out + b * o_bs + (int64_t)d * o_ds;
    float wk[W];
#pragma unroll
    for (int k = 0; k < W; ++k) wk[k] = w[d * W + k];
    const float bv = HAS_BIAS ? bias[d] : 0.f;
    for (int t = threadIdx.x * 4; t < L; t += THREADS * 4) {
        float e[8], o[4];
        if (!REV) {                               // e[i] = x[t - 4 + i]
            ld4z<T>(xr, t - 4, L, e);
            ld4z<T>(xr, t, L, e + 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float acc = bv;
#pragma unroll
                for (int k = 0; k < W; ++k) acc = fmaf(wk[k], e[4 + j - (W - 1) + k], acc);
                o[j] = SILU ? siluf_(acc) : acc;
            }
        } else {                                  // e[i] = x[t + i]
            ld4z<T>(xr, t, L, e);
            ld4z<T>(xr, t + 4, L, e + 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float acc = bv;
#pragma unroll
                for (int k = 0; k < W; ++k) acc = fmaf(wk[k], e[j + (W - 1) - k], acc);
                o[j] = SILU ? siluf_(acc) : acc;
            }
        }
        st4<T>(orow, t, L, o);
    }
}

template <typename T, int W, bool SILU, bool HAS_BIAS, bool REV>
__global__ __launch_bounds__(THREADS) void bwd_vec_kernel(int D, int L, const T* __restrict__ x, int64_t x_bs,
                                                          int64_t x_ds, const float* __restrict__ w,
                                                          const float* __restrict__ bias, const T* __restrict__ dout,
                                                          int64_t g_bs, int64_t g_ds, T* __restrict__ dx,
                                                          int64_t dx_bs, int64_t dx_ds, float* __restrict__ ws,
                                                          int dx_acc, uint32_t* __restrict__ dx_max) {
    __shared__ float sred[THREADS / 64][MAXW + 2];
    const int row = blockIdx.x;
    const int b = row / D, d = row % D;
    const T* xr = x + b * x_bs + (int64_t)d * x_ds;
    const T* gr = dout + b * g_bs + (int64_t)d * g_ds;
    T* dxr = dx + b * dx_bs + (int64_t)d * dx_ds;
    float wk[W];
#pragma unroll
    for (int k = 0; k < W; ++k) wk[k] = w[d * W + k];
    const float bv = HAS_BIAS ? bias[d] : 0.f;
    float dw[W], db = 0.f, dmax = 0.f;
#pragma unroll
    for (int k = 0; k < W; ++k) dw[k] = 0.f;
    for (int t = threadIdx.x * 4; t < L; t += THREADS * 4) {
        float xs[12], g[8], o[4];                 // xs[i] = x[t - 4 + i]
        ld4z<T>(xr, t - 4, L, xs);
        ld4z<T>(xr, t, L, xs + 4);
        ld4z<T>(xr, t + 4, L, xs + 8);
        // g[q] = dL/dpre at position p(q) (0 outside [0, L)): !REV p = t + q, REV p = t - 4 + q
        ld4z<T>(gr, REV ? t - 4 : t, L, g);
        ld4z<T>(gr, REV ? t : t + 4, L, g + 4);
        if (SILU) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                float pre = bv;
#pragma unroll
                for (int k = 0; k < W; ++k)
                    pre = fmaf(wk[k], REV ? xs[q + (W - 1) - k] : xs[q + 4 - (W - 1) + k], pre);
                g[q] *= silu_grad(pre);           // g is already 0 outside the row
            }
        }
        if (!REV) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float acc = 0.f;
#pragma unroll
                for (int k = 0; k < W; ++k) acc = fmaf(wk[k], g[j + (W - 1) - k], acc);
                o[j] = acc;
                db += g[j];
#pragma unroll
                for (int k = 0; k < W; ++k) dw[k] = fmaf(g[j], xs[j + 4 - (W - 1) + k], dw[k]);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float acc = 0.f;
#pragma unroll
                for (int k = 0; k < W; ++k) acc = fmaf(wk[k], g[j + 4 - (W - 1) + k], acc);
                o[j] = acc;
                db += g[4 + j];
#pragma unroll
                for (int k = 0; k < W; ++k) dw[k] = fmaf(g[4 + j], xs[4 + j + (W - 1) - k], dw[k]);
            }
        }
        if (dx_acc) {                             // the other BiMamba direction's dx, summed in place (round 6)
            float p[4];
            ld4z<T>(dxr, t, L, p);
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] += p[j];
        }
        st4<T>(dxr, t, L, o);
        if (dx_max) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (t + j < L) dmax = fmaxf(dmax, fabsf(o[j]));
        }
    }
#pragma unroll
    for (int k = 0; k <= W; ++k) {
        float v = (k < W) ? dw[k] : db;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
        if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6][k] = v;
    }
    if (dx_max) {
        const float m = wave_max(dmax);
        if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6][MAXW + 1] = m;
    }
    __syncthreads();
    if (threadIdx.x <= W) {
        float v = 0.f;
        for (int i = 0; i < THREADS / 64; ++i) v += sred[i][threadIdx.x];
        ws[(int64_t)row * (MAXW + 1) + threadIdx.x] = v;
    }
    if (dx_max && threadIdx.x == MAXW + 1) {
        float m = 0.f;
        for (int i = 0; i < THREADS / 64; ++i) m = fmaxf(m, sred[i][MAXW + 1]);
        ws[(int64_t)gridDim.x * (MAXW + 1) + row] = m;          // wsmax[row]
    }
}

// ---------------------------------------------------------------- short rows (L <= SHORT_L)
// DPMamba's chunked sequences (intra L = 250, inter L = 34) would leave a 2048-wide row tile almost
// empty: here each wave owns one row, held whole in a wave-private LDS line with its (W-1) halo; a
// workgroup is 4 independent rows.
constexpr int SHORT_L = 256;
constexpr int SPAD = SHORT_L + 2 * MAXW;

template <typename T, int W, bool SILU, bool HAS_BIAS>
__global__ __launch_bounds__(THREADS) void fwd_short_kernel(int rows, int D, int L, const T* __restrict__ x,
                                                            int64_t x_bs, int64_t x_ds, const float* __restrict__ w,
                                                            const float* __restrict__ bias, T* __restrict__ out,
                                                            int64_t o_bs, int64_t o_ds, int rev) {
    __shared__ float s[4][SPAD];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    if (row >= rows) return;                       // no workgroup barrier below: rows are wave-private
    const int b = row / D, d = row % D;
    const T* xr = x + b * x_bs + (int64_t)d * x_ds;
    T* orow = out + b * o_bs + (int64_t)d * o_ds;
    float* sw = s[wave];
    for (int i = lane; i < L + W - 1; i += 64) {   // sw[i] = x[i - (W-1)]
        const int t = i - (W - 1);
        sw[i] = t >= 0 ? io<T>::ld(&xr[rev ? L - 1 - t : t]) : 0.f;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float wk[W];
#pragma unroll
    for (int k = 0; k < W; ++k) wk[k] = w[d * W + k];
    const float bv = HAS_BIAS ? bias[d] : 0.f;
    for (int t = lane; t < L; t += 64) {
        float acc = bv;
#pragma unroll
        for (int k = 0; k < W; ++k) acc += wk[k] * sw[t + k];
        io<T>::st(&orow[rev ? L - 1 - t : t], SILU ? siluf_(acc) : acc);
    }
}

template <typename T, int W, bool SILU, bool HAS_BIAS>
__global__ __launch_bounds__(THREADS) void bwd_short_kernel(int rows, int D, int L, const T* __restrict__ x,
                                                            int64_t x_bs, int64_t x_ds, const float* __restrict__ w,
                                                            const float* __restrict__ bias,
                                                            const T* __restrict__ dout, int64_t g_bs, int64_t g_ds,
                                                            T* __restrict__ dx, int64_t dx_bs, int64_t dx_ds,
                                                            float* __restrict__ ws, int rev, int dx_acc,
                                                            uint32_t* __restrict__ dx_max) {
    __shared__ float sx[4][SPAD];
    __shared__ float sg[4][SPAD];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    if (row >= rows) return;
    const int b = row / D, d = row % D;
    const T* xr = x + b * x_bs + (int64_t)d * x_ds;
    const T* gr = dout + b * g_bs + (int64_t)d * g_ds;
    T* dxr = dx + b * dx_bs + (int64_t)d * dx_ds;
    float wk[W];
#pragma unroll
    for (int k = 0; k < W; ++k) wk[k] = w[d * W + k];
    const float bv = HAS_BIAS ? bias[d] : 0.f;
    float* px = sx[wave];
    float* pg = sg[wave];
    for (int i = lane; i < L + 2 * (W - 1); i += 64) {     // px[i] = x[i - (W-1)]
        const int t = i - (W - 1);
        px[i] = (t >= 0 && t < L) ? io<T>::ld(&xr[rev ? L - 1 - t : t]) : 0.f;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int i = lane; i < L + W - 1; i += 64) {           // pg[i] = dpre[i]
        float g = 0.f;
        if (i < L) {
            g = io<T>::ld(&gr[rev ? L - 1 - i : i]);
            if (SILU) {
                float pre = bv;
#pragma unroll
                for (int k = 0; k < W; ++k) pre += wk[k] * px[i + k];
                const float sgm = sigmoidf_(pre);
                g *= sgm * (1.f + pre * (1.f - sgm));
            }
        }
        pg[i] = g;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float dw[W], db = 0.f, dmax = 0.f;
#pragma unroll
    for (int k = 0; k < W; ++k) dw[k] = 0.f;
    for (int t = lane; t < L; t += 64) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < W; ++k) acc += wk[k] * pg[t + (W - 1) - k];
        T* q = &dxr[rev ? L - 1 - t : t];
        const float v = dx_acc ? acc + io<T>::ld(q) : acc;
        io<T>::st(q, v);
        dmax = fmaxf(dmax, fabsf(v));
        const float g = pg[t];
        db += g;
#pragma unroll
        for (int k = 0; k < W; ++k) dw[k] += g * px[t + k];
    }
#pragma unroll
    for (int k = 0; k <= W; ++k) {
        float v = (k < W) ? dw[k] : db;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
        if (lane == 0) ws[(int64_t)row * (MAXW + 1) + k] = v;
    }
    if (dx_max) {
        const float m = wave_max(dmax);
        if (lane == 0) ws[(int64_t)rows * (MAXW + 1) + row] = m;   // wsmax[row]
    }
}

// dweight / dbias: per-row partials summed over the batch, one workgroup per channel (deterministic:
// fixed per-thread strides, then a fixed tree)
// max over the rows' wsmax entries -> *out (atomic max: the scan's dz max may share the word)
__global__ __launch_bounds__(1024) void rowmax_kernel(const float* __restrict__ wsmax, int rows, uint32_t* out) {
    __shared__ float red[16];
    float m = 0.f;
    for (int i = threadIdx.x; i < rows; i += 1024) m = fmaxf(m, wsmax[i]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 16; ++i) m = fmaxf(m, red[i]);
        atomicMax(out, __float_as_uint(m));
    }
}

__global__ __launch_bounds__(THREADS) void reduce_kernel(const float* ws, int batch, int D, int W, float* dw, float* db) {
    __shared__ float red[THREADS / 64][MAXW + 1];
    const int d = blockIdx.x;
    float v[MAXW + 1];
#pragma unroll
    for (int k = 0; k <= MAXW; ++k) v[k] = 0.f;
    for (int b = threadIdx.x; b < batch; b += THREADS) {
        const float* p = ws + ((int64_t)b * D + d) * (MAXW + 1);
#pragma unroll
        for (int k = 0; k <= MAXW; ++k) v[k] += p[k];
    }
#pragma unroll
    for (int k = 0; k <= MAXW; ++k) {
        float t = v[k];
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) t += __shfl_xor(t, m, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][k] = t;
    }
    __syncthreads();
    if (threadIdx.x <= W) {
        const int k = threadIdx.x;
        const float t = red[0][k] + red[1][k] + red[2][k] + red[3][k];
        if (k < W) dw[d * W + k] = t;
        else if (db) db[d] = t;
    }
}

}  // namespace cconv
}  // namespace avse

using namespace avse::cconv;
using avse::bf16_t;

namespace {

// vectorised-row eligibility: 4-element aligned rows and batch steps, and (for tensors read as 4-vectors) a
// row stride that covers the last vector (x_ds >= round_up(L, 4), e.g. the 128-B padded time stride)
template <typename T>
bool vec_rows(const T* p, int64_t bs, int64_t ds, int64_t L, bool read) {
    return ((uintptr_t)p % (4 * sizeof(T))) == 0 && bs % 4 == 0 && ds % 4 == 0 && ds > 0 &&
           (!read || ds >= (L + 3) / 4 * 4);
}

template <typename T, int W, bool S, bool HB>
void launch_fwd(int64_t batch, int64_t dim, int64_t seqlen, const T* x, int64_t x_bs, int64_t x_ds, const float* w,
                const float* bias, T* out, int64_t o_bs, int64_t o_ds, int rev, hipStream_t st) {
    const int rows = (int)(batch * dim);
    if (seqlen <= SHORT_L)
        hipLaunchKernelGGL((fwd_short_kernel<T, W, S, HB>), dim3((unsigned)((rows + 3) / 4)), dim3(THREADS), 0, st,
                           rows, (int)dim, (int)seqlen, x, x_bs, x_ds, w, bias, out, o_bs, o_ds, rev);
    else if (vec_rows<T>(x, x_bs, x_ds, seqlen, true) && vec_rows<T>(out, o_bs, o_ds, seqlen, false)) {
        if (rev)
            hipLaunchKernelGGL((fwd_vec_kernel<T, W, S, HB, true>), dim3((unsigned)rows), dim3(THREADS), 0, st,
                               (int)dim, (int)seqlen, x, x_bs, x_ds, w, bias, out, o_bs, o_ds);
        else
            hipLaunchKernelGGL((fwd_vec_kernel<T, W, S, HB, false>), dim3((unsigned)rows), dim3(THREADS), 0, st,
                               (int)dim, (int)seqlen, x, x_bs, x_ds, w, bias, out, o_bs, o_ds);
    } else
        hipLaunchKernelGGL((fwd_kernel<T, W, S, HB>), dim3((unsigned)rows), dim3(THREADS), 0, st, (int)dim,
                           (int)seqlen, x, x_bs, x_ds, w, bias, out, o_bs, o_ds, rev);
}

template <typename T, int W, bool S, bool HB>
void launch_bwd(int64_t batch, int64_t dim, int64_t seqlen, const T* x, int64_t x_bs, int64_t x_ds, const float* w,
                const float* bias, const T* dout, int64_t g_bs, int64_t g_ds, T* dx, int64_t dx_bs, int64_t dx_ds,
                float* ws, int rev, int dx_acc, uint32_t* dx_max, hipStream_t st) {
    const int rows = (int)(batch * dim);
    if (seqlen <= SHORT_L)
        hipLaunchKernelGGL((bwd_short_kernel<T, W, S, HB>), dim3((unsigned)((rows + 3) / 4)), dim3(THREADS), 0, st,
                           rows, (int)dim, (int)seqlen, x, x_bs, x_ds, w, bias, dout, g_bs, g_ds, dx, dx_bs, dx_ds, ws,
                           rev, dx_acc, dx_max);
    else if (vec_rows<T>(x, x_bs, x_ds, seqlen, true) && vec_rows<T>(dout, g_bs, g_ds, seqlen, true) &&
             vec_rows<T>(dx, dx_bs, dx_ds, seqlen, false)) {
        if (rev)
            hipLaunchKernelGGL((bwd_vec_kernel<T, W, S, HB, true>), dim3((unsigned)rows), dim3(THREADS), 0, st,
                               (int)dim, (int)seqlen, x, x_bs, x_ds, w, bias, dout, g_bs, g_ds, dx, dx_bs, dx_ds, ws,
                               dx_acc, dx_max);
        else
            hipLaunchKernelGGL((bwd_vec_kernel<T, W, S, HB, false>), dim3((unsigned)rows), dim3(THREADS), 0, st,
                               (int)dim, (int)seqlen, x, x_bs, x_ds, w, bias, dout, g_bs, g_ds, dx, dx_bs, dx_ds, ws,
                               dx_acc, dx_max);
    } else
        hipLaunchKernelGGL((bwd_kernel<T, W, S, HB>), dim3((unsigned)rows), dim3(THREADS), 0, st, (int)dim,
                           (int)seqlen, x, x_bs, x_ds, w, bias, dout, g_bs, g_ds, dx, dx_bs, dx_ds, ws, rev, dx_acc,
                           dx_max);
}

// width / silu / bias -> template instance
template <template <typename, int, bool, bool> class F, typename T, typename... Args>
int dispatch(int64_t width, bool silu, bool has_bias, Args... args) {
#define AVSE_CC(WW)                                                                          \
    case WW:                                                                                 \
        if (silu) {                                                                          \
            if (has_bias) F<T, WW, true, true>::run(args...);                                \
            else F<T, WW, true, false>::run(args...);                                        \
        } else {                                                                             \
            if (has_bias) F<T, WW, false, true>::run(args...);                               \
            else F<T, WW, false, false>::run(args...);                                       \
        }                                                                                    \
        return AVSE_OK;
    switch ((int)width) {
        AVSE_CC(1) AVSE_CC(2) AVSE_CC(3) AVSE_CC(4)
        default: return AVSE_ESHAPE;
    }
#undef AVSE_CC
}

template <typename T, int W, bool S, bool HB>
struct Fwd {
    template <typename... A> static void run(A... a) { launch_fwd<T, W, S, HB>(a...); }
};
template <typename T, int W, bool S, bool HB>
struct Bwd {
    template <typename... A> static void run(A... a) { launch_bwd<T, W, S, HB>(a...); }
};

template <typename T>
int cconv_fwd(int64_t batch, int64_t dim, int64_t seqlen, int64_t width, const T* x, int64_t x_bs, int64_t x_ds,
              const float* weight, const float* bias, T* out, int64_t out_bs, int64_t out_ds, int32_t silu,
              int32_t reverse, avse_stream_t stream) {
    if (!x || !weight || !out) return AVSE_EINVAL;
    if (batch <= 0 || dim <= 0 || seqlen <= 0 || width < 1 || width > MAXW) return AVSE_ESHAPE;
    if (batch * dim > (1LL << 31) - 1) return AVSE_ESHAPE;
    const int rc = dispatch<Fwd, T>(width, silu != 0, bias != nullptr, batch, dim, seqlen, x, x_bs, x_ds, weight, bias,
                                    out, out_bs, out_ds, (int)reverse, (hipStream_t)stream);
    if (rc != AVSE_OK) return rc;
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

template <typename T>
int cconv_bwd(int64_t batch, int64_t dim, int64_t seqlen, int64_t width, const T* x, int64_t x_bs, int64_t x_ds,
              const float* weight, const float* bias, const T* dout, int64_t dout_bs, int64_t dout_ds, T* dx,
              int64_t dx_bs, int64_t dx_ds, float* dweight, float* dbias, int32_t silu, int32_t reverse,
              float* workspace, int32_t dx_accumulate, uint32_t* dx_max, avse_stream_t stream) {
    if (!x || !weight || !dout || !dx || !dweight || !workspace) return AVSE_EINVAL;
    if (bias && !dbias) return AVSE_EINVAL;
    if (batch <= 0 || dim <= 0 || seqlen <= 0 || width < 1 || width > MAXW) return AVSE_ESHAPE;
    if (batch * dim > (1LL << 31) - 1) return AVSE_ESHAPE;
    hipStream_t st = (hipStream_t)stream;
    const int rc = dispatch<Bwd, T>(width, silu != 0, bias != nullptr, batch, dim, seqlen, x, x_bs, x_ds, weight, bias,
                                    dout, dout_bs, dout_ds, dx, dx_bs, dx_ds, workspace, (int)reverse,
                                    (int)(dx_accumulate != 0), dx_max, st);
    if (rc != AVSE_OK) return rc;
    AVSE_CHECK_LAUNCH();
    if (dx_max) {
        const int rows = (int)(batch * dim);
        hipLaunchKernelGGL(rowmax_kernel, dim3(1), dim3(1024), 0, st, workspace + (int64_t)rows * (MAXW + 1), rows,
                           dx_max);
        AVSE_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL(reduce_kernel, dim3((unsigned)dim), dim3(THREADS), 0, st, workspace, (int)batch, (int)dim,
                       (int)width, dweight, dbias);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // namespace

extern "C" {

int64_t avse_cconv_bwd_workspace_bytes(int64_t batch, int64_t dim, int64_t width) {
    (void)width;
    return 4 * batch * dim * (MAXW + 2);         // per row: dw / db partials, then (after all rows) max |dx|
}

int avse_cconv_fwd(int64_t batch, int64_t dim, int64_t seqlen, int64_t width, const float* x, int64_t x_bs,
                   int64_t x_ds, const float* weight, const float* bias, float* out, int64_t out_bs, int64_t out_ds,
                   int32_t silu, int32_t reverse, avse_stream_t stream) {
    return cconv_fwd<float>(batch, dim, seqlen, width, x, x_bs, x_ds, weight, bias, out, out_bs, out_ds, silu,
                            reverse, stream);
}

int avse_cconv_bwd(int64_t batch, int64_t dim, int64_t seqlen, int64_t width, const float* x, int64_t x_bs,
                   int64_t x_ds, const float* weight, const float* bias, const float* dout, int64_t dout_bs,
                   int64_t dout_ds, float* dx, int64_t dx_bs, int64_t dx_ds, float* dweight, float* dbias,
                   int32_t silu, int32_t reverse, float* workspace, int32_t dx_accumulate, uint32_t* dx_max,
                   avse_stream_t stream) {
    return cconv_bwd<float>(batch, dim, seqlen, width, x, x_bs, x_ds, weight, bias, dout, dout_bs, dout_ds, dx, dx_bs,
                            dx_ds, dweight, dbias, silu, reverse, workspace, dx_accumulate, dx_max, stream);
}

int avse_cconv_fwd_bf16(int64_t batch, int64_t dim, int64_t seqlen, int64_t width, const uint16_t* x, int64_t x_bs,
                        int64_t x_ds, const float* weight, const float* bias, uint16_t* out, int64_t out_bs,
                        int64_t out_ds, int32_t silu, int32_t reverse, avse_stream_t stream) {
    return cconv_fwd<bf16_t>(batch, dim, seqlen, width, (const bf16_t*)x, x_bs, x_ds, weight, bias, (bf16_t*)out,
                             out_bs, out_ds, silu, reverse, stream);
}

int avse_cconv_bwd_bf16(int64_t batch, int64_t dim, int64_t seqlen, int64_t width, const uint16_t* x, int64_t x_bs,
                        int64_t x_ds, const float* weight, const float* bias, const uint16_t* dout, int64_t dout_bs,
                        int64_t dout_ds, uint16_t* dx, int64_t dx_bs, int64_t dx_ds, float* dweight, float* dbias,
                        int32_t silu, int32_t reverse, float* workspace, int32_t dx_accumulate, uint32_t* dx_max,
                        avse_stream_t stream) {
    return cconv_bwd<bf16_t>(batch, dim, seqlen, width, (const bf16_t*)x, x_bs, x_ds, weight, bias,
                             (const bf16_t*)dout, dout_bs, dout_ds, (bf16_t*)dx, dx_bs, dx_ds, dweight, dbias, silu,
                             reverse, workspace, dx_accumulate, dx_max, stream);
}

}  // extern "C"
