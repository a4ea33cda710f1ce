// Fused PReLU -> GlobalLayerNorm forward / backward for gfx950 (avse4 TCN hot path).
//
// Replaces the (nn.PReLU(), GlobalLayerNorm) pairs of /root/reference/baseline/avse4/model.py:
//   TemporalBlock.net          :259-266  conv1x1 -> PReLU -> gLN -> ...
//   DepthwiseSeparableConv.net :284-292  dwconv  -> PReLU -> gLN -> conv1x1
// gLN (model.py:225-252): per sample mean/var over (C, K), EPS 1e-8 inside pow(var + EPS, .5),
// biased variance; y = gamma_c (p - mean) / sqrt(var + EPS) + beta_c with p = PReLU(x) (one slope).
//
// Layout (B, C, K), K contiguous.  Every kernel is one pass over rows (b, c) with one 256-thread
// workgroup per row (lane-contiguous loads); per-row partial sums go to small workspaces that tiny
// finalize kernels reduce (deterministic, double accumulation across rows).  Statistics use sums
// shifted by the sample's first element, which removes the E[x^2]-E[x]^2 cancellation.
// HBM: fwd = 2 reads + 1 write of x, bwd = 2 reads of (x, dy) + 1 write of dx.
#include "common.h"

namespace avse {
namespace gln {

constexpr int THREADS = 256;
constexpr int DW_U = 8, DW_UB = 4;          // elements per thread in flight (forward, backward passes)

__device__ inline float prelu(float x, float a) { return x > 0.f ? x : a * x; }

// 4 consecutive fp32 per thread: dwordx4 buffer loads (rows need only dword alignment; outside the row's range: 0)
typedef unsigned int u4_t __attribute__((ext_vector_type(4)));
__device__ inline float4 ld4(__amdgpu_buffer_rsrc_t r, int voff_elems) {
    const u4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, voff_elems * 4, 0, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ inline float f4at(const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }
// a row's quadruple t..t+3: one dwordx4 store, the row's last partial quadruple element by element
__device__ inline void st4_row(__amdgpu_buffer_rsrc_t r, float* row, int t, int K, const float (&v)[4]) {
    if (t + 4 <= K) {
        const u4_t o = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
        __builtin_amdgcn_raw_buffer_store_b128(o, r, t * 4, 0, 0);
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (t + e < K) row[t + e] = v[e];
    }
}
constexpr int V4 = 4, UB4 = 2;                  // elements per thread per access, accesses in flight (1 / 4: +-2 %)

template <typename T>
__device__ inline T block_sum(T v, T* red) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

// row partials of shifted sums: ws[row] = (sum(p - s), sum((p - s)^2)), s = p(x[b, 0, 0]); rows row0 + blockIdx.x
__global__ __launch_bounds__(THREADS) void stats_kernel(int row0, int C, int K, const float* __restrict__ x,
                                                        const float* __restrict__ alpha, float2* __restrict__ ws) {
    __shared__ float red[4];
    const int row = row0 + (int)blockIdx.x, b = row / C;
    const float a = alpha[0];
    const float shift = prelu(x[(int64_t)b * C * K], a);
    const auto rx = make_rsrc(x + (int64_t)row * K, K);
    float s1 = 0.f, s2 = 0.f;
    for (int t0 = 0; t0 < K; t0 += UB4 * V4 * THREADS) {
        float4 xv[UB4];
#pragma unroll
        for (int j = 0; j < UB4; ++j) xv[j] = ld4(rx, t0 + (j * THREADS + (int)threadIdx.x) * V4);
#pragma unroll
        for (int j = 0; j < UB4; ++j) {
            const int t = t0 + (j * THREADS + (int)threadIdx.x) * V4;
#pragma unroll
            for (int e = 0; e < V4; ++e) {
                const float v = (t + e < K) ? prelu(f4at(xv[j], e), a) - shift : 0.f;
                s1 += v;
                s2 += v * v;
            }
        }
    }
    s1 = block_sum(s1, red);
    s2 = block_sum(s2, red);
    if (threadIdx.x == 0) ws[row] = make_float2(s1, s2);
}

template <typename T>
__device__ inline T block_sum_max(T v, T* red) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// sample b's (sum_c v.x, sum_c v.y) over its C row partials, in double, by a 256-thread block (fixed order:
// every caller gets the same bits)
__device__ inline double2 sample_sums(const float2* __restrict__ ws, int b, int C, double* red /* [8] */,
                                      const float* __restrict__ wgt = nullptr) {
    double s1 = 0.0, s2 = 0.0;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        const float2 v = ws[(int64_t)b * C + c];
        const double g = wgt ? (double)wgt[c] : 1.0;
        s1 += g * v.x;
        s2 += g * v.y;
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        s1 += __shfl_xor(s1, m, 64);
        s2 += __shfl_xor(s2, m, 64);
    }
    __syncthreads();                                   // red may still be read by a previous call
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = s1;
        red[4 + (threadIdx.x >> 6)] = s2;
    }
    __syncthreads();
    return make_double2((red[0] + red[1]) + (red[2] + red[3]), (red[4] + red[5]) + (red[6] + red[7]));
}

// mean, rstd = 1 / sqrt(var + EPS) of sample b from its shifted row sums
__device__ inline float2 sample_stats(double2 sums, int C, int K, float shift, float eps) {
    const double n = (double)C * K;
    const double m1 = sums.x / n, m2 = sums.y / n;
    const double var = fmax(m2 - m1 * m1, 0.0);
    return make_float2((float)(m1 + shift), (float)(1.0 / sqrt(var + (double)eps)));
}

// The backward's second pass walks the rows in reverse: its first rows are the ones the reduction pass read last,
// still in the Infinity Cache / L2 when it starts ((y1, dy) of C4 is 262 MB against the 256 MB memory-side cache):
// C4 dwconv_gln_bwd 0.193 -> 0.186 ms.  The forward's apply pass keeps the launch order (reversed it measured
// 0.0965 -> 0.101 ms).
__device__ inline int second_pass_row() { return gridDim.x - 1 - blockIdx.x; }

// power-of-two scale of the split planes from the bits of an upper bound of max |y| (the projection GEMM's split_exp:
// bound 2^e in [2^14, 2^15); values up to twice the bound still fit fp16)
__device__ inline int split_exp_gln(uint32_t mb) {
    const int ef = (int)((mb >> 23) & 0xff);
    if (mb == 0) return 0;
    const int k = ef == 0 ? -127 : ef - 127;
    return min(100, max(-100, 14 - k));
}

// Q output: the apply's y as the split-fp16 planes of the 1x1 Conv1d GEMM that consumes it (csrc/projgemm.hip
// avse_gemm_f32s): hi = fp16(y 2^e), lo = fp16(y 2^e - hi) in rows of kp (a multiple of 8) elements; the padding
// columns K .. kp - 1 are written as 0 (a weight-gradient GEMM over time chunks sums over them)
struct QOut {
    const uint32_t* maxbits;
    _Float16* hi;
    _Float16* lo;
    int kp;
};

// the row's quadruple t .. t + 3 (t < K) into the planes, elements past K as 0
__device__ inline void q_store_quad(const QOut& q, int row, int t, int K, const float (&o4)[4], float sc) {
    uint32_t h[2], l[2];
#pragma unroll
    for (int e2 = 0; e2 < 2; ++e2) {
        const float s0 = t + 2 * e2 < K ? o4[2 * e2] * sc : 0.f;
        const float s1 = t + 2 * e2 + 1 < K ? o4[2 * e2 + 1] * sc : 0.f;
        const _Float16 h0 = (_Float16)s0, h1 = (_Float16)s1;
        const _Float16 l0 = (_Float16)(s0 - (float)h0), l1 = (_Float16)(s1 - (float)h1);
        h[e2] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
        l[e2] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
    }
    const int64_t off = (int64_t)row * q.kp + t;
    *reinterpret_cast<uint2*>(q.hi + off) = uint2{h[0], h[1]};
    *reinterpret_cast<uint2*>(q.lo + off) = uint2{l[0], l[1]};
}
// the row's padding columns past its last quadruple: 0
__device__ inline void q_zero_pad(const QOut& q, int row, int K) {
    for (int t = (K + 3) / 4 * 4 + 4 * (int)threadIdx.x; t < q.kp; t += 4 * THREADS) {
        const int64_t off = (int64_t)row * q.kp + t;
        *reinterpret_cast<uint2*>(q.hi + off) = uint2{0u, 0u};
        *reinterpret_cast<uint2*>(q.lo + off) = uint2{0u, 0u};
    }
}

// apply with the finalize folded in: every row block re-derives its sample's statistics from the row partials (the
// same sums in the same order in every block: bitwise equal), the channel-0 block stores them for the backward.
// shift_src: the tensor whose (b, 0, 0) element defines the shift (y1 here)
template <bool QO = false>
__global__ __launch_bounds__(THREADS) void apply_fused_kernel(int row0, int C, int K, const float* __restrict__ x,
                                                              const float* __restrict__ alpha,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta,
                                                              const float2* __restrict__ ws, float eps,
                                                              float2* __restrict__ stats, float* __restrict__ y,
                                                              QOut q = QOut{}) {
    __shared__ double red[8];
    const int row = row0 + (int)blockIdx.x, b = row / C, c = row % C;
    const float a = alpha[0];
    const float2 st = sample_stats(sample_sums(ws, b, C, red), C, K, prelu(x[(int64_t)b * C * K], a), eps);
    if (c == 0 && threadIdx.x == 0) stats[b] = st;
    const float g = gamma[c] * st.y, o = beta[c] - gamma[c] * st.y * st.x;
    const float* xr = x + (int64_t)row * K;
    float* yr = QO ? nullptr : y + (int64_t)row * K;
    const auto rx = make_rsrc(xr, K), ry = make_rsrc(QO ? xr : yr, K);
    float sc = 1.f;
    if constexpr (QO) sc = __builtin_ldexpf(1.f, split_exp_gln(*q.maxbits));
    for (int t0 = 0; t0 < K; t0 += UB4 * V4 * THREADS) {
        float4 xv[UB4];
#pragma unroll
        for (int jj = 0; jj < UB4; ++jj) xv[jj] = ld4(rx, t0 + (jj * THREADS + (int)threadIdx.x) * V4);
#pragma unroll
        for (int jj = 0; jj < UB4; ++jj) {
            const int t = t0 + (jj * THREADS + (int)threadIdx.x) * V4;
            float o4[4];
#pragma unroll
            for (int e = 0; e < V4; ++e) o4[e] = g * prelu(f4at(xv[jj], e), a) + o;
            if constexpr (QO) {
                if (t < K) q_store_quad(q, row, t, K, o4, sc);
            } else {
                st4_row(ry, yr, t, K, o4);
            }
        }
    }
    if constexpr (QO) q_zero_pad(q, row, K);
}

// An upper bound of max |y| for the split planes, before any apply block writes: per row, y = g p + o is affine in
// p = PReLU(.), so max |y| over the row is max(|g pmin + o|, |g pmax + o|) from the row's PReLU extremes (mm, written
// by the statistics pass).  One block per sample re-derives its statistics as the apply does and max-reduces its rows.
__global__ __launch_bounds__(256) void q_bound_kernel(int C, int K, const float* __restrict__ x,
                                                      const float* __restrict__ alpha, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, const float2* __restrict__ ws,
                                                      const float2* __restrict__ mm, float eps,
                                                      uint32_t* __restrict__ maxbits) {
    __shared__ double red[8];
    __shared__ float fred[4];
    const int b = blockIdx.x;
    const float a = alpha[0];
    const float2 st = sample_stats(sample_sums(ws, b, C, red), C, K, prelu(x[(int64_t)b * C * K], a), eps);
    float m = 0.f;
    for (int c = threadIdx.x; c < C; c += 256) {
        const float g = gamma[c] * st.y, o = beta[c] - gamma[c] * st.y * st.x;
        const float2 e = mm[(int64_t)b * C + c];
        m = fmaxf(m, fmaxf(fabsf(g * e.x + o), fabsf(g * e.y + o)));
    }
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) fred[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        // a few ulps of headroom over the apply's own rounding of g p + o (the scale only needs an upper bound)
        const uint32_t v = __float_as_uint(fmaxf(fmaxf(fred[0], fred[1]), fmaxf(fred[2], fred[3])) * 1.0001f);
        if (v) atomicMax(maxbits, v);
    }
}


// backward pass 1: per row S1 = sum dy, S2 = sum dy * xhat.  4 consecutive elements per thread (dwordx4 loads, rows
// need only dword alignment; the row's last partial quadruple is masked per element), 2 quadruples in flight
template <bool MM = false>
__global__ __launch_bounds__(THREADS) void bwd_reduce_kernel(int row0, int C, int K, const float* __restrict__ x,
                                                             const float* __restrict__ alpha, const float2* __restrict__ stats,
                                                             const float* __restrict__ dy, float2* __restrict__ ws,
                                                             float2* __restrict__ mm = nullptr) {
    constexpr int V = 4, UB = 2;                  // 1 / 4 in flight: within +-2 % (tools/gln_ub_ab.sh @ 8f1eec2)
    __shared__ float red[4];
    const int row = row0 + (int)blockIdx.x, b = row / C;
    const float a = alpha[0];
    const float2 st = stats[b];
    const auto rx = make_rsrc(x + (int64_t)row * K, K), rg = make_rsrc(dy + (int64_t)row * K, K);
    float s1 = 0.f, s2 = 0.f;
    float gmax = 0.f, xhmax = 0.f;                       // MM: the row's max |dy|, max |xhat| (the dx planes' bound)
    for (int t0 = 0; t0 < K; t0 += UB * V * THREADS) {
        float4 gv[UB], xv[UB];
#pragma unroll
        for (int j = 0; j < UB; ++j) {
            const int t = t0 + (j * THREADS + (int)threadIdx.x) * V;
            gv[j] = ld4(rg, t);
            xv[j] = ld4(rx, t);
        }
#pragma unroll
        for (int j = 0; j < UB; ++j) {
            const int t = t0 + (j * THREADS + (int)threadIdx.x) * V;
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const float g = (t + e < K) ? f4at(gv[j], e) : 0.f;
                const float xh = (prelu(f4at(xv[j], e), a) - st.x) * st.y;
                s1 += g;
                s2 += g * xh;
                if constexpr (MM) {
                    gmax = fmaxf(gmax, fabsf(g));
                    xhmax = (t + e < K) ? fmaxf(xhmax, fabsf(xh)) : xhmax;
                }
            }
        }
    }
    s1 = block_sum(s1, red);
    s2 = block_sum(s2, red);
    if (threadIdx.x == 0) ws[row] = make_float2(s1, s2);
    if constexpr (MM) {
        gmax = block_sum_max(gmax, red);
        xhmax = block_sum_max(xhmax, red);
        if (threadIdx.x == 0) mm[row] = make_float2(gmax, xhmax);
    }
}

// An upper bound of max |dx| of the PReLU -> gLN backward before its apply pass writes the planes: per row
// |dx| <= max(1, |a|) rstd (|gamma_c| max|dy| + |mean_g| + max|xhat| |mean_gxh|) from the reduction's row maxima (mm).
// One block per sample re-derives (mean_g, mean_gxh) as the apply pass does.
__global__ __launch_bounds__(256) void q_bwd_bound_kernel(int C, int K, const float* __restrict__ alpha,
                                                          const float* __restrict__ gamma,
                                                          const float2* __restrict__ stats,
                                                          const float2* __restrict__ ws_rows,
                                                          const float2* __restrict__ mm, uint32_t* __restrict__ maxbits) {
    __shared__ double dred[8];
    __shared__ float fred[4];
    const int b = blockIdx.x;
    const float a = alpha[0];
    const float2 st = stats[b];
    const double2 sg12 = sample_sums(ws_rows, b, C, dred, gamma);
    const double nn = (double)C * K;
    const float smx = fabsf((float)(sg12.x / nn)), smy = fabsf((float)(sg12.y / nn));
    const float sl = fmaxf(1.f, fabsf(a)) * st.y;
    float m = 0.f;
    for (int c = threadIdx.x; c < C; c += 256) {
        const float2 e = mm[(int64_t)b * C + c];
        m = fmaxf(m, sl * (fabsf(gamma[c]) * e.x + smx + e.y * smy));
    }
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) fred[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t v = __float_as_uint(fmaxf(fmaxf(fred[0], fred[1]), fmaxf(fred[2], fred[3])) * 1.001f);
        if (v) atomicMax(maxbits, v);
    }
}

// per sample: (mean_g, mean_gxh) over (C, K) with g = dy * gamma; per channel dgamma, dbeta (sum over b)
__global__ void bwd_finalize(int B, int C, int K, const float2* __restrict__ ws, const float* __restrict__ gamma,
                             float2* __restrict__ smeans, float* __restrict__ dgamma, float* __restrict__ dbeta) {
    __shared__ double red1[4], red2[4];
    const int blk = blockIdx.x;
    if (blk < B) {
        const int b = blk;
        double s1 = 0.0, s2 = 0.0;
        for (int c = threadIdx.x; c < C; c += blockDim.x) {
            const float2 v = ws[(int64_t)b * C + c];
            s1 += (double)gamma[c] * v.x;
            s2 += (double)gamma[c] * v.y;
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            s1 += __shfl_xor(s1, m, 64);
            s2 += __shfl_xor(s2, m, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            red1[threadIdx.x >> 6] = s1;
            red2[threadIdx.x >> 6] = s2;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            const double n = (double)C * K;
            smeans[b] = make_float2((float)((red1[0] + red1[1] + red1[2] + red1[3]) / n),
                                    (float)((red2[0] + red2[1] + red2[2] + red2[3]) / n));
        }
    } else {
        const int c0 = (blk - B) * blockDim.x;
        const int c = c0 + threadIdx.x;
        if (c < C) {
            double g = 0.0, bt = 0.0;
            for (int b = 0; b < B; ++b) {
                const float2 v = ws[(int64_t)b * C + c];
                bt += v.x;
                g += v.y;
            }
            dgamma[c] = (float)g;
            dbeta[c] = (float)bt;
        }
    }
}

// backward pass 2: dx = (x > 0 ? 1 : a) * rstd * (dy*gamma - mean_g - xhat*mean_gxh); dalpha row partial.  The
// sample's (mean_g, mean_gxh) re-derived per row block from the row partials (as dwconv_gln_bwd does), so a sample
// group needs no finalize launch between its two passes
template <bool QO = false>
__global__ __launch_bounds__(THREADS) void bwd_apply_kernel(int row0, int C, int K, const float* __restrict__ x,
                                                            const float* __restrict__ alpha, const float* __restrict__ gamma,
                                                            const float2* __restrict__ stats,
                                                            const float2* __restrict__ ws_rows,
                                                            const float* __restrict__ dy, float* __restrict__ dx,
                                                            float* __restrict__ ws_alpha, QOut q = QOut{}) {
    __shared__ float red[4];
    __shared__ double dred[8];
    const int row = row0 + second_pass_row(), b = row / C, c = row % C;
    const float a = alpha[0];
    const float2 st = stats[b];
    const double2 sg12 = sample_sums(ws_rows, b, C, dred, gamma);
    const double nn = (double)C * K;
    const float2 sm = make_float2((float)(sg12.x / nn), (float)(sg12.y / nn));
    const float gm = gamma[c];
    const float* xr = x + (int64_t)row * K;
    const float* gr = dy + (int64_t)row * K;
    float* dr = QO ? nullptr : dx + (int64_t)row * K;
    const auto rx = make_rsrc(xr, K), rg = make_rsrc(gr, K), rd = make_rsrc(QO ? gr : dr, K);
    float sc = 1.f;
    if constexpr (QO) sc = __builtin_ldexpf(1.f, split_exp_gln(*q.maxbits));
    float da = 0.f;
    for (int t0 = 0; t0 < K; t0 += UB4 * V4 * THREADS) {
        float4 xv[UB4], gv[UB4];
#pragma unroll
        for (int j = 0; j < UB4; ++j) {
            const int t = t0 + (j * THREADS + (int)threadIdx.x) * V4;
            xv[j] = ld4(rx, t);
            gv[j] = ld4(rg, t);
        }
#pragma unroll
        for (int j = 0; j < UB4; ++j) {
            const int t = t0 + (j * THREADS + (int)threadIdx.x) * V4;
            float o4[4];
#pragma unroll
            for (int e = 0; e < V4; ++e) {
                const float xvv = f4at(xv[j], e);
                const float xh = (prelu(xvv, a) - st.x) * st.y;
                const float dp = st.y * (f4at(gv[j], e) * gm - sm.x - xh * sm.y);
                o4[e] = xvv > 0.f ? dp : a * dp;
                da += (xvv > 0.f || t + e >= K) ? 0.f : dp * xvv;
            }
            if constexpr (QO) {
                if (t < K) q_store_quad(q, row, t, K, o4, sc);
            } else {
                st4_row(rd, dr, t, K, o4);
            }
        }
    }
    if constexpr (QO) q_zero_pad(q, row, K);
    da = block_sum(da, red);
    if (threadIdx.x == 0) ws_alpha[row] = da;
}

__global__ void alpha_finalize(int rows, const float* __restrict__ ws_alpha, float* __restrict__ dalpha) {
    __shared__ double red[4];
    double s = 0.0;
    for (int i = threadIdx.x; i < rows; i += blockDim.x) s += ws_alpha[i];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) dalpha[0] = (float)(red[0] + red[1] + red[2] + red[3]);
}

// ----------------------------------------------------------------------------------------------------------
// Fused depthwise dilated conv1d <-> PReLU -> gLN (DepthwiseSeparableConv.net[:3], model.py:278-292)
//   fwd: ONE pass computes y1 = dwconv(x) per row (streaming: the taps' neighbours come from the cache lines the
//        row's workgroup just loaded) and, from the registers, the row's shifted PReLU statistics; the apply pass
//        re-derives the sample statistics from the row partials (finalize folded in) and reads y1 once.
//   bwd: the row reduction of (y1, dy) (bwd_reduce_kernel); ONE pass (finalize folded in) that recomputes the
//        gLN/PReLU input gradient at each tap's position from (y1, dy) and runs the dwconv backward on it (dx, dW
//        row partials) plus the PReLU-slope partial of the own elements; one tail launch for dW, dgamma / dbeta and
//        the slope.
constexpr int DW_MAXP = 7, DW_MAXHALO = 512;

template <int P, bool MM = false>
__global__ __launch_bounds__(THREADS) void dwconv_stats_kernel(int row0, int C, int K, int dil, const float* __restrict__ x,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ alpha, float* __restrict__ y1,
                                                               float2* __restrict__ ws, float2* __restrict__ mm = nullptr) {
    // streaming form, no LDS: thread t-loop over the row with the taps' neighbours (+-halo) read straight from the
    // cache lines this workgroup just brought in (each x line leaves HBM once); the same k-ordered sums as the tiled
    // form (bitwise equal y1, same per-thread element order for the statistics)
    __shared__ float red[4];
    const int row = row0 + (int)blockIdx.x, b = row / C, c = row % C;
    const int halo = (P - 1) / 2 * dil;
    const float a = alpha[0];
    const float* xr = x + (int64_t)row * K;
    float* yr = y1 + (int64_t)row * K;
    float wk[P];
#pragma unroll
    for (int k = 0; k < P; ++k) wk[k] = w[c * P + k];
    // the sample's shift p(y1[b, 0, 0]), recomputed with row (b, 0)'s exact arithmetic (zero taps add +0)
    float y00 = 0.f;
    {
        const float* x0 = x + (int64_t)b * C * K;
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const int t = k * dil - halo;
            y00 += w[k] * ((t >= 0 && t < K) ? x0[t] : 0.f);
        }
    }
    const float shift = prelu(y00, a);
    float s1 = 0.f, s2 = 0.f;
    float pmin = __builtin_inff(), pmax = -__builtin_inff();         // MM: the row's PReLU extremes (the split planes' bound)
    const auto rx = make_rsrc(xr, K);                 // taps outside the row load 0 (buffer range check, no branch)
    for (int t0 = 0; t0 < K; t0 += DW_U * THREADS) {  // DW_U elements per thread in flight
        float acc[DW_U];
#pragma unroll
        for (int j = 0; j < DW_U; ++j) {
            const int t = t0 + j * THREADS + threadIdx.x;
            acc[j] = 0.f;
#pragma unroll
            for (int k = 0; k < P; ++k) acc[j] += wk[k] * bufld<float>::ld(rx, t + k * dil - halo, 0);
        }
#pragma unroll
        for (int j = 0; j < DW_U; ++j) {
            const int t = t0 + j * THREADS + threadIdx.x;
            if (t < K) {
                yr[t] = acc[j];
                const float pv = prelu(acc[j], a);
                const float v = pv - shift;
                s1 += v;
                s2 += v * v;
                if constexpr (MM) {
                    pmin = fminf(pmin, pv);
                    pmax = fmaxf(pmax, pv);
                }
            }
        }
    }
    s1 = block_sum(s1, red);
    s2 = block_sum(s2, red);
    if (threadIdx.x == 0) ws[row] = make_float2(s1, s2);
    if constexpr (MM) {
        pmin = -block_sum_max(-pmin, red);
        pmax = block_sum_max(pmax, red);
        if (threadIdx.x == 0) mm[row] = make_float2(pmin, pmax);
    }
}

template <int P>
__global__ __launch_bounds__(THREADS) void dwconv_gln_bwd_kernel(int row0, int C, int K, int dil, const float* __restrict__ x,
                                                                 const float* __restrict__ w, const float* __restrict__ y1,
                                                                 const float* __restrict__ alpha,
                                                                 const float* __restrict__ gamma,
                                                                 const float2* __restrict__ stats,
                                                                 const float2* __restrict__ ws_rows,
                                                                 const float* __restrict__ dy, float* __restrict__ dx,
                                                                 float* __restrict__ ws_dw, float* __restrict__ ws_alpha) {
    // streaming form, no LDS: the PReLU -> gLN input gradient g1(u) is recomputed at each of the P taps' positions
    // from (y1, dy) cache lines (each line leaves HBM once), then dx = the transposed conv of g1 and the row's dW /
    // PReLU-slope partials
    __shared__ float red[THREADS / 64][DW_MAXP + 1];
    __shared__ double dred[8];
    const int row = row0 + second_pass_row(), b = row / C, c = row % C;
    const int halo = (P - 1) / 2 * dil;
    const float a = alpha[0];
    const float2 st = stats[b];
    // the sample's (mean_g, mean_gxh) with g = dy * gamma, from the row partials of bwd_reduce_kernel
    const double2 sg12 = sample_sums(ws_rows, b, C, dred, gamma);
    const double nn = (double)C * K;
    const float2 sm = make_float2((float)(sg12.x / nn), (float)(sg12.y / nn));
    const float gm = gamma[c];
    const float* xr = x + (int64_t)row * K;
    const float* yr = y1 + (int64_t)row * K;
    const float* gr = dy + (int64_t)row * K;
    float* dr = dx + (int64_t)row * K;
    float wk[P], dw[P], da = 0.f;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        wk[k] = w[c * P + k];
        dw[k] = 0.f;
    }
    const auto rx = make_rsrc(xr, K), ry = make_rsrc(yr, K), rg = make_rsrc(gr, K);   // outside the row: 0
    for (int t0 = 0; t0 < K; t0 += DW_UB * THREADS) {
        float acc[DW_UB], gown[DW_UB];
#pragma unroll
        for (int j = 0; j < DW_UB; ++j) {
            const int t = t0 + j * THREADS + threadIdx.x;
            acc[j] = 0.f;
            gown[j] = 0.f;
#pragma unroll
            for (int k = 0; k < P; ++k) {
                // d(gLN(PReLU(y1)))/dy1 applied to dy at u (0 outside the row: y1 = dy = 0 there gives dp = -rstd
                // mean_g..., so mask it)
                const int u = t + halo - k * dil;
                const float yv = bufld<float>::ld(ry, u, 0), gv = bufld<float>::ld(rg, u, 0);
                const float xh = (prelu(yv, a) - st.x) * st.y;
                float dp = st.y * (gv * gm - sm.x - xh * sm.y);
                dp = (u >= 0 && u < K) ? dp : 0.f;
                const float gk = yv > 0.f ? dp : a * dp;
                acc[j] += wk[k] * gk;
                if (k == (P - 1) / 2) {                   // the own element: g for dW, the slope partial
                    gown[j] = gk;
                    if (t < K && yv <= 0.f) da += dp * yv;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < DW_UB; ++j) {
            const int t = t0 + j * THREADS + threadIdx.x;
            if (t < K) {
                dr[t] = acc[j];
#pragma unroll
                for (int k = 0; k < P; ++k) dw[k] += gown[j] * bufld<float>::ld(rx, t + k * dil - halo, 0);
            }
        }
    }
#pragma unroll
    for (int k = 0; k <= P; ++k) {
        float v = k < P ? dw[k] : da;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][k] = v;
    }
    __syncthreads();
    if (threadIdx.x <= P) {
        const float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
        if (threadIdx.x < P) ws_dw[(int64_t)row * DW_MAXP + threadIdx.x] = v;
        else ws_alpha[row] = v;
    }
}

// The backward pass with 4 consecutive elements per thread and dwordx4 tap loads (dil % 4 == 0, so every tap
// quadruple is either wholly before the row or starts inside it; the row's tail is clipped dword by dword by the
// buffer range check).  y1 is NOT read: at each of the P tap positions it is recomputed from x with the forward's
// exact arithmetic (dwconv_stats_kernel: acc = 0, then += w_m x_m for m = 0..P-1), from the 2P - 1 x quadruples
// t + (m - k) dil that also serve the dW taps, so this pass moves x + dy + dx (12 B per element) instead of
// x + y1 + dy + dx (16): the x quadruples of the neighbouring taps come from the lines this row's workgroup just
// loaded.  Same per-element arithmetic and tap order as the y1-reading form.
template <int P>
__global__ __launch_bounds__(THREADS) void dwconv_gln_bwd4_kernel(int row0, int C, int K, int dil, const float* __restrict__ x,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ alpha,
                                                                  const float* __restrict__ gamma,
                                                                  const float2* __restrict__ stats,
                                                                  const float2* __restrict__ ws_rows,
                                                                  const float* __restrict__ dy, float* __restrict__ dx,
                                                                  float* __restrict__ ws_dw, float* __restrict__ ws_alpha) {
    // 4 consecutive elements per thread, one quadruple per loop trip: its 2P - 1 + P tap loads are already 8 in flight
    // (P = 3), and the smaller register footprint keeps more waves resident (2 quadruples per trip: 0.144 ms, 3: 0.175,
    // 4: 0.169, 1: 0.132 at C4; tools/gln_ub_ab.sh @ 8f1eec2)
    constexpr int V = 4, UB = 1;
    constexpr int H = (P - 1) / 2, NX = 2 * P - 1;
    __shared__ float red[THREADS / 64][DW_MAXP + 1];
    __shared__ double dred[8];
    const int row = row0 + second_pass_row(), b = row / C, c = row % C;
    const int halo = H * dil;
    const float a = alpha[0];
    const float2 st = stats[b];
    const double2 sg12 = sample_sums(ws_rows, b, C, dred, gamma);
    const double nn = (double)C * K;
    const float2 sm = make_float2((float)(sg12.x / nn), (float)(sg12.y / nn));
    const float gm = gamma[c];
    const float* xr = x + (int64_t)row * K;
    const float* gr = dy + (int64_t)row * K;
    float* dr = dx + (int64_t)row * K;
    float wk[P], dw[P], da = 0.f;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        wk[k] = w[c * P + k];
        dw[k] = 0.f;
    }
    const auto rx = make_rsrc(xr, K), rg = make_rsrc(gr, K), rd = make_rsrc(dr, K);
    for (int t0 = 0; t0 < K; t0 += UB * V * THREADS) {
        float acc[UB][V], gown[UB][V];
        float4 xq[UB][NX];                        // x at t + (i - (P - 1)) dil, i = 0 .. 2P - 2
        float4 gq[UB][P];                         // dy at the tap positions u_k = t + halo - k dil
#pragma unroll
        for (int j = 0; j < UB; ++j) {
            const int t = t0 + (j * THREADS + (int)threadIdx.x) * V;
#pragma unroll
            for (int i = 0; i < NX; ++i) xq[j][i] = ld4(rx, t + (i - (P - 1)) * dil);
#pragma unroll
            for (int k = 0; k < P; ++k) gq[j][k] = ld4(rg, t + halo - k * dil);
        }
#pragma unroll
        for (int j = 0; j < UB; ++j) {
            const int t = t0 + (j * THREADS + (int)threadIdx.x) * V;
#pragma unroll
            for (int e = 0; e < V; ++e) acc[j][e] = gown[j][e] = 0.f;
#pragma unroll
            for (int k = 0; k < P; ++k) {
                const int u = t + halo - k * dil;
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    // y1(u + e) = sum_m w_m x(u + e + m dil - halo) = sum_m w_m xq[(P - 1) + m - k]
                    float yv = 0.f;
#pragma unroll
                    for (int m = 0; m < P; ++m) yv += wk[m] * f4at(xq[j][P - 1 + m - k], e);
                    const float gv = f4at(gq[j][k], e);
                    const float xh = (prelu(yv, a) - st.x) * st.y;
                    float dp = st.y * (gv * gm - sm.x - xh * sm.y);
                    dp = (u + e >= 0 && u + e < K) ? dp : 0.f;
                    const float gk = yv > 0.f ? dp : a * dp;
                    acc[j][e] += wk[k] * gk;
                    if (k == H) {
                        gown[j][e] = gk;          // 0 past the row's end (dp masked)
                        if (yv <= 0.f) da += dp * yv;
                    }
                }
            }
            if (t + V <= K) {
                const u4_t o = {__float_as_uint(acc[j][0]), __float_as_uint(acc[j][1]), __float_as_uint(acc[j][2]),
                                __float_as_uint(acc[j][3])};
                __builtin_amdgcn_raw_buffer_store_b128(o, rd, t * 4, 0, 0);
            } else {                                  // the row's last, partial quadruple (or none past the end)
#pragma unroll
                for (int e = 0; e < V; ++e)
                    if (t + e < K) dr[t + e] = acc[j][e];
            }
#pragma unroll
            for (int k = 0; k < P; ++k) {
                const int q = t + k * dil - halo;     // x taps outside the row are zero padding
#pragma unroll
                for (int e = 0; e < V; ++e)
                    dw[k] += (q + e >= 0 && q + e < K) ? gown[j][e] * f4at(xq[j][P - 1 + k - H], e) : 0.f;
            }
        }
    }
#pragma unroll
    for (int k = 0; k <= P; ++k) {
        float v = k < P ? dw[k] : da;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][k] = v;
    }
    __syncthreads();
    if (threadIdx.x <= P) {
        const float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
        if (threadIdx.x < P) ws_dw[(int64_t)row * DW_MAXP + threadIdx.x] = v;
        else ws_alpha[row] = v;
    }
}

__global__ void dw_sum_kernel(const float* __restrict__ ws, int B, int C, int P, float* __restrict__ dw) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C * P) return;
    const int c = i / P, k = i % P;
    float v = 0.f;
    for (int b = 0; b < B; ++b) v += ws[((int64_t)b * C + c) * DW_MAXP + k];
    dw[i] = v;
}

// the fused backward's tail, one launch: block 0 = dalpha (alpha_finalize), the next blocks dW (dw_sum_kernel) and
// per channel dgamma / dbeta (sum over b of the row partials: bwd_finalize's channel blocks)
__global__ void dw_tail_kernel(const float* __restrict__ ws_dw, const float2* __restrict__ ws_rows,
                               const float* __restrict__ ws_alpha, int B, int C, int P, float* __restrict__ dw,
                               float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dalpha) {
    if (blockIdx.x == 0) {
        // 32 loads per thread in flight: the row partials were written by workgroups on every XCD, so each pass of
        // this loop is a round trip to the memory-side cache (8 in flight: 4 round trips, 12.8 us for C4's 8192 rows)
        // (a guarded load per element had become a branch + wait per load: 32 serial round trips, 13.5 us; the buffer
        // range check returns 0 past the end without a branch)
        __shared__ double red[4];
        double s = 0.0;
        const auto ra = make_rsrc(ws_alpha, (int64_t)B * C);
        for (int i0 = 0; i0 < B * C; i0 += 32 * blockDim.x) {
            float v[32];
#pragma unroll
            for (int j = 0; j < 32; ++j) v[j] = bufld<float>::ld(ra, i0 + j * (int)blockDim.x + (int)threadIdx.x, 0);
#pragma unroll
            for (int j = 0; j < 32; ++j) s += v[j];
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) dalpha[0] = (float)(red[0] + red[1] + red[2] + red[3]);
        return;
    }
    // sums over the batch with 16 loads in flight per thread (buffer loads: no per-load branch)
    const int i = (blockIdx.x - 1) * blockDim.x + threadIdx.x;
    if (i < C * P) {
        const int c = i / P, k = i % P;
        const auto rw = make_rsrc(ws_dw, (int64_t)B * C * DW_MAXP);
        float v = 0.f;
        for (int b0 = 0; b0 < B; b0 += 16) {
            float t[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) t[j] = bufld<float>::ld(rw, (b0 + j < B ? (b0 + j) * C + c : B * C) * DW_MAXP + k, 0);
#pragma unroll
            for (int j = 0; j < 16; ++j) v += t[j];
        }
        dw[i] = v;
    } else if (i < C * P + C) {
        const int c = i - C * P;
        const auto rr = make_rsrc(reinterpret_cast<const float*>(ws_rows), (int64_t)2 * B * C);
        double g = 0.0, bt = 0.0;
        for (int b0 = 0; b0 < B; b0 += 16) {
            float t[16][2];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int e = (b0 + j < B ? (b0 + j) * C + c : B * C) * 2;
                t[j][0] = bufld<float>::ld(rr, e, 0);
                t[j][1] = bufld<float>::ld(rr, e + 1, 0);
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                bt += t[j][0];
                g += t[j][1];
            }
        }
        dgamma[c] = (float)g;
        dbeta[c] = (float)bt;
    }
}

}  // namespace gln
}  // namespace avse

using namespace avse::gln;

// Each call is one launch pair over all samples: launch pairs per Infinity-Cache-sized sample group measured slower in
// isolation (round 5: C4 dwconv_gln fwd 0.095 -> 0.136 ms, prelu_gln_bwd 0.131 -> 0.151 ms), and so did a one-launch
// sample-pipelined form (profiles/r05r_gln_pipelined_ab.jsonl).

extern "C" {

// ws rows (float2) | slope partials (float) | sample means (float2) | the split-output bound's row maxima (float2)
int64_t avse_prelu_gln_workspace_bytes(int64_t B, int64_t C) { return 8 * B * C + 4 * B * C + 16 * B + 8 * B * C; }

int avse_prelu_gln_fwd(int64_t B, int64_t C, int64_t K, const float* x, const float* alpha, const float* gamma,
                       const float* beta, float eps, float* y, float* stats, float* workspace, avse_stream_t stream) {
    if (!x || !alpha || !gamma || !beta || !y || !stats || !workspace) return AVSE_EINVAL;
    if (B <= 0 || C <= 0 || K <= 0 || B * C > (1LL << 31) - 1) return AVSE_ESHAPE;
    hipStream_t st = (hipStream_t)stream;
    float2* ws = (float2*)workspace;
    // row statistics, then the apply pass (x re-read from the Infinity Cache)
    const int64_t S = B;
    for (int64_t b0 = 0; b0 < B; b0 += S) {
        const int row0 = (int)(b0 * C);
        const unsigned rows = (unsigned)((b0 + S <= B ? S : B - b0) * C);
        hipLaunchKernelGGL(stats_kernel, dim3(rows), dim3(THREADS), 0, st, row0, (int)C, (int)K, x, alpha, ws);
        AVSE_CHECK_LAUNCH();
        hipLaunchKernelGGL(apply_fused_kernel<false>, dim3(rows), dim3(THREADS), 0, st, row0, (int)C, (int)K, x, alpha, gamma,
                           beta, (const float2*)ws, eps, (float2*)stats, y);
        AVSE_CHECK_LAUNCH();
    }
    return AVSE_OK;
}

int avse_prelu_gln_bwd(int64_t B, int64_t C, int64_t K, const float* x, const float* alpha, const float* gamma,
                       const float* stats, const float* dy, float* dx, float* dalpha, float* dgamma, float* dbeta,
                       float* workspace, avse_stream_t stream) {
    if (!x || !alpha || !gamma || !stats || !dy || !dx || !dalpha || !dgamma || !dbeta || !workspace) return AVSE_EINVAL;
    if (B <= 0 || C <= 0 || K <= 0 || B * C > (1LL << 31) - 1) return AVSE_ESHAPE;
    hipStream_t st = (hipStream_t)stream;
    const unsigned all_rows = (unsigned)(B * C);
    float2* ws = (float2*)workspace;
    float* ws_a = (float*)(ws + B * C);
    float2* smeans = (float2*)(ws_a + B * C);
    // (x, dy) row reduction, then the apply pass, per group of samples (its (x, dy) re-read from the Infinity Cache)
    const int64_t S = B;
    for (int64_t b0 = 0; b0 < B; b0 += S) {
        const int row0 = (int)(b0 * C);
        const unsigned rows = (unsigned)((b0 + S <= B ? S : B - b0) * C);
        hipLaunchKernelGGL(bwd_reduce_kernel<false>, dim3(rows), dim3(THREADS), 0, st, row0, (int)C, (int)K, x, alpha,
                           (const float2*)stats, dy, ws);
        AVSE_CHECK_LAUNCH();
        hipLaunchKernelGGL(bwd_apply_kernel<false>, dim3(rows), dim3(THREADS), 0, st, row0, (int)C, (int)K, x, alpha, gamma,
                           (const float2*)stats, (const float2*)ws, dy, dx, ws_a);
        AVSE_CHECK_LAUNCH();
    }
    // dgamma / dbeta (sum over samples of the row partials) and the PReLU slope
    const unsigned cblocks = (unsigned)((C + 255) / 256);
    hipLaunchKernelGGL(bwd_finalize, dim3((unsigned)B + cblocks), dim3(256), 0, st, (int)B, (int)C, (int)K, ws, gamma,
                       smeans, dgamma, dbeta);
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL(alpha_finalize, dim3(1), dim3(256), 0, st, (int)all_rows, ws_a, dalpha);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_prelu_gln_bwd_q(int64_t B, int64_t C, int64_t K, const float* x, const float* alpha, const float* gamma,
                         const float* stats, const float* dy, void* dx_hi, void* dx_lo, int64_t kp, uint32_t* dx_maxbits,
                         float* dalpha, float* dgamma, float* dbeta, float* workspace, avse_stream_t stream) {
    if (!x || !alpha || !gamma || !stats || !dy || !dx_hi || !dx_lo || !dx_maxbits || !dalpha || !dgamma || !dbeta ||
        !workspace)
        return AVSE_EINVAL;
    if (B <= 0 || C <= 0 || K <= 0 || B * C > (1LL << 31) - 1) return AVSE_ESHAPE;
    if (kp < K || kp % 8 || B * C * kp >= (1LL << 40)) return AVSE_ESHAPE;
    if (((uintptr_t)dx_hi | (uintptr_t)dx_lo) % 16 || ((uintptr_t)workspace % 8)) return AVSE_EALIGN;
    hipStream_t st = (hipStream_t)stream;
    const unsigned rows = (unsigned)(B * C);
    float2* ws = (float2*)workspace;
    float* ws_a = (float*)(ws + B * C);
    float2* smeans = (float2*)(ws_a + B * C);
    float2* mm = smeans + B;
    if ((uintptr_t)smeans % 8) return AVSE_EALIGN;
    if (hipMemsetAsync(dx_maxbits, 0, 4, st) != hipSuccess) return AVSE_ELAUNCH;
    hipLaunchKernelGGL(bwd_reduce_kernel<true>, dim3(rows), dim3(THREADS), 0, st, 0, (int)C, (int)K, x, alpha,
                       (const float2*)stats, dy, ws, mm);
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL(q_bwd_bound_kernel, dim3((unsigned)B), dim3(256), 0, st, (int)C, (int)K, alpha, gamma,
                       (const float2*)stats, (const float2*)ws, (const float2*)mm, dx_maxbits);
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL(bwd_apply_kernel<true>, dim3(rows), dim3(THREADS), 0, st, 0, (int)C, (int)K, x, alpha, gamma,
                       (const float2*)stats, (const float2*)ws, dy, nullptr, ws_a,
                       QOut{dx_maxbits, (_Float16*)dx_hi, (_Float16*)dx_lo, (int)kp});
    AVSE_CHECK_LAUNCH();
    const unsigned cblocks = (unsigned)((C + 255) / 256);
    hipLaunchKernelGGL(bwd_finalize, dim3((unsigned)B + cblocks), dim3(256), 0, st, (int)B, (int)C, (int)K, ws, gamma,
                       smeans, dgamma, dbeta);
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL(alpha_finalize, dim3(1), dim3(256), 0, st, (int)rows, ws_a, dalpha);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

// ------------------------------------------------------------------ fused dwconv <-> PReLU -> gLN

int64_t avse_dwconv_gln_workspace_bytes(int64_t B, int64_t C) {
    return 8 * B * C + 4 * B * C + 16 * B + 4 * B * C * DW_MAXP;
}

#define AVSE_DW_P_SWITCH(P, LAUNCH) \
    switch ((int)(P)) {              \
        case 1: LAUNCH(1); break;    \
        case 3: LAUNCH(3); break;    \
        case 5: LAUNCH(5); break;    \
        default: LAUNCH(7); break;   \
    }

static int dw_check(int64_t B, int64_t C, int64_t K, int64_t P, int64_t dil) {
    if (B <= 0 || C <= 0 || K <= 0 || dil <= 0 || (P != 1 && P != 3 && P != 5 && P != 7) ||
        (P - 1) / 2 * dil > DW_MAXHALO || B * C > (1LL << 31) - 1)
        return AVSE_ESHAPE;
    return AVSE_OK;
}

int avse_dwconv_gln_fwd(int64_t B, int64_t C, int64_t K, int64_t P, int64_t dil, const float* x, const float* w,
                        const float* alpha, const float* gamma, const float* beta, float eps, float* y1, float* y,
                        float* stats, float* workspace, avse_stream_t stream) {
    if (!x || !w || !alpha || !gamma || !beta || !y1 || !y || !stats || !workspace) return AVSE_EINVAL;
    if (int rc = dw_check(B, C, K, P, dil)) return rc;
    hipStream_t st = (hipStream_t)stream;
    float2* ws = (float2*)workspace;
    // per group of samples: y1 (written by the first pass) re-read from the Infinity Cache by the apply pass
    const int64_t S = B;
    for (int64_t b0 = 0; b0 < B; b0 += S) {
        const int row0 = (int)(b0 * C);
        const unsigned rows = (unsigned)((b0 + S <= B ? S : B - b0) * C);
#define L_(PP) hipLaunchKernelGGL(dwconv_stats_kernel<PP>, dim3(rows), dim3(THREADS), 0, st, row0, (int)C, (int)K, \
                              (int)dil, x, w, alpha, y1, ws)
        AVSE_DW_P_SWITCH(P, L_)
#undef L_
        AVSE_CHECK_LAUNCH();
        hipLaunchKernelGGL(apply_fused_kernel<false>, dim3(rows), dim3(THREADS), 0, st, row0, (int)C, (int)K, y1, alpha, gamma,
                           beta, (const float2*)ws, eps, (float2*)stats, y);
        AVSE_CHECK_LAUNCH();
    }
    return AVSE_OK;
}

int avse_dwconv_gln_fwd_q(int64_t B, int64_t C, int64_t K, int64_t P, int64_t dil, const float* x, const float* w,
                          const float* alpha, const float* gamma, const float* beta, float eps, float* y1, void* y_hi,
                          void* y_lo, int64_t kp, uint32_t* y_maxbits, float* stats, float* workspace,
                          avse_stream_t stream) {
    if (!x || !w || !alpha || !gamma || !beta || !y1 || !y_hi || !y_lo || !y_maxbits || !stats || !workspace)
        return AVSE_EINVAL;
    if (int rc = dw_check(B, C, K, P, dil)) return rc;
    if (kp < K || kp % 8 || B * C * kp >= (1LL << 40)) return AVSE_ESHAPE;
    if (((uintptr_t)y_hi | (uintptr_t)y_lo) % 16) return AVSE_EALIGN;
    hipStream_t st = (hipStream_t)stream;
    float2* ws = (float2*)workspace;
    float2* mm = ws + B * C;                      // the row extremes (the backward's slope-partial region)
    const unsigned rows = (unsigned)(B * C);
    if (hipMemsetAsync(y_maxbits, 0, 4, st) != hipSuccess) return AVSE_ELAUNCH;
#define L_(PP) hipLaunchKernelGGL((dwconv_stats_kernel<PP, true>), dim3(rows), dim3(THREADS), 0, st, 0, (int)C, (int)K, \
                              (int)dil, x, w, alpha, y1, ws, mm)
    AVSE_DW_P_SWITCH(P, L_)
#undef L_
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL(q_bound_kernel, dim3((unsigned)B), dim3(256), 0, st, (int)C, (int)K, y1, alpha, gamma, beta,
                       (const float2*)ws, (const float2*)mm, eps, y_maxbits);
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL(apply_fused_kernel<true>, dim3(rows), dim3(THREADS), 0, st, 0, (int)C, (int)K, y1, alpha, gamma,
                       beta, (const float2*)ws, eps, (float2*)stats, nullptr,
                       QOut{y_maxbits, (_Float16*)y_hi, (_Float16*)y_lo, (int)kp});
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_dwconv_gln_bwd(int64_t B, int64_t C, int64_t K, int64_t P, int64_t dil, const float* x, const float* w,
                        const float* y1, const float* alpha, const float* gamma, const float* stats, const float* dy,
                        float* dx, float* dw, float* dalpha, float* dgamma, float* dbeta, float* workspace,
                        avse_stream_t stream) {
    if (!x || !w || !y1 || !alpha || !gamma || !stats || !dy || !dx || !dw || !dalpha || !dgamma || !dbeta || !workspace)
        return AVSE_EINVAL;
    if (int rc = dw_check(B, C, K, P, dil)) return rc;
    hipStream_t st = (hipStream_t)stream;
    float2* ws = (float2*)workspace;
    float* ws_a = (float*)(ws + B * C);
    float* ws_dw = (float*)((float2*)(ws_a + B * C) + B);
    // per group of samples: dy (read by the reduction) re-read from the Infinity Cache by the main pass
    const int64_t S = B;
    for (int64_t b0 = 0; b0 < B; b0 += S) {
    const int row0 = (int)(b0 * C);
    const unsigned rows = (unsigned)((b0 + S <= B ? S : B - b0) * C);
    hipLaunchKernelGGL(bwd_reduce_kernel<false>, dim3(rows), dim3(THREADS), 0, st, row0, (int)C, (int)K, y1, alpha,
                       (const float2*)stats, dy, ws);
    AVSE_CHECK_LAUNCH();
#define L_(PP) hipLaunchKernelGGL(dwconv_gln_bwd_kernel<PP>, dim3(rows), dim3(THREADS), 0, st, row0, (int)C, (int)K, \
                              (int)dil, x, w, y1, alpha, gamma, (const float2*)stats, (const float2*)ws, dy, dx, ws_dw, \
                              ws_a)
#define L4_(PP) hipLaunchKernelGGL(dwconv_gln_bwd4_kernel<PP>, dim3(rows), dim3(THREADS), 0, st, row0, (int)C, (int)K, \
                               (int)dil, x, w, alpha, gamma, (const float2*)stats, (const float2*)ws, dy, dx, ws_dw, ws_a)
    if (dil % 4 == 0) {
        AVSE_DW_P_SWITCH(P, L4_)
    } else {
        AVSE_DW_P_SWITCH(P, L_)
    }
#undef L_
#undef L4_
    AVSE_CHECK_LAUNCH();
    }
    const int n = (int)(C * P + C);
    hipLaunchKernelGGL(dw_tail_kernel, dim3(1 + (n + 255) / 256), dim3(256), 0, st, ws_dw, (const float2*)ws, ws_a,
                       (int)B, (int)C, (int)P, dw, dgamma, dbeta, dalpha);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
