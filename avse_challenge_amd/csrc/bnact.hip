// Fused BatchNorm -> [+ residual] -> activation (none / ReLU / PReLU) for gfx950: forward (training: batch
// statistics and the running-stat update; eval: running statistics) and backward.
//
// Replaces the MIOpen BatchNorm + separate PReLU / ReLU / residual-add passes of the avse1 lip stream
// (/root/reference/baseline/avse1/model.py:29-34 frontend3D BatchNorm3d -> PReLU; utils/resnet.py:40-67
// BasicBlock bn1 -> PReLU, bn2 + shortcut -> PReLU, downsample BatchNorm2d) and of the avse1 audio net
// (model.py:181-267 BatchNorm2d -> ReLU, channels-last).  In the round-2 avse1 step profile MIOpen's
// BatchNorm kernels and the PReLU passes took ~77 ms of kernel time per step (profiles/r02_avse1_*).
//
// One layout covers both memory formats: the activation is an (N, C, S) row-major view -- NCHW / NCDHW
// (S = H*W or T*H*W) and channels-last NHWC (N = batch*H*W, S = 1).  Every kernel maps a thread to a
// fixed column j of the (N, C*S) matrix (channel j / S) and walks rows, so all loads are coalesced
// row segments whatever S is (3x3 ResNet maps or 1-wide NHWC rows), and per-channel sums are per-column
// register partials, summed over the workgroup's row offsets in LDS, written as one (C*S)-wide row per
// row block and reduced per channel by a one-workgroup-per-channel kernel in fp64 (deterministic, no
// atomics).  The forward statistics are shifted by each channel's first element (x[0, c, 0]) so that
// E[x^2] - E[x]^2 does not cancel for large-mean inputs (raw 0..255 lip pixels through Conv3d).
//
// HBM traffic per element: forward 4 B (statistics) + 8 B (apply, +4 with a residual); backward 8 B
// (partials) + 12 B (apply); with a residual 12 + 4 (dres written) and 12.
#include <algorithm>

#include "common.h"

namespace avse {
namespace bnact {

constexpr int THREADS = 256;
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_PRELU = 2 };

struct Geo {
    int64_t N, CS, S;
    int C, TW, RPI, tiles, nrb;
};

template <int V> struct vld;
template <> struct vld<1> {
    __device__ static inline void ld(const float* p, float* v) { v[0] = *p; }
    __device__ static inline void st(float* p, const float* v) { *p = v[0]; }
};
template <> struct vld<4> {
    __device__ static inline void ld(const float* p, float* v) {
        const float4 q = *reinterpret_cast<const float4*>(p);
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    }
    __device__ static inline void st(float* p, const float* v) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    }
};

// per-column constants of the thread's V columns: z = (x - mean) a + b (+ res) -- centred first, as torch does,
// so large-mean inputs do not lose the low bits of z to a cancelling a x + (beta - mean a) -- act slope, rstd
// The mean is carried as a float pair (hi + lo): x - hi is exact for x near the mean (Sterbenz), so the
// centred value keeps its low bits even when |mean| >> std (a ReLU/PReLU mask computed from z would
// otherwise flip for |z| below a * ulp(mean); torch's CPU kernels centre in double).
template <int V, int ACT>
struct ColConst {
    float a[V], b[V], al[V], mean[V], mlo[V], rstd[V], gam[V];
    __device__ inline float centred(float v, int k) const { return (v - mean[k]) - mlo[k]; }
    __device__ inline void load(const Geo& g, int64_t j0, const float* stats, const float* gamma, const float* beta,
                                const float* alpha, int alpha_n) {
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const int c = (int)((j0 + k) / g.S);
            mean[k] = stats[4 * c];
            mlo[k] = stats[4 * c + 1];
            rstd[k] = stats[4 * c + 2];
            gam[k] = gamma ? gamma[c] : 1.f;
            a[k] = gam[k] * rstd[k];
            b[k] = beta ? beta[c] : 0.f;
            al[k] = ACT == ACT_PRELU ? alpha[alpha_n > 1 ? c : 0] : 0.f;
        }
    }
};

template <int ACT>
__device__ inline float act_fwd(float z, float al) {
    if constexpr (ACT == ACT_RELU) return z > 0.f ? z : 0.f;
    else if constexpr (ACT == ACT_PRELU) return z > 0.f ? z : al * z;
    else return z;
}
template <int ACT>
__device__ inline float act_bwd(float z, float g, float al) {
    if constexpr (ACT == ACT_RELU) return z > 0.f ? g : 0.f;
    else if constexpr (ACT == ACT_PRELU) return z > 0.f ? g : al * g;
    else return g;
}

// Sum NQ per-thread column partials over the workgroup's RPI row offsets (quantity MAXQ, if in range: their max);
// row offset 0 writes ws[(blockIdx.y * NQ + q) * CS + j].
template <int V, int NQ, int MAXQ = -1>
__device__ inline void block_partials(const Geo& g, float (&p)[NQ][V], bool valid, int64_t j0, float* ws) {
    __shared__ float part[NQ][THREADS * V];
    const int tx = threadIdx.x % g.TW, ty = threadIdx.x / g.TW;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int k = 0; k < V; ++k) part[q][threadIdx.x * V + k] = p[q][k];
    __syncthreads();
    if (ty == 0 && valid) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            float s[V];
#pragma unroll
            for (int k = 0; k < V; ++k) s[k] = p[q][k];
            for (int t = 1; t < g.RPI; ++t)
#pragma unroll
                for (int k = 0; k < V; ++k)
                    s[k] = q == MAXQ ? fmaxf(s[k], part[q][(t * g.TW + tx) * V + k]) : s[k] + part[q][(t * g.TW + tx) * V + k];
            vld<V>::st(ws + ((int64_t)blockIdx.y * NQ + q) * g.CS + j0, s);
        }
    }
}

// max |out| of the workgroup -> one atomicMax on the float bits (non-negative floats order like their bits) into
// omax: the producer-side max of the split operands (the convolution that consumes the output skips its absmax pass)
__device__ inline void block_max_out(float m, uint32_t* omax) {
    __shared__ uint32_t red[THREADS / 64];
    uint32_t b = __float_as_uint(m);
    for (int o = 32; o >= 1; o >>= 1) b = max(b, (uint32_t)__shfl_xor((int)b, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        b = red[0];
#pragma unroll
        for (int w = 1; w < THREADS / 64; ++w) b = max(b, red[w]);
        if (b) atomicMax(omax, b);
    }
}

// ---- split output ("Q": the operand layout of dconv.hip / sconv.hip, round 5)
// With QOUT the apply passes write their channels-last output (S = 1, C % 64 == 0) directly as the fp16 hi / lo split the
// next convolution reads -- per pixel C / 16 chunks of 64 B = [hi of 16 channels][lo of 16 channels], the bytes of the
// fp32 tensor -- instead of fp32 values that a separate split pass (read 4 B + write 4 B per element) would convert.
// The split scale has to be known before the pass, so it comes from an upper bound of max |out| assembled from the
// per-channel statistics (a bound is enough: any power-of-two scale with no fp16 overflow keeps the 22-bit split; see
// stats_combine / bwd_combine), published as float bits where the exact max would be (y_max / dx_max).
__device__ inline int q_split_exp(uint32_t mb) {          // dconv.hip split_exp: max 2^e in [2^14, 2^15)
    const int ef = (int)((mb >> 23) & 0xff);
    if (mb == 0) return 0;
    const int k = ef == 0 ? -127 : ef - 127;
    return min(100, max(-100, 14 - k));
}
// 4 channels c .. c + 3 (c % 4 == 0) of pixel r: hi at 64 (c / 16) + 2 (c % 16), lo 32 B further
__device__ inline void q_store4(uint16_t* q, int64_t r, int64_t C, int64_t c, const float* v, float sc) {
    uint32_t hi[2], lo[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const float s0 = v[2 * k] * sc, s1 = v[2 * k + 1] * sc;
        const _Float16 h0 = (_Float16)s0, h1 = (_Float16)s1;
        const _Float16 l0 = (_Float16)(s0 - (float)h0), l1 = (_Float16)(s1 - (float)h1);
        hi[k] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
        lo[k] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
    }
    uint16_t* base = q + r * 2 * C + 32 * (c >> 4) + (c & 15);
    *reinterpret_cast<uint2*>(base) = make_uint2(hi[0], hi[1]);
    *reinterpret_cast<uint2*>(base + 16) = make_uint2(lo[0], lo[1]);
}
// the bound's float bits, rounded up by 2^-10 (the apply pass's own fp32 rounding stays below it)
__device__ inline void q_bound_out(double bnd, uint32_t* omax) {
    const float f = (float)(bnd * (1.0 + 1.0 / 1024.0));
    if (f > 0.f) atomicMax(omax, __float_as_uint(f));
}

// ---- forward: statistics partials (shifted sums; MAXD: also max |x - shift| per column, for the split bound),
// finalize, apply
template <int V, bool MAXD>
__global__ __launch_bounds__(THREADS) void stats_kernel(Geo g, const float* __restrict__ x, float* __restrict__ ws) {
    constexpr int NQ = MAXD ? 3 : 2;
    const int tx = threadIdx.x % g.TW, ty = threadIdx.x / g.TW;
    const int64_t j0 = ((int64_t)blockIdx.x * g.TW + tx) * V;
    const bool valid = j0 < g.CS;
    float p[NQ][V], K[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) p[q][k] = 0.f;
        K[k] = valid ? x[((j0 + k) / g.S) * g.S] : 0.f;
    }
    if (valid) {
        for (int64_t r = (int64_t)blockIdx.y * g.RPI + ty; r < g.N; r += (int64_t)gridDim.y * g.RPI) {
            float v[V];
            vld<V>::ld(x + r * g.CS + j0, v);
#pragma unroll
            for (int k = 0; k < V; ++k) {
                const float d = v[k] - K[k];
                p[0][k] += d;
                p[1][k] = fmaf(d, d, p[1][k]);
                if constexpr (MAXD) p[NQ - 1][k] = fmaxf(p[NQ - 1][k], fabsf(d));
            }
        }
    }
    block_partials<V, NQ, MAXD ? 2 : -1>(g, p, valid, j0, ws);
}

__device__ inline double block_sum_d(double v, double* red) {
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
    return s;
}

// Per-channel reduction of the column partials in two launches: chan_partial_kernel splits channel c's
// nrb * S partial entries over G workgroups (grid (C, G), fp64 sums, one value per workgroup and quantity),
// then a one-thread-per-channel combine.  (One workgroup per channel left most CUs idle: 64-512 workgroups
// looping over up to 172800 entries each took ~150 us per call at the avse1 shapes.)
constexpr int MAXG = 64;
inline int chan_groups(const Geo& g) {
    const int64_t cnt = (int64_t)g.nrb * g.S;
    return (int)std::max<int64_t>(1, std::min<int64_t>(MAXG, (cnt + 2047) / 2048));
}

__device__ inline double block_max_d(double v, double* red) {
    for (int m = 32; m >= 1; m >>= 1) v = fmax(v, __shfl_xor(v, m, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s = fmax(s, red[w]);
    return s;
}

// quantity MAXQ (if in range) is a column max, reduced by max; reset: the split bound's word, zeroed in stream order
// before the combine kernel's atomicMax
template <int NQ, int MAXQ = -1>
__global__ __launch_bounds__(THREADS) void chan_partial_kernel(Geo g, const float* __restrict__ ws,
                                                               double* __restrict__ fin, uint32_t* __restrict__ reset) {
    __shared__ double red[THREADS / 64];
    const int c = blockIdx.x, G = gridDim.y, gi = blockIdx.y;
    if (reset && c == 0 && gi == 0 && threadIdx.x == 0) *reset = 0u;
    const int S = (int)g.S, cnt = g.nrb * S;              // < 2^23: nrb * S <= 4096 * 1024 (make_geo)
    const int per = (cnt + G - 1) / G, i0 = gi * per, i1 = min(cnt, i0 + per);
    double acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = 0.0;
    for (int i = i0 + threadIdx.x; i < i1; i += THREADS) {
        const int y = i / S, sidx = i - y * S;
        const int64_t col = (int64_t)c * g.S + sidx;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const double v = ws[((int64_t)y * NQ + q) * g.CS + col];
            acc[q] = q == MAXQ ? fmax(acc[q], v) : acc[q] + v;
        }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const double v = q == MAXQ ? block_max_d(acc[q], red) : block_sum_d(acc[q], red);
        if (threadIdx.x == 0) fin[((int64_t)c * G + gi) * NQ + q] = v;
    }
}

// fin: sum (x - shift), sum (x - shift)^2, max |x - shift| per channel.  stats[4 c + 3] = a bound of max |x - mean| (the
// backward's split bound needs it); qb (split output): the channel's bound of |act(BN(x))| goes to omax (zeroed by
// chan_partial_kernel)
__global__ void stats_combine(Geo g, const float* __restrict__ x, const double* __restrict__ fin, int G, float eps,
                              float momentum, float* __restrict__ running_mean, float* __restrict__ running_var,
                              float* __restrict__ stats, uint32_t* __restrict__ omax, int qb,
                              const float* __restrict__ gamma, const float* __restrict__ beta,
                              const float* __restrict__ alpha, int alpha_n, int act) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (!qb && c == 0 && omax) *omax = 0u;               // the apply pass's max, reset in stream order before it
    if (c >= g.C) return;
    double s1 = 0.0, s2 = 0.0, dmax = 0.0;
    for (int gi = 0; gi < G; ++gi) {
        s1 += fin[((int64_t)c * G + gi) * 3];
        s2 += fin[((int64_t)c * G + gi) * 3 + 1];
        dmax = fmax(dmax, fin[((int64_t)c * G + gi) * 3 + 2]);
    }
    const double n = (double)g.N * (double)g.S;
    const double m1 = s1 / n;
    double var = s2 / n - m1 * m1;
    if (var < 0.0) var = 0.0;
    const double mean = (double)x[(int64_t)c * g.S] + m1;
    const float hi = (float)mean;
    stats[4 * c] = hi;
    stats[4 * c + 1] = (float)(mean - (double)hi);
    const double rstd = 1.0 / sqrt(var + (double)eps);
    stats[4 * c + 2] = (float)rstd;
    // |x - mean| <= max |x - shift| + |shift - mean|; |z| <= |gamma rstd| that + |beta|; ReLU / PReLU scale by <= max(1, |slope|)
    const double dev = dmax + fabs(m1);
    stats[4 * c + 3] = (float)(dev * (1.0 + 1.0 / 1024.0));
    if (qb) {
        const double ga = gamma ? fabs((double)gamma[c]) : 1.0;
        double bz = ga * rstd * dev + (beta ? fabs((double)beta[c]) : 0.0);
        if (act == ACT_PRELU) bz *= fmax(1.0, fabs((double)alpha[alpha_n > 1 ? c : 0]));
        q_bound_out(bz, omax);
    }
    if (running_mean) running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
    if (running_var) running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * var * n / (n - 1.0));
}

__global__ void eval_stats_kernel(int C, const float* __restrict__ rm, const float* __restrict__ rv, float eps,
                                  float* __restrict__ stats, uint32_t* __restrict__ omax) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c == 0 && omax) *omax = 0u;
    if (c < C) {
        stats[4 * c] = rm[c];
        stats[4 * c + 1] = 0.f;
        stats[4 * c + 2] = (float)(1.0 / sqrt((double)rv[c] + (double)eps));
        stats[4 * c + 3] = 0.f;
    }
}

template <int V, int ACT, bool RES, bool QOUT = false>
__global__ __launch_bounds__(THREADS) void apply_kernel(Geo g, const float* __restrict__ x, const float* __restrict__ res,
                                                        const float* __restrict__ stats, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, const float* __restrict__ alpha,
                                                        int alpha_n, float* __restrict__ y, uint32_t* __restrict__ ymax) {
    const int tx = threadIdx.x % g.TW, ty = threadIdx.x / g.TW;
    const int64_t j0 = ((int64_t)blockIdx.x * g.TW + tx) * V;
    float m = 0.f;
    if constexpr (QOUT) {                                 // S = 1, V = 4, no residual (host-checked)
        const float sc = __builtin_ldexpf(1.f, q_split_exp(*ymax));
        if (j0 < g.CS) {
            ColConst<V, ACT> cc;
            cc.load(g, j0, stats, gamma, beta, alpha, alpha_n);
            for (int64_t r = (int64_t)blockIdx.y * g.RPI + ty; r < g.N; r += (int64_t)gridDim.y * g.RPI) {
                float v[V];
                vld<V>::ld(x + r * g.CS + j0, v);
#pragma unroll
                for (int k = 0; k < V; ++k) v[k] = act_fwd<ACT>(fmaf(cc.centred(v[k], k), cc.a[k], cc.b[k]), cc.al[k]);
                q_store4(reinterpret_cast<uint16_t*>(y), r, g.CS, j0, v, sc);
            }
        }
        return;
    }
    if (j0 < g.CS) {
        ColConst<V, ACT> cc;
        cc.load(g, j0, stats, gamma, beta, alpha, alpha_n);
        for (int64_t r = (int64_t)blockIdx.y * g.RPI + ty; r < g.N; r += (int64_t)gridDim.y * g.RPI) {
            const int64_t o = r * g.CS + j0;
            float v[V], rv[V];
            vld<V>::ld(x + o, v);
            if (RES) vld<V>::ld(res + o, rv);
#pragma unroll
            for (int k = 0; k < V; ++k) {
                float z = fmaf(cc.centred(v[k], k), cc.a[k], cc.b[k]);
                if (RES) z += rv[k];
                v[k] = act_fwd<ACT>(z, cc.al[k]);
                m = fmaxf(m, fabsf(v[k]));
            }
            vld<V>::st(y + o, v);
        }
    }
    if (ymax) block_max_out(m, ymax);                    // workgroup-uniform condition
}

// ---- backward: partials of sum dz, sum dz*xhat, PReLU slope; finalize; apply
template <int V, int ACT, bool RES, bool MAXDZ = false>
__global__ __launch_bounds__(THREADS) void bwd_partial_kernel(Geo g, const float* __restrict__ x,
                                                              const float* __restrict__ res, const float* __restrict__ dy,
                                                              const float* __restrict__ stats,
                                                              const float* __restrict__ gamma, const float* __restrict__ beta,
                                                              const float* __restrict__ alpha, int alpha_n,
                                                              float* __restrict__ ws, float* __restrict__ dres) {
    constexpr int NQ = MAXDZ ? 4 : 3;
    const int tx = threadIdx.x % g.TW, ty = threadIdx.x / g.TW;
    const int64_t j0 = ((int64_t)blockIdx.x * g.TW + tx) * V;
    const bool valid = j0 < g.CS;
    float p[NQ][V];
#pragma unroll
    for (int k = 0; k < V; ++k)
#pragma unroll
        for (int q = 0; q < NQ; ++q) p[q][k] = 0.f;
    if (valid) {
        ColConst<V, ACT> cc;
        cc.load(g, j0, stats, gamma, beta, alpha, alpha_n);
        for (int64_t r = (int64_t)blockIdx.y * g.RPI + ty; r < g.N; r += (int64_t)gridDim.y * g.RPI) {
            const int64_t o = r * g.CS + j0;
            float v[V], gv[V], rv[V], dz[V];
            vld<V>::ld(x + o, v);
            vld<V>::ld(dy + o, gv);
            if (RES) vld<V>::ld(res + o, rv);
#pragma unroll
            for (int k = 0; k < V; ++k) {
                float z = fmaf(cc.centred(v[k], k), cc.a[k], cc.b[k]);
                if (RES) z += rv[k];
                dz[k] = act_bwd<ACT>(z, gv[k], cc.al[k]);
                const float xh = cc.centred(v[k], k) * cc.rstd[k];
                p[0][k] += dz[k];
                p[1][k] = fmaf(dz[k], xh, p[1][k]);
                if (ACT == ACT_PRELU && !(z > 0.f)) p[2][k] = fmaf(gv[k], z, p[2][k]);
                if constexpr (MAXDZ) p[3][k] = fmaxf(p[3][k], fabsf(dz[k]));
            }
            if (RES) vld<V>::st(dres + o, dz);
        }
    }
    block_partials<V, NQ, MAXDZ ? 3 : -1>(g, p, valid, j0, ws);
}

// qb (split output): fin carries a fourth quantity, max |dz|; the channel's bound of |dx| goes to omax (zeroed by
// chan_partial_kernel): |dx| <= |gamma rstd| (max |dz| + |k1| + max |xhat| |k2|), max |xhat| from the forward's
// stats[4 c + 3] (training; eval: |gamma rstd| max |dz|)
__global__ void bwd_combine(Geo g, const double* __restrict__ fin, int G, int training, float* __restrict__ dgamma,
                            float* __restrict__ dbeta, float* __restrict__ dalpha_c, float* __restrict__ kbuf,
                            uint32_t* __restrict__ omax, int qb, const float* __restrict__ stats,
                            const float* __restrict__ gamma) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (!qb && c == 0 && omax) *omax = 0u;               // the apply pass's max, reset in stream order before it
    if (c >= g.C) return;
    const int NQ = qb ? 4 : 3;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, dzmax = 0.0;
    for (int gi = 0; gi < G; ++gi) {
        s0 += fin[((int64_t)c * G + gi) * NQ];
        s1 += fin[((int64_t)c * G + gi) * NQ + 1];
        s2 += fin[((int64_t)c * G + gi) * NQ + 2];
        if (qb) dzmax = fmax(dzmax, fin[((int64_t)c * G + gi) * NQ + 3]);
    }
    const double n = (double)g.N * (double)g.S;
    if (dbeta) dbeta[c] = (float)s0;
    if (dgamma) dgamma[c] = (float)s1;
    if (dalpha_c) dalpha_c[c] = (float)s2;
    kbuf[2 * c] = training ? (float)(s0 / n) : 0.f;
    kbuf[2 * c + 1] = training ? (float)(s1 / n) : 0.f;
    if (qb) {
        const double rstd = (double)stats[4 * c + 2];
        const double ga = (gamma ? fabs((double)gamma[c]) : 1.0) * rstd;
        const double b = training ? dzmax + fabs(s0 / n) + (double)stats[4 * c + 3] * rstd * fabs(s1 / n) : dzmax;
        q_bound_out(ga * b, omax);
    }
}

template <int V, int ACT, bool RES, bool QOUT = false>
__device__ inline void bwd_apply_cols(const Geo& g, int64_t j0, int ty, const float* __restrict__ x,
                                      const float* __restrict__ dy, const float* __restrict__ dres,
                                      const float* __restrict__ stats, const float* __restrict__ gamma,
                                      const float* __restrict__ beta, const float* __restrict__ alpha, int alpha_n,
                                      const float* __restrict__ kbuf, float* __restrict__ dx, float& m, float qsc = 1.f) {
    ColConst<V, ACT> cc;
    cc.load(g, j0, stats, gamma, beta, alpha, alpha_n);
    float k1[V], k2[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
        const int c = (int)((j0 + k) / g.S);
        k1[k] = kbuf[2 * c];
        k2[k] = kbuf[2 * c + 1];
    }
    for (int64_t r = (int64_t)blockIdx.y * g.RPI + ty; r < g.N; r += (int64_t)gridDim.y * g.RPI) {
        const int64_t o = r * g.CS + j0;
        float v[V], dz[V];
        vld<V>::ld(x + o, v);
        if (RES) {
            vld<V>::ld(dres + o, dz);                  // dz of the pre-activation, written by the partial pass
        } else {
            float gv[V];
            vld<V>::ld(dy + o, gv);
#pragma unroll
            for (int k = 0; k < V; ++k) dz[k] = act_bwd<ACT>(fmaf(cc.centred(v[k], k), cc.a[k], cc.b[k]), gv[k], cc.al[k]);
        }
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const float xh = cc.centred(v[k], k) * cc.rstd[k];
            v[k] = cc.a[k] * (dz[k] - k1[k] - xh * k2[k]);
            if constexpr (!QOUT) m = fmaxf(m, fabsf(v[k]));
        }
        if constexpr (QOUT) q_store4(reinterpret_cast<uint16_t*>(dx), r, g.CS, j0, v, qsc);
        else vld<V>::st(dx + o, v);
    }
}

template <int V, int ACT, bool RES, bool QOUT = false>
__global__ __launch_bounds__(THREADS) void bwd_apply_kernel(Geo g, const float* __restrict__ x,
                                                            const float* __restrict__ dy, const float* __restrict__ dres,
                                                            const float* __restrict__ stats,
                                                            const float* __restrict__ gamma, const float* __restrict__ beta,
                                                            const float* __restrict__ alpha, int alpha_n,
                                                            const float* __restrict__ kbuf, float* __restrict__ dx,
                                                            uint32_t* __restrict__ dxmax) {
    const int tx = threadIdx.x % g.TW, ty = threadIdx.x / g.TW;
    const int64_t j0 = ((int64_t)blockIdx.x * g.TW + tx) * V;
    float m = 0.f;
    if constexpr (QOUT) {                                 // S = 1, V = 4 (host-checked)
        const float sc = __builtin_ldexpf(1.f, q_split_exp(*dxmax));
        if (j0 < g.CS)
            bwd_apply_cols<V, ACT, RES, true>(g, j0, ty, x, dy, dres, stats, gamma, beta, alpha, alpha_n, kbuf, dx, m, sc);
        return;
    }
    if (j0 < g.CS) bwd_apply_cols<V, ACT, RES>(g, j0, ty, x, dy, dres, stats, gamma, beta, alpha, alpha_n, kbuf, dx, m);
    if (dxmax) block_max_out(m, dxmax);                  // workgroup-uniform condition
}

// ---- host side
inline int pow2ceil(int64_t v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

inline Geo make_geo(int64_t N, int64_t C, int64_t S, int V) {
    Geo g;
    g.N = N; g.S = S; g.C = (int)C; g.CS = C * S;
    const int64_t cw = (g.CS + V - 1) / V;
    g.TW = cw >= THREADS ? THREADS : pow2ceil(cw);
    g.RPI = THREADS / g.TW;
    g.tiles = (int)((cw + g.TW - 1) / g.TW);
    const int64_t want = (N + (int64_t)g.RPI * 8 - 1) / ((int64_t)g.RPI * 8);      // >= 8 rows per thread
    const int64_t cap = std::max<int64_t>(1, 4096 / g.tiles);
    g.nrb = (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(want, cap), 65535));
    return g;
}

inline bool shape_ok(int64_t N, int64_t C, int64_t S) {
    return N > 0 && C > 0 && S > 0 && N * C * S < (1LL << 40) && C * S < (1LL << 31) && C < (1 << 20) &&
           (C * S + 3) / 4 <= (int64_t)THREADS * 0x7FFFFFFF;
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// fp64 per-channel partials after the column partials and kbuf (the largest nrb of either vector width)
inline double* fin_ptr(float* workspace, const Geo& g) {
    const Geo g1 = make_geo(g.N, g.C, g.S, 1), g4 = make_geo(g.N, g.C, g.S, 4);
    const int64_t nrb = std::max(g1.nrb, g4.nrb);
    const uintptr_t p = (uintptr_t)(workspace + 4 * nrb * g.CS + 2 * (int64_t)g.C);
    return reinterpret_cast<double*>((p + 15) & ~(uintptr_t)15);
}

template <template <int, int, bool> class K>
struct dispatch {
    template <typename... A>
    static void run(int V, int act, bool res, dim3 grid, hipStream_t st, A... a) {
#define AVSE_BNACT_CASE(VV, AA, RR) \
    if (V == VV && act == AA && res == RR) { hipLaunchKernelGGL((K<VV, AA, RR>::fn), grid, dim3(THREADS), 0, st, a...); return; }
        AVSE_BNACT_CASE(4, ACT_NONE, false) AVSE_BNACT_CASE(4, ACT_RELU, false) AVSE_BNACT_CASE(4, ACT_PRELU, false)
        AVSE_BNACT_CASE(4, ACT_NONE, true) AVSE_BNACT_CASE(4, ACT_RELU, true) AVSE_BNACT_CASE(4, ACT_PRELU, true)
        AVSE_BNACT_CASE(1, ACT_NONE, false) AVSE_BNACT_CASE(1, ACT_RELU, false) AVSE_BNACT_CASE(1, ACT_PRELU, false)
        AVSE_BNACT_CASE(1, ACT_NONE, true) AVSE_BNACT_CASE(1, ACT_RELU, true) AVSE_BNACT_CASE(1, ACT_PRELU, true)
#undef AVSE_BNACT_CASE
    }
};
template <int V, int A, bool R> struct ApplyK { static constexpr auto fn = apply_kernel<V, A, R>; };
template <int V, int A, bool R> struct ApplyQK { static constexpr auto fn = apply_kernel<V, A, R, true>; };
template <int V, int A, bool R> struct BwdPartQK { static constexpr auto fn = bwd_partial_kernel<V, A, R, true>; };
template <int V, int A, bool R> struct BwdApplyQK { static constexpr auto fn = bwd_apply_kernel<V, A, R, true>; };
// the split-output kernels: V = 4, no residual
template <template <int, int, bool> class K>
struct dispatch_q {
    template <typename... A>
    static void run(int act, dim3 grid, hipStream_t st, A... a) {
        if (act == ACT_NONE) hipLaunchKernelGGL((K<4, ACT_NONE, false>::fn), grid, dim3(THREADS), 0, st, a...);
        else if (act == ACT_RELU) hipLaunchKernelGGL((K<4, ACT_RELU, false>::fn), grid, dim3(THREADS), 0, st, a...);
        else hipLaunchKernelGGL((K<4, ACT_PRELU, false>::fn), grid, dim3(THREADS), 0, st, a...);
    }
};
template <int V, int A, bool R> struct BwdPartK { static constexpr auto fn = bwd_partial_kernel<V, A, R>; };
template <int V, int A, bool R> struct BwdApplyK { static constexpr auto fn = bwd_apply_kernel<V, A, R>; };

}  // namespace bnact
}  // namespace avse

using namespace avse::bnact;

extern "C" {

int64_t avse_bnact_workspace_bytes(int64_t N, int64_t C, int64_t S) {
    if (!shape_ok(N, C, S)) return 0;
    const Geo g = make_geo(N, C, S, 1);                 // V = 1 has the most row blocks
    const Geo g4 = make_geo(N, C, S, 4);
    const int64_t nrb = std::max(g.nrb, g4.nrb);
    // column partials (up to 4 rows of C*S per row block), kbuf (2 C floats), then 8-aligned fp64 per-channel partials
    return 4 * (4 * nrb * C * S + 2 * C) + 16 + 8 * (int64_t)C * MAXG * 4;
}

static int bnact_fwd_impl(int64_t N, int64_t C, int64_t S, const float* x, const float* res, const float* gamma,
                          const float* beta, int32_t act, const float* alpha, int32_t alpha_n, int32_t training, float eps,
                          float momentum, float* running_mean, float* running_var, float* stats, float* y,
                          float* workspace, uint32_t* y_max, bool qout, hipStream_t st) {
    if (!x || !y || !stats || !workspace || (act == ACT_PRELU && !alpha)) return AVSE_EINVAL;
    if (!training && (!running_mean || !running_var)) return AVSE_EINVAL;
    if (!shape_ok(N, C, S) || act < ACT_NONE || act > ACT_PRELU) return AVSE_ESHAPE;
    if (act == ACT_PRELU && alpha_n != 1 && alpha_n != C) return AVSE_ESHAPE;
    if (training && N * S < 2) return AVSE_ESHAPE;       // as torch: more than one value per channel
    const int V = ((C * S) % 4 == 0 && al16(x) && al16(y) && (!res || al16(res)) && al16(workspace)) ? 4 : 1;
    if (qout && (!y_max || !training || res || S != 1 || C % 64 || V != 4)) return AVSE_ESHAPE;
    const Geo g = make_geo(N, C, S, V);
    const dim3 grid(g.tiles, g.nrb);
    if (training) {
        if (V == 4) hipLaunchKernelGGL((stats_kernel<4, true>), grid, dim3(THREADS), 0, st, g, x, workspace);
        else hipLaunchKernelGGL((stats_kernel<1, true>), grid, dim3(THREADS), 0, st, g, x, workspace);
        AVSE_CHECK_LAUNCH();
        const int G = chan_groups(g);
        double* fin = fin_ptr(workspace, g);
        hipLaunchKernelGGL((chan_partial_kernel<3, 2>), dim3((unsigned)C, G), dim3(THREADS), 0, st, g,
                           (const float*)workspace, fin, qout ? y_max : (uint32_t*)nullptr);
        AVSE_CHECK_LAUNCH();
        hipLaunchKernelGGL(stats_combine, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, g, x, (const double*)fin,
                           G, eps, momentum, running_mean, running_var, stats, y_max, (int)qout, gamma, beta, alpha,
                           (int)alpha_n, (int)act);
    } else {
        hipLaunchKernelGGL(eval_stats_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, (int)C, running_mean,
                           running_var, eps, stats, y_max);
    }
    AVSE_CHECK_LAUNCH();
    if (qout)
        dispatch_q<ApplyQK>::run(act, grid, st, g, x, res, (const float*)stats, gamma, beta, alpha, (int)alpha_n, y, y_max);
    else
        dispatch<ApplyK>::run(V, act, res != nullptr, grid, st, g, x, res, (const float*)stats, gamma, beta, alpha,
                              (int)alpha_n, y, y_max);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_bnact_fwd(int64_t N, int64_t C, int64_t S, const float* x, const float* res, const float* gamma,
                   const float* beta, int32_t act, const float* alpha, int32_t alpha_n, int32_t training, float eps,
                   float momentum, float* running_mean, float* running_var, float* stats, float* y, float* workspace,
                   uint32_t* y_max, avse_stream_t stream) {
    return bnact_fwd_impl(N, C, S, x, res, gamma, beta, act, alpha, alpha_n, training, eps, momentum, running_mean,
                          running_var, stats, y, workspace, y_max, false, (hipStream_t)stream);
}

int avse_bnact_fwd_q(int64_t N, int64_t C, int64_t S, const float* x, const float* gamma, const float* beta, int32_t act,
                     const float* alpha, int32_t alpha_n, float eps, float momentum, float* running_mean,
                     float* running_var, float* stats, void* yq, float* workspace, uint32_t* y_bound,
                     avse_stream_t stream) {
    return bnact_fwd_impl(N, C, S, x, nullptr, gamma, beta, act, alpha, alpha_n, 1, eps, momentum, running_mean,
                          running_var, stats, (float*)yq, workspace, y_bound, true, (hipStream_t)stream);
}

static int bnact_bwd_impl(int64_t N, int64_t C, int64_t S, const float* x, const float* res, const float* dy,
                          const float* stats, const float* gamma, const float* beta, int32_t act, const float* alpha,
                          int32_t alpha_n, int32_t training, float* dx, float* dres, float* dgamma, float* dbeta,
                          float* dalpha_c, float* workspace, uint32_t* dx_max, bool qout, hipStream_t st) {
    if (!x || !dy || !stats || !dx || !workspace || (act == ACT_PRELU && (!alpha || !dalpha_c)) || (res && !dres))
        return AVSE_EINVAL;
    if (!shape_ok(N, C, S) || act < ACT_NONE || act > ACT_PRELU) return AVSE_ESHAPE;
    if (act == ACT_PRELU && alpha_n != 1 && alpha_n != C) return AVSE_ESHAPE;
    const int V = ((C * S) % 4 == 0 && al16(x) && al16(dy) && al16(dx) && (!res || (al16(res) && al16(dres))) &&
                   al16(workspace)) ? 4 : 1;
    if (qout && (!dx_max || res || S != 1 || C % 64 || V != 4)) return AVSE_ESHAPE;
    const Geo g = make_geo(N, C, S, V);
    const dim3 grid(g.tiles, g.nrb);
    float* kbuf = workspace + 4 * (int64_t)g.nrb * g.CS;
    const int G = chan_groups(g);
    double* fin = fin_ptr(workspace, g);
    if (qout) {
        dispatch_q<BwdPartQK>::run(act, grid, st, g, x, res, dy, stats, gamma, beta, alpha, (int)alpha_n, workspace, dres);
        AVSE_CHECK_LAUNCH();
        hipLaunchKernelGGL((chan_partial_kernel<4, 3>), dim3((unsigned)C, G), dim3(THREADS), 0, st, g,
                           (const float*)workspace, fin, dx_max);
    } else {
        dispatch<BwdPartK>::run(V, act, res != nullptr, grid, st, g, x, res, dy, stats, gamma, beta, alpha, (int)alpha_n,
                                workspace, dres);
        AVSE_CHECK_LAUNCH();
        hipLaunchKernelGGL((chan_partial_kernel<3>), dim3((unsigned)C, G), dim3(THREADS), 0, st, g,
                           (const float*)workspace, fin, (uint32_t*)nullptr);
    }
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL(bwd_combine, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, g, (const double*)fin, G,
                       (int)training, dgamma, dbeta, dalpha_c, kbuf, dx_max, (int)qout, stats, gamma);
    AVSE_CHECK_LAUNCH();
    if (qout)
        dispatch_q<BwdApplyQK>::run(act, grid, st, g, x, dy, (const float*)dres, stats, gamma, beta, alpha, (int)alpha_n,
                                   (const float*)kbuf, dx, dx_max);
    else
        dispatch<BwdApplyK>::run(V, act, res != nullptr, grid, st, g, x, dy, (const float*)dres, stats, gamma, beta,
                                 alpha, (int)alpha_n, (const float*)kbuf, dx, dx_max);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_bnact_bwd(int64_t N, int64_t C, int64_t S, const float* x, const float* res, const float* dy, const float* stats,
                   const float* gamma, const float* beta, int32_t act, const float* alpha, int32_t alpha_n,
                   int32_t training, float* dx, float* dres, float* dgamma, float* dbeta, float* dalpha_c,
                   float* workspace, uint32_t* dx_max, avse_stream_t stream) {
    return bnact_bwd_impl(N, C, S, x, res, dy, stats, gamma, beta, act, alpha, alpha_n, training, dx, dres, dgamma,
                          dbeta, dalpha_c, workspace, dx_max, false, (hipStream_t)stream);
}

int avse_bnact_bwd_q(int64_t N, int64_t C, int64_t S, const float* x, const float* dy, const float* stats,
                     const float* gamma, const float* beta, int32_t act, const float* alpha, int32_t alpha_n,
                     int32_t training, void* dxq, float* dgamma, float* dbeta, float* dalpha_c, float* workspace,
                     uint32_t* dx_bound, avse_stream_t stream) {
    return bnact_bwd_impl(N, C, S, x, nullptr, dy, stats, gamma, beta, act, alpha, alpha_n, training, (float*)dxq,
                          nullptr, dgamma, dbeta, dalpha_c, workspace, dx_bound, true, (hipStream_t)stream);
}

}  // extern "C"
