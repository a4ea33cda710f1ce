// Max pooling over (H, W) planes for gfx950: nn.MaxPool3d((1, KH, KW), (1, SH, SW), (0, PH, PW)) of the lip
// front-ends (/root/reference/baseline/avse1/model.py:29-34 frontend3D; avse4 VisualFrontend, same pooling)
// on (B, C, T, H, W) = B*C*T contiguous planes.  PyTorch's max_pool3d_with_indices kernels took 9 ms forward
// + 2.3 ms backward per avse1 C2 step (profiles/r02_avse1_*) for ~2.5 GB of traffic.
//
// Forward: one thread per output element, the window's first maximum (strict '>'; a NaN is taken, as torch),
// its position in the window stored as one byte (kh << 4 | kw).  Backward: one thread per input element gathers dy from the
// (at most ceil(K/S)^2) windows that contain it and chose it -- deterministic, no atomics, every dx written.
#include "common.h"

namespace avse {
namespace maxpool {

constexpr int THREADS = 256;

// n / d for a runtime-invariant d by multiply-high (Granlund-Montgomery round-up): exact for every 32-bit n.
// The plane / row / column decompositions are the only per-element integer work: hardware-less 32-bit division
// by a runtime value costs ~25 VALU instructions, which made the gather backward VALU-bound (2.4 ms, 0.10 HBM).
struct FastDiv {
    uint32_t d, m, s;
    void init(uint32_t dv) {
        d = dv;
        s = 0;
        while ((1ull << s) < dv) ++s;
        m = (uint32_t)(((1ull << 32) * ((1ull << s) - dv)) / dv + 1);
    }
    __device__ inline uint32_t div(uint32_t n) const { return (uint32_t)(((uint64_t)__umulhi(n, m) + n) >> s); }
};

struct P2 {
    int64_t planes;
    int H, W, Ho, Wo, KH, KW, SH, SW, PH, PW;
    FastDiv fW, fH, fWo, fHo, fSH, fSW;
};

// I: uint32_t when the element count fits (the index divisions are then 32-bit), else int64_t
template <typename I>
__global__ __launch_bounds__(THREADS) void fwd_kernel(P2 p, const float* __restrict__ x, float* __restrict__ y,
                                                      uint8_t* __restrict__ idx) {
    const I n = (I)(p.planes * p.Ho * p.Wo);
    for (I o = (I)blockIdx.x * THREADS + threadIdx.x; o < n; o += (I)gridDim.x * THREADS) {
        int wo, ho;
        int64_t pl;
        if constexpr (sizeof(I) == 4) {
            const uint32_t t = p.fWo.div(o), q = p.fHo.div(t);
            wo = (int)(o - t * p.Wo);
            ho = (int)(t - q * p.Ho);
            pl = q;
        } else {
            wo = (int)(o % p.Wo);
            const I t = o / p.Wo;
            ho = (int)(t % p.Ho);
            pl = t / p.Ho;
        }
        const float* xp = x + pl * p.H * p.W;
        const int h0 = ho * p.SH - p.PH, w0 = wo * p.SW - p.PW;
        // torch: maxval = -inf, index = first in-bounds element; take v if v > maxval or v is NaN
        const int kh0 = h0 < 0 ? -h0 : 0, kw0 = w0 < 0 ? -w0 : 0;
        float best = -__builtin_inff();
        int arg = (kh0 << 4) | kw0;                 // (kh, kw) packed in one byte: KH, KW <= 15
        for (int kh = kh0; kh < p.KH; ++kh) {
            const int h = h0 + kh;
            if (h >= p.H) break;
            for (int kw = kw0; kw < p.KW; ++kw) {
                const int w = w0 + kw;
                if (w >= p.W) break;
                const float v = xp[h * p.W + w];
                if (v > best || v != v) {
                    best = v;
                    arg = (kh << 4) | kw;
                }
            }
        }
        y[o] = best;
        idx[o] = (uint8_t)arg;
    }
}

template <typename I>
__global__ __launch_bounds__(THREADS) void bwd_kernel(P2 p, const float* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                      float* __restrict__ dx) {
    const I n = (I)(p.planes * p.H * p.W);
    for (I i = (I)blockIdx.x * THREADS + threadIdx.x; i < n; i += (I)gridDim.x * THREADS) {
        int w, h;
        int64_t pl;
        if constexpr (sizeof(I) == 4) {
            const uint32_t t = p.fW.div(i), q = p.fH.div(t);
            w = (int)(i - t * p.W);
            h = (int)(t - q * p.H);
            pl = q;
        } else {
            w = (int)(i % p.W);
            const I t = i / p.W;
            h = (int)(t % p.H);
            pl = t / p.H;
        }
        // windows ho with ho*SH - PH <= h <= ho*SH - PH + KH - 1
        const int hh = h + p.PH, ww = w + p.PW;
        const int ho_lo = hh >= p.KH ? (int)p.fSH.div(hh - p.KH) + 1 : 0, ho_hi = min(p.Ho - 1, (int)p.fSH.div(hh));
        const int wo_lo = ww >= p.KW ? (int)p.fSW.div(ww - p.KW) + 1 : 0, wo_hi = min(p.Wo - 1, (int)p.fSW.div(ww));
        float g = 0.f;
        const int64_t ob = pl * p.Ho * p.Wo;
        for (int ho = ho_lo; ho <= ho_hi; ++ho)
            for (int wo = wo_lo; wo <= wo_hi; ++wo) {
                const int64_t o = ob + (int64_t)ho * p.Wo + wo;
                const int a = idx[o];
                if (ho * p.SH - p.PH + (a >> 4) == h && wo * p.SW - p.PW + (a & 15) == w) g += dy[o];
            }
        dx[i] = g;
    }
}

// Forward of the same pooling when W % 4 == 0: one thread makes two horizontally adjacent outputs (2wp, 2wp + 1),
// whose windows span input columns 4wp - 1 .. 4wp + 3 of three rows: per row one float4 (4wp .. 4wp + 3) and one
// scalar (4wp - 1) instead of 6 scalar loads; y as float2, the two argmax bytes as one 16-bit store.  The scan order
// and the comparison (first maximum, a NaN taken) are the generic kernel's, so y and idx are bit-identical to it.
__global__ __launch_bounds__(THREADS) void fwd_k3s2p1_w4_kernel(P2 p, FastDiv fPb, FastDiv fHo, uint32_t n_pair,
                                                                const float* __restrict__ x, float* __restrict__ y,
                                                                uint8_t* __restrict__ idx) {
    const int Pb = p.Wo >> 1;
    for (uint32_t i = blockIdx.x * THREADS + threadIdx.x; i < n_pair; i += gridDim.x * THREADS) {
        const uint32_t t = fPb.div(i), q = fHo.div(t);
        const int wp = (int)(i - t * Pb), ho = (int)(t - q * p.Ho);
        const float* xp = x + (int64_t)q * p.H * p.W + 4 * wp;
        float v[3][5];
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            const int h = 2 * ho - 1 + kh;
            const bool ok = h >= 0 && h < p.H;
            const float4 c = ok ? *reinterpret_cast<const float4*>(xp + (int64_t)h * p.W) : make_float4(0.f, 0.f, 0.f, 0.f);
            v[kh][0] = (ok && wp > 0) ? xp[(int64_t)h * p.W - 1] : 0.f;
            v[kh][1] = c.x; v[kh][2] = c.y; v[kh][3] = c.z; v[kh][4] = c.w;
        }
        const int kh0 = ho == 0 ? 1 : 0;
        const int hmax = min(3, p.H - (2 * ho - 1));          // rows past the input's end
        float best[2];
        int arg[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int kw0 = (wp == 0 && j == 0) ? 1 : 0;
            best[j] = -__builtin_inff();
            arg[j] = (kh0 << 4) | kw0;
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) {
                if (kh < kh0 || kh >= hmax) continue;
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) {
                    if (kw < kw0) continue;
                    const float e = v[kh][2 * j + kw];
                    if (e > best[j] || e != e) {
                        best[j] = e;
                        arg[j] = (kh << 4) | kw;
                    }
                }
            }
        }
        const int64_t o = (int64_t)q * p.Ho * p.Wo + (int64_t)ho * p.Wo + 2 * wp;
        *reinterpret_cast<float2*>(y + o) = make_float2(best[0], best[1]);
        *reinterpret_cast<uint16_t*>(idx + o) = (uint16_t)(arg[0] | (arg[1] << 8));
    }
}

// Backward of the lip front-ends' pooling, kernel 3, stride 2, pad 1 (both (H, W) dims): input row h is covered by
// windows ho in {h/2, h/2 + 1} when h is odd and by ho = h/2 alone when it is even, so one thread owns the 2x2 input
// block (2m .. 2m+1, 2n .. 2n+1) and reads the 4 candidate windows (m | m+1, n | n+1) once each: 4 dy + 4 argmax
// byte loads per 4 dx (the generic gather loads up to 4 of each per dx element), float2 row stores.  The per-element
// sums run over the windows in the generic kernel's (ho, wo) order, so dx is bit-identical to it.
template <bool EVEN_W>
__global__ __launch_bounds__(THREADS) void bwd_k3s2p1_kernel(P2 p, FastDiv fNb, FastDiv fMb, uint32_t n_blk,
                                                             const float* __restrict__ dy,
                                                             const uint8_t* __restrict__ idx, float* __restrict__ dx) {
    const int Mb = (p.H + 1) >> 1, Nb = (p.W + 1) >> 1;
    for (uint32_t i = blockIdx.x * THREADS + threadIdx.x; i < n_blk; i += gridDim.x * THREADS) {
        const uint32_t t = fNb.div(i), q = fMb.div(t);
        const int n = (int)(i - t * Nb), m = (int)(t - q * Mb);
        const int64_t ob = (int64_t)q * p.Ho * p.Wo;
        float g[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) {
            const int ho = m + dh;
            if (ho >= p.Ho) break;
#pragma unroll
            for (int dw = 0; dw < 2; ++dw) {
                const int wo = n + dw;
                if (wo >= p.Wo) break;
                const int64_t o = ob + (int64_t)ho * p.Wo + wo;
                const int a = idx[o];
                const int di = 2 * dh - 1 + (a >> 4), dj = 2 * dw - 1 + (a & 15);   // target - (2m, 2n)
                const float v = dy[o];
                if (di == 0 && dj == 0) g[0][0] += v;
                if (di == 0 && dj == 1) g[0][1] += v;
                if (di == 1 && dj == 0) g[1][0] += v;
                if (di == 1 && dj == 1) g[1][1] += v;
            }
        }
        float* xp = dx + (int64_t)q * p.H * p.W + (int64_t)(2 * m) * p.W + 2 * n;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            if (2 * m + r >= p.H) break;
            if (EVEN_W) {
                *reinterpret_cast<float2*>(xp + r * p.W) = make_float2(g[r][0], g[r][1]);
            } else {
                xp[r * p.W] = g[r][0];
                if (2 * n + 1 < p.W) xp[r * p.W + 1] = g[r][1];
            }
        }
    }
}

inline bool make(P2& p, int64_t planes, int64_t H, int64_t W, int64_t KH, int64_t KW, int64_t SH, int64_t SW,
                 int64_t PH, int64_t PW) {
    if (planes <= 0 || H <= 0 || W <= 0 || KH <= 0 || KW <= 0 || SH <= 0 || SW <= 0 || PH < 0 || PW < 0) return false;
    if (KH > 15 || KW > 15 || 2 * PH > KH || 2 * PW > KW || H > (1 << 20) || W > (1 << 20)) return false;  // pad <= k/2
    p.planes = planes; p.H = (int)H; p.W = (int)W; p.KH = (int)KH; p.KW = (int)KW;
    p.SH = (int)SH; p.SW = (int)SW; p.PH = (int)PH; p.PW = (int)PW;
    p.Ho = (int)((H + 2 * PH - KH) / SH + 1);
    p.Wo = (int)((W + 2 * PW - KW) / SW + 1);
    if (p.Ho <= 0 || p.Wo <= 0) return false;
    p.fW.init((uint32_t)p.W); p.fH.init((uint32_t)p.H); p.fWo.init((uint32_t)p.Wo); p.fHo.init((uint32_t)p.Ho);
    p.fSH.init((uint32_t)p.SH); p.fSW.init((uint32_t)p.SW);
    return true;
}

inline unsigned blocks_for(int64_t n) {
    const int64_t b = (n + THREADS - 1) / THREADS;
    return (unsigned)(b < 65536 ? b : 65536);
}

}  // namespace maxpool
}  // namespace avse

using namespace avse::maxpool;

extern "C" {

int64_t avse_maxpool2d_out_size(int64_t H, int64_t K, int64_t S, int64_t P) { return (H + 2 * P - K) / S + 1; }

int avse_maxpool2d_fwd(int64_t planes, int64_t H, int64_t W, int64_t KH, int64_t KW, int64_t SH, int64_t SW, int64_t PH,
                       int64_t PW, const float* x, float* y, uint8_t* idx, avse_stream_t stream) {
    if (!x || !y || !idx) return AVSE_EINVAL;
    P2 p;
    if (!make(p, planes, H, W, KH, KW, SH, SW, PH, PW)) return AVSE_ESHAPE;
    const int64_t n = p.planes * p.Ho * p.Wo;
    const bool k3s2p1 = p.KH == 3 && p.KW == 3 && p.SH == 2 && p.SW == 2 && p.PH == 1 && p.PW == 1;
    if (k3s2p1 && p.W % 4 == 0 && p.planes * p.H * p.W < (1LL << 31) && ((uintptr_t)x & 15) == 0 &&
        ((uintptr_t)y & 7) == 0 && ((uintptr_t)idx & 1) == 0) {
        FastDiv fPb, fHo;
        fPb.init((uint32_t)(p.Wo / 2));
        fHo.init((uint32_t)p.Ho);
        const int64_t np = n / 2;
        hipLaunchKernelGGL(fwd_k3s2p1_w4_kernel, dim3(blocks_for(np)), dim3(THREADS), 0, (hipStream_t)stream, p, fPb,
                           fHo, (uint32_t)np, x, y, idx);
    } else if (p.planes * p.H * p.W < (1LL << 31))   // 32-bit index math needs the input count to fit too
        hipLaunchKernelGGL(fwd_kernel<uint32_t>, dim3(blocks_for(n)), dim3(THREADS), 0, (hipStream_t)stream, p, x, y, idx);
    else
        hipLaunchKernelGGL(fwd_kernel<int64_t>, dim3(blocks_for(n)), dim3(THREADS), 0, (hipStream_t)stream, p, x, y, idx);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_maxpool2d_bwd(int64_t planes, int64_t H, int64_t W, int64_t KH, int64_t KW, int64_t SH, int64_t SW, int64_t PH,
                       int64_t PW, const float* dy, const uint8_t* idx, float* dx, avse_stream_t stream) {
    if (!dy || !idx || !dx) return AVSE_EINVAL;
    P2 p;
    if (!make(p, planes, H, W, KH, KW, SH, SW, PH, PW)) return AVSE_ESHAPE;
    const int64_t n = p.planes * p.H * p.W;
    const bool k3s2p1 = p.KH == 3 && p.KW == 3 && p.SH == 2 && p.SW == 2 && p.PH == 1 && p.PW == 1;
    const int64_t nb = p.planes * ((p.H + 1) / 2) * ((p.W + 1) / 2);
    if (k3s2p1 && n < (1LL << 31) && ((uintptr_t)dx & 7) == 0) {
        FastDiv fNb, fMb;
        fNb.init((uint32_t)((p.W + 1) / 2));
        fMb.init((uint32_t)((p.H + 1) / 2));
        if (p.W % 2 == 0)
            hipLaunchKernelGGL(bwd_k3s2p1_kernel<true>, dim3(blocks_for(nb)), dim3(THREADS), 0, (hipStream_t)stream, p,
                               fNb, fMb, (uint32_t)nb, dy, idx, dx);
        else
            hipLaunchKernelGGL(bwd_k3s2p1_kernel<false>, dim3(blocks_for(nb)), dim3(THREADS), 0, (hipStream_t)stream, p,
                               fNb, fMb, (uint32_t)nb, dy, idx, dx);
    } else if (n < (1LL << 31))
        hipLaunchKernelGGL(bwd_kernel<uint32_t>, dim3(blocks_for(n)), dim3(THREADS), 0, (hipStream_t)stream, p, dy, idx, dx);
    else
        hipLaunchKernelGGL(bwd_kernel<int64_t>, dim3(blocks_for(n)), dim3(THREADS), 0, (hipStream_t)stream, p, dy, idx, dx);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
