// Max pooling over (H, W) planes for gfx950: nn.MaxPool3d((1, KH, KW), (1, SH, SW), (0, PH, PW)) of the lip
// front-ends (/root/reference/baseline/avse1/model.py:29-34 frontend3D; avse4 VisualFrontend, same pooling)
// on (B, C, T, H, W) = B*C*T contiguous planes.  PyTorch's max_pool3d_with_indices kernels took 9 ms forward
// + 2.3 ms backward per avse1 C2 step (profiles/r02_avse1_*) for ~2.5 GB of traffic.
//
// Forward: one thread per output element, the window's first maximum (strict '>'; a NaN is taken, as torch),
// its position in the window stored as one byte.  Backward: one thread per input element gathers dy from the
// (at most ceil(K/S)^2) windows that contain it and chose it -- deterministic, no atomics, every dx written.
#include "common.h"

namespace avse {
namespace maxpool {

constexpr int THREADS = 256;

struct P2 {
    int64_t planes;
    int H, W, Ho, Wo, KH, KW, SH, SW, PH, PW;
};

// I: uint32_t when the element count fits (the index divisions are then 32-bit), else int64_t
template <typename I>
__global__ __launch_bounds__(THREADS) void fwd_kernel(P2 p, const float* __restrict__ x, float* __restrict__ y,
                                                      uint8_t* __restrict__ idx) {
    const I n = (I)(p.planes * p.Ho * p.Wo);
    for (I o = (I)blockIdx.x * THREADS + threadIdx.x; o < n; o += (I)gridDim.x * THREADS) {
        const int wo = (int)(o % (I)p.Wo);
        const I t = o / (I)p.Wo;
        const int ho = (int)(t % (I)p.Ho);
        const int64_t pl = (int64_t)(t / (I)p.Ho);
        const float* xp = x + pl * p.H * p.W;
        const int h0 = ho * p.SH - p.PH, w0 = wo * p.SW - p.PW;
        // torch: maxval = -inf, index = first in-bounds element; take v if v > maxval or v is NaN
        const int kh0 = h0 < 0 ? -h0 : 0, kw0 = w0 < 0 ? -w0 : 0;
        float best = -__builtin_inff();
        int arg = kh0 * p.KW + kw0;
        for (int kh = kh0; kh < p.KH; ++kh) {
            const int h = h0 + kh;
            if (h >= p.H) break;
            for (int kw = kw0; kw < p.KW; ++kw) {
                const int w = w0 + kw;
                if (w >= p.W) break;
                const float v = xp[h * p.W + w];
                if (v > best || v != v) {
                    best = v;
                    arg = kh * p.KW + kw;
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
        const int w = (int)(i % (I)p.W);
        const I t = i / (I)p.W;
        const int h = (int)(t % (I)p.H);
        const int64_t pl = (int64_t)(t / (I)p.H);
        // windows ho with ho*SH - PH <= h <= ho*SH - PH + KH - 1
        const int hh = h + p.PH, ww = w + p.PW;
        const int ho_lo = hh >= p.KH ? (hh - p.KH) / p.SH + 1 : 0, ho_hi = min(p.Ho - 1, hh / p.SH);
        const int wo_lo = ww >= p.KW ? (ww - p.KW) / p.SW + 1 : 0, wo_hi = min(p.Wo - 1, ww / p.SW);
        float g = 0.f;
        const int64_t ob = pl * p.Ho * p.Wo;
        for (int ho = ho_lo; ho <= ho_hi; ++ho)
            for (int wo = wo_lo; wo <= wo_hi; ++wo) {
                const int64_t o = ob + (int64_t)ho * p.Wo + wo;
                const int a = idx[o];
                if (ho * p.SH - p.PH + a / p.KW == h && wo * p.SW - p.PW + a % p.KW == w) g += dy[o];
            }
        dx[i] = g;
    }
}

inline bool make(P2& p, int64_t planes, int64_t H, int64_t W, int64_t KH, int64_t KW, int64_t SH, int64_t SW,
                 int64_t PH, int64_t PW) {
    if (planes <= 0 || H <= 0 || W <= 0 || KH <= 0 || KW <= 0 || SH <= 0 || SW <= 0 || PH < 0 || PW < 0) return false;
    if (KH * KW > 255 || 2 * PH > KH || 2 * PW > KW || H > (1 << 20) || W > (1 << 20)) return false;   // torch: pad <= k/2
    p.planes = planes; p.H = (int)H; p.W = (int)W; p.KH = (int)KH; p.KW = (int)KW;
    p.SH = (int)SH; p.SW = (int)SW; p.PH = (int)PH; p.PW = (int)PW;
    p.Ho = (int)((H + 2 * PH - KH) / SH + 1);
    p.Wo = (int)((W + 2 * PW - KW) / SW + 1);
    return p.Ho > 0 && p.Wo > 0;
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
    // 32-bit index math needs the input count to fit too (the loop's last increment stays below 2^32)
    if (p.planes * p.H * p.W < (1LL << 31))
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
    if (n < (1LL << 31))
        hipLaunchKernelGGL(bwd_kernel<uint32_t>, dim3(blocks_for(n)), dim3(THREADS), 0, (hipStream_t)stream, p, dy, idx, dx);
    else
        hipLaunchKernelGGL(bwd_kernel<int64_t>, dim3(blocks_for(n)), dim3(THREADS), 0, (hipStream_t)stream, p, dy, idx, dx);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
