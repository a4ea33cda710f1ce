// Depthwise (groups = channels) dilated conv1d, "same" padding, forward / backward for gfx950.
//
// Replaces nn.Conv1d(C, C, P, padding=(P-1)*dil/2, dilation=dil, groups=C, bias=False) of
// /root/reference/baseline/avse4/model.py:278-285 (DepthwiseSeparableConv, P=3, dil 2^x) and
// model.py:191-198 (VisualConv1D, P=3, dil 1):  y[t] = sum_k w[c,k] x[t + (k - (P-1)/2) * dil].
// One workgroup per (b, c) row; forward: the row streams through LDS in TILE pieces with a (P-1)/2*dil
// halo each side; backward: streaming loads (below); each HBM byte moves once (fwd: 8 B/elem, bwd: 12 B/elem — the SURVEY §8d
// algorithmic bytes).  dW is reduced per row in registers/LDS and summed over the batch by a
// second kernel (deterministic).
#include "common.h"

namespace avse {
namespace dwc {

constexpr int THREADS = 256, PER = 8, TILE = THREADS * PER, MAXP = 7, MAXHALO = 512;

template <int P>
__global__ __launch_bounds__(THREADS) void fwd_kernel(int C, int K, int dil, const float* __restrict__ x,
                                                      const float* __restrict__ w, float* __restrict__ y) {
    __shared__ float s[TILE + 2 * MAXHALO];
    const int row = blockIdx.x, c = row % C;
    const int halo = (P - 1) / 2 * dil;
    const float* xr = x + (int64_t)row * K;
    float* yr = y + (int64_t)row * K;
    float wk[P];
#pragma unroll
    for (int k = 0; k < P; ++k) wk[k] = w[c * P + k];
    for (int t0 = 0; t0 < K; t0 += TILE) {
        __syncthreads();
        for (int i = threadIdx.x; i < TILE + 2 * halo; i += THREADS) {
            const int t = t0 - halo + i;
            s[i] = (t >= 0 && t < K) ? xr[t] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int p = 0; p < PER; ++p) {
            const int i = threadIdx.x + p * THREADS, t = t0 + i;
            if (t < K) {
                float acc = 0.f;
#pragma unroll
                for (int k = 0; k < P; ++k) acc += wk[k] * s[i + k * dil];
                yr[t] = acc;
            }
        }
    }
}

// dx[t] = sum_k w[k] dy[t - (k - h) * dil];  dw[k] += dy[t] * x[t + (k - h) * dil]
// Streaming form, no LDS: thread t-loop over the row, BU elements per thread in flight; the taps' neighbours come
// from the cache lines this workgroup just brought in (buffer loads: outside the row reads 0, no branches), so each
// HBM byte still moves once (tools/avse4 TCN profile: the LDS-tiled form ran at 3.8 TB/s, latency-bound).
template <int P>
__global__ __launch_bounds__(THREADS) void bwd_kernel(int C, int K, int dil, const float* __restrict__ x,
                                                      const float* __restrict__ w, const float* __restrict__ dy,
                                                      float* __restrict__ dx, float* __restrict__ ws) {
    constexpr int BU = 4;
    __shared__ float red[THREADS / 64][MAXP];
    const int row = blockIdx.x, c = row % C;
    const int halo = (P - 1) / 2 * dil;
    const float* xr = x + (int64_t)row * K;
    const float* gr = dy + (int64_t)row * K;
    float* dr = dx + (int64_t)row * K;
    float wk[P], dw[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        wk[k] = w[c * P + k];
        dw[k] = 0.f;
    }
    const auto rx = make_rsrc(xr, K), rg = make_rsrc(gr, K);
    for (int t0 = 0; t0 < K; t0 += BU * THREADS) {
        float acc[BU], g[BU], xv[BU][P];
#pragma unroll
        for (int j = 0; j < BU; ++j) {
            const int t = t0 + j * THREADS + threadIdx.x;
            acc[j] = 0.f;
#pragma unroll
            for (int k = 0; k < P; ++k) {
                const float gk = bufld<float>::ld(rg, t + halo - k * dil, 0);
                acc[j] += wk[k] * gk;
                if (k == (P - 1) / 2) g[j] = gk;
                xv[j][k] = bufld<float>::ld(rx, t + k * dil - halo, 0);
            }
        }
#pragma unroll
        for (int j = 0; j < BU; ++j) {
            const int t = t0 + j * THREADS + threadIdx.x;
            if (t < K) {
                dr[t] = acc[j];
#pragma unroll
                for (int k = 0; k < P; ++k) dw[k] += g[j] * xv[j][k];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        float v = dw[k];
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < P) ws[(int64_t)row * MAXP + threadIdx.x] = red[0][threadIdx.x] + red[1][threadIdx.x] +
                                                                  red[2][threadIdx.x] + red[3][threadIdx.x];
}

__global__ void dw_reduce_kernel(const float* __restrict__ ws, int B, int C, int P, float* __restrict__ dw) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C * P) return;
    const int c = i / P, k = i % P;
    float v = 0.f;
#pragma unroll 16
    for (int b = 0; b < B; ++b) v += ws[((int64_t)b * C + c) * MAXP + k];
    dw[i] = v;
}

}  // namespace dwc
}  // namespace avse

using namespace avse::dwc;

extern "C" {

int64_t avse_dwconv_bwd_workspace_bytes(int64_t B, int64_t C) { return 4 * B * C * MAXP; }

int avse_dwconv_fwd(int64_t B, int64_t C, int64_t K, int64_t P, int64_t dil, const float* x, const float* w, float* y,
                    avse_stream_t stream) {
    if (!x || !w || !y) return AVSE_EINVAL;
    if (B <= 0 || C <= 0 || K <= 0 || dil <= 0 || (P != 1 && P != 3 && P != 5 && P != 7) ||
        (P - 1) / 2 * dil > MAXHALO || B * C > (1LL << 31) - 1)
        return AVSE_ESHAPE;
    hipStream_t st = (hipStream_t)stream;
    dim3 grid((unsigned)(B * C)), block(THREADS);
    switch ((int)P) {
        case 1: hipLaunchKernelGGL(fwd_kernel<1>, grid, block, 0, st, (int)C, (int)K, (int)dil, x, w, y); break;
        case 3: hipLaunchKernelGGL(fwd_kernel<3>, grid, block, 0, st, (int)C, (int)K, (int)dil, x, w, y); break;
        case 5: hipLaunchKernelGGL(fwd_kernel<5>, grid, block, 0, st, (int)C, (int)K, (int)dil, x, w, y); break;
        default: hipLaunchKernelGGL(fwd_kernel<7>, grid, block, 0, st, (int)C, (int)K, (int)dil, x, w, y); break;
    }
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_dwconv_bwd(int64_t B, int64_t C, int64_t K, int64_t P, int64_t dil, const float* x, const float* w,
                    const float* dy, float* dx, float* dw, float* workspace, avse_stream_t stream) {
    if (!x || !w || !dy || !dx || !dw || !workspace) return AVSE_EINVAL;
    if (B <= 0 || C <= 0 || K <= 0 || dil <= 0 || (P != 1 && P != 3 && P != 5 && P != 7) ||
        (P - 1) / 2 * dil > MAXHALO || B * C > (1LL << 31) - 1)
        return AVSE_ESHAPE;
    hipStream_t st = (hipStream_t)stream;
    dim3 grid((unsigned)(B * C)), block(THREADS);
    switch ((int)P) {
        case 1: hipLaunchKernelGGL(bwd_kernel<1>, grid, block, 0, st, (int)C, (int)K, (int)dil, x, w, dy, dx, workspace); break;
        case 3: hipLaunchKernelGGL(bwd_kernel<3>, grid, block, 0, st, (int)C, (int)K, (int)dil, x, w, dy, dx, workspace); break;
        case 5: hipLaunchKernelGGL(bwd_kernel<5>, grid, block, 0, st, (int)C, (int)K, (int)dil, x, w, dy, dx, workspace); break;
        default: hipLaunchKernelGGL(bwd_kernel<7>, grid, block, 0, st, (int)C, (int)K, (int)dil, x, w, dy, dx, workspace); break;
    }
    AVSE_CHECK_LAUNCH();
    const int n = (int)(C * P);
    hipLaunchKernelGGL(dw_reduce_kernel, dim3((n + 255) / 256), dim3(256), 0, st, workspace, (int)B, (int)C, (int)P, dw);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
