// PReLU forward / backward (per-channel or single slope) for gfx950.
//
// Replaces nn.PReLU in the avse1 lip stream (frontend3D / ResNet BasicBlock / TCN:
// /root/reference/baseline/avse1/model.py:29-34, utils/resnet.py:45-46, utils/tcn.py:170-196)
// and the avse4 TCN (baseline/avse4/model.py:260,282).  torch's prelu_backward is a
// TensorIterator two-output reduction that took 2 ms on average and 20.9 ms on the
// (32,64,75,48,48) front-end activation (rocprofv3, profiles/).  Here: one workgroup per
// (n, c) row of the (N, C, S) view, float4 streaming, the slope gradient reduced in registers /
// LDS per row and summed over n by a second tiny kernel (deterministic).  HBM-bound:
// fwd 8 B/elem, bwd 12 B/elem.
#include <algorithm>

#include "common.h"

namespace avse {
namespace prelu {

constexpr int THREADS = 256;

__global__ __launch_bounds__(THREADS) void fwd_kernel(int C, int64_t S, int per_channel, const float* __restrict__ x,
                                                      const float* __restrict__ a, float* __restrict__ y) {
    const int64_t row = blockIdx.x;
    const float av = a[per_channel ? (int)(row % C) : 0];
    const float* xr = x + row * S;
    float* yr = y + row * S;
    if ((S & 3) == 0) {
        const float4* x4 = reinterpret_cast<const float4*>(xr);
        float4* y4 = reinterpret_cast<float4*>(yr);
        for (int64_t i = threadIdx.x; i < S / 4; i += THREADS) {
            float4 v = x4[i];
            v.x = v.x > 0.f ? v.x : av * v.x;
            v.y = v.y > 0.f ? v.y : av * v.y;
            v.z = v.z > 0.f ? v.z : av * v.z;
            v.w = v.w > 0.f ? v.w : av * v.w;
            y4[i] = v;
        }
    } else {
        for (int64_t i = threadIdx.x; i < S; i += THREADS) {
            const float v = xr[i];
            yr[i] = v > 0.f ? v : av * v;
        }
    }
}

__global__ __launch_bounds__(THREADS) void bwd_kernel(int C, int64_t S, int per_channel, const float* __restrict__ x,
                                                      const float* __restrict__ a, const float* __restrict__ dy,
                                                      float* __restrict__ dx, float* __restrict__ ws) {
    __shared__ float red[THREADS / 64];
    const int64_t row = blockIdx.x;
    const float av = a[per_channel ? (int)(row % C) : 0];
    const float* xr = x + row * S;
    const float* gr = dy + row * S;
    float* dr = dx + row * S;
    float da = 0.f;
    if ((S & 3) == 0) {
        const float4* x4 = reinterpret_cast<const float4*>(xr);
        const float4* g4 = reinterpret_cast<const float4*>(gr);
        float4* d4 = reinterpret_cast<float4*>(dr);
        for (int64_t i = threadIdx.x; i < S / 4; i += THREADS) {
            const float4 v = x4[i], g = g4[i];
            float4 o;
            o.x = v.x > 0.f ? g.x : av * g.x; da += v.x > 0.f ? 0.f : g.x * v.x;
            o.y = v.y > 0.f ? g.y : av * g.y; da += v.y > 0.f ? 0.f : g.y * v.y;
            o.z = v.z > 0.f ? g.z : av * g.z; da += v.z > 0.f ? 0.f : g.z * v.z;
            o.w = v.w > 0.f ? g.w : av * g.w; da += v.w > 0.f ? 0.f : g.w * v.w;
            d4[i] = o;
        }
    } else {
        for (int64_t i = threadIdx.x; i < S; i += THREADS) {
            const float v = xr[i], g = gr[i];
            dr[i] = v > 0.f ? g : av * g;
            da += v > 0.f ? 0.f : g * v;
        }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) da += __shfl_xor(da, m, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = da;
    __syncthreads();
    if (threadIdx.x == 0) ws[row] = red[0] + red[1] + red[2] + red[3];
}

// da[c] = sum_n ws[n*C + c]  (per_channel) or sum over all rows (single slope)
__global__ void reduce_kernel(const float* __restrict__ ws, int64_t N, int C, int per_channel, float* __restrict__ da) {
    __shared__ float red[256 / 64];
    const int c = blockIdx.x;
    float v = 0.f;
    if (per_channel) {
        for (int64_t n = threadIdx.x; n < N; n += blockDim.x) v += ws[n * C + c];
    } else {
        for (int64_t i = threadIdx.x; i < N * C; i += blockDim.x) v += ws[i];
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) da[c] = red[0] + red[1] + red[2] + red[3];
}

// ---- channels-last (NHWC) layout: an (R, C) row-major view, C % 4 == 0, slope index = column.
// The avse1 lip ResNet runs channels-last (MIOpen's NHWC convolutions); the NCS kernels above would
// launch one 256-thread workgroup per 9-element (n, c) row at layer4 (3x3 maps).

__global__ __launch_bounds__(THREADS) void nhwc_fwd_kernel(int64_t n4, int C4, int per_channel,
                                                           const float4* __restrict__ x, const float* __restrict__ a,
                                                           float4* __restrict__ y) {
    const float a0 = a[0];
    for (int64_t f = (int64_t)blockIdx.x * THREADS + threadIdx.x; f < n4; f += (int64_t)gridDim.x * THREADS) {
        const float4 av = per_channel ? reinterpret_cast<const float4*>(a)[f % C4] : make_float4(a0, a0, a0, a0);
        float4 v = x[f];
        v.x = v.x > 0.f ? v.x : av.x * v.x;
        v.y = v.y > 0.f ? v.y : av.y * v.y;
        v.z = v.z > 0.f ? v.z : av.z * v.z;
        v.w = v.w > 0.f ? v.w : av.w * v.w;
        y[f] = v;
    }
}

// thread = (row offset, 4-channel group): RPI = 256 / C4 rows per workgroup pass, the group fixed for the
// whole grid-stride loop, so the slope-gradient partial stays in registers; the workgroup's RPI partials per
// group are summed in LDS and written as one C-wide row of ws (summed over workgroups by nhwc_reduce_kernel)
__global__ __launch_bounds__(THREADS) void nhwc_bwd_kernel(int64_t R, int C4, int per_channel,
                                                           const float4* __restrict__ x, const float* __restrict__ a,
                                                           const float4* __restrict__ dy, float4* __restrict__ dx,
                                                           float* __restrict__ ws) {
    __shared__ float4 part[THREADS];
    const int RPI = THREADS / C4;
    const int cg = threadIdx.x % C4, roff = threadIdx.x / C4;
    const float a0 = a[0];
    const float4 av = per_channel ? reinterpret_cast<const float4*>(a)[cg] : make_float4(a0, a0, a0, a0);
    float4 da = make_float4(0.f, 0.f, 0.f, 0.f);
    if (roff < RPI) {
        for (int64_t r = (int64_t)blockIdx.x * RPI + roff; r < R; r += (int64_t)gridDim.x * RPI) {
            const int64_t f = r * C4 + cg;
            const float4 v = x[f], g = dy[f];
            float4 o;
            o.x = v.x > 0.f ? g.x : av.x * g.x; da.x += v.x > 0.f ? 0.f : g.x * v.x;
            o.y = v.y > 0.f ? g.y : av.y * g.y; da.y += v.y > 0.f ? 0.f : g.y * v.y;
            o.z = v.z > 0.f ? g.z : av.z * g.z; da.z += v.z > 0.f ? 0.f : g.z * v.z;
            o.w = v.w > 0.f ? g.w : av.w * g.w; da.w += v.w > 0.f ? 0.f : g.w * v.w;
            dx[f] = o;
        }
    }
    part[threadIdx.x] = da;
    __syncthreads();
    if (roff == 0) {
        float4 s = da;
        for (int k = 1; k < RPI; ++k) {
            const float4 q = part[k * C4 + cg];
            s.x += q.x; s.y += q.y; s.z += q.z; s.w += q.w;
        }
        reinterpret_cast<float4*>(ws + (int64_t)blockIdx.x * 4 * C4)[cg] = s;
    }
}

// da[c] = sum_w ws[w * C + c] (per channel) or the sum of everything (single slope).  Per channel: workgroup g takes
// channels 64 g .. 64 g + 63, its 4 waves the partial rows w = wave (mod 4), 8 independent loads in flight per lane
// (a serial loop over the 1024 rows was 1024 dependent L2 round trips: ~1.4 ms per call for the avse1 TCN's
// (2400, 512) PReLU); the 4 wave sums are added in a fixed order (deterministic).  Single slope: one workgroup, the
// same 8 loads in flight per lane, then a fixed-order block sum.
__global__ void nhwc_reduce_kernel(const float* __restrict__ ws, int nblk, int C, int per_channel, float* __restrict__ da) {
    constexpr int U = 8;
    __shared__ float red[4][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (per_channel) {
        const int c = blockIdx.x * 64 + lane;
        const bool ok = c < C;
        float acc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = 0.f;
        for (int w0 = wv; w0 < nblk; w0 += 4 * U) {
            float v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int w = w0 + 4 * u;
                v[u] = (ok && w < nblk) ? ws[(int64_t)w * C + c] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] += v[u];
        }
        float sum = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) sum += acc[u];
        red[wv][lane] = sum;
        __syncthreads();
        if (wv == 0 && ok) da[c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
        return;
    }
    const int64_t n = (int64_t)nblk * C;
    float acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = 0.f;
    for (int64_t i0 = threadIdx.x; i0 < n; i0 += (int64_t)U * blockDim.x) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + (int64_t)u * blockDim.x;
            v[u] = i < n ? ws[i] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] += v[u];
    }
    float v = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) v += acc[u];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    if (lane == 0) red[wv][0] = v;
    __syncthreads();
    if (threadIdx.x == 0) da[0] = red[0][0] + red[1][0] + red[2][0] + red[3][0];
}

inline bool nhwc_ok(int64_t R, int64_t C) {
    return R > 0 && C > 0 && C % 4 == 0 && C / 4 <= THREADS && THREADS % (C / 4) == 0 && R * C < (1LL << 40);
}
inline int nhwc_bwd_blocks(int64_t R, int64_t C) {
    const int64_t rpi = THREADS / (C / 4);
    return (int)std::min<int64_t>(1024, (R + rpi - 1) / rpi);
}

}  // namespace prelu
}  // namespace avse

using namespace avse::prelu;

extern "C" {

int avse_prelu_fwd(int64_t N, int64_t C, int64_t S, int32_t num_params, const float* x, const float* a, float* y,
                   avse_stream_t stream) {
    if (!x || !a || !y) return AVSE_EINVAL;
    if (N <= 0 || C <= 0 || S <= 0 || (num_params != 1 && num_params != C) || N * C > (1LL << 31) - 1) return AVSE_ESHAPE;
    if (((uintptr_t)x | (uintptr_t)y) & 15) return AVSE_EALIGN;
    hipLaunchKernelGGL(fwd_kernel, dim3((unsigned)(N * C)), dim3(THREADS), 0, (hipStream_t)stream, (int)C, S,
                       (int)(num_params > 1), x, a, y);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int64_t avse_prelu_bwd_workspace_bytes(int64_t N, int64_t C) { return 4 * N * C; }

int avse_prelu_bwd(int64_t N, int64_t C, int64_t S, int32_t num_params, const float* x, const float* a, const float* dy,
                   float* dx, float* da, float* workspace, avse_stream_t stream) {
    if (!x || !a || !dy || !dx || !da || !workspace) return AVSE_EINVAL;
    if (N <= 0 || C <= 0 || S <= 0 || (num_params != 1 && num_params != C) || N * C > (1LL << 31) - 1) return AVSE_ESHAPE;
    if (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx) & 15) return AVSE_EALIGN;
    hipStream_t st = (hipStream_t)stream;
    const int pc = num_params > 1;
    hipLaunchKernelGGL(bwd_kernel, dim3((unsigned)(N * C)), dim3(THREADS), 0, st, (int)C, S, pc, x, a, dy, dx, workspace);
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL(reduce_kernel, dim3(pc ? (unsigned)C : 1u), dim3(256), 0, st, workspace, N, (int)C, pc, da);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_prelu_nhwc_fwd(int64_t R, int64_t C, int32_t num_params, const float* x, const float* a, float* y,
                        avse_stream_t stream) {
    if (!x || !a || !y) return AVSE_EINVAL;
    if (!nhwc_ok(R, C) || (num_params != 1 && num_params != C)) return AVSE_ESHAPE;
    if (((uintptr_t)x | (uintptr_t)y | (num_params > 1 ? (uintptr_t)a : 0)) & 15) return AVSE_EALIGN;
    const int64_t n4 = R * C / 4;
    const int blocks = (int)std::min<int64_t>(8192, (n4 + THREADS - 1) / THREADS);
    hipLaunchKernelGGL(nhwc_fwd_kernel, dim3(blocks), dim3(THREADS), 0, (hipStream_t)stream, n4, (int)(C / 4),
                       (int)(num_params > 1), reinterpret_cast<const float4*>(x), a, reinterpret_cast<float4*>(y));
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int64_t avse_prelu_nhwc_bwd_workspace_bytes(int64_t R, int64_t C) {
    return nhwc_ok(R, C) ? 4 * (int64_t)nhwc_bwd_blocks(R, C) * C : 0;
}

int avse_prelu_nhwc_bwd(int64_t R, int64_t C, int32_t num_params, const float* x, const float* a, const float* dy,
                        float* dx, float* da, float* workspace, avse_stream_t stream) {
    if (!x || !a || !dy || !dx || !da || !workspace) return AVSE_EINVAL;
    if (!nhwc_ok(R, C) || (num_params != 1 && num_params != C)) return AVSE_ESHAPE;
    if (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx | (uintptr_t)workspace | (num_params > 1 ? (uintptr_t)a : 0)) & 15)
        return AVSE_EALIGN;
    hipStream_t st = (hipStream_t)stream;
    const int nblk = nhwc_bwd_blocks(R, C), pc = num_params > 1;
    hipLaunchKernelGGL(nhwc_bwd_kernel, dim3(nblk), dim3(THREADS), 0, st, R, (int)(C / 4), pc,
                       reinterpret_cast<const float4*>(x), a, reinterpret_cast<const float4*>(dy),
                       reinterpret_cast<float4*>(dx), workspace);
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL(nhwc_reduce_kernel, dim3(pc ? (unsigned)((C + 63) / 64) : 1u), dim3(256), 0, st, workspace, nblk,
                       (int)C, pc, da);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
