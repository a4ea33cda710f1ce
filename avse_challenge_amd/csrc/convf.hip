// AudioFeatNet.convf = nn.Conv2d(64, 4, 1) (/root/reference/baseline/avse1/model.py:211-213, the 1x1 conv after the
// dilated stack, called at :246-249) on the (B, 64, 376, 257) channels-last activations, for gfx950: forward, input
// gradient and weight / bias gradient as HBM-streaming kernels (MIOpen ran them as implicit GEMMs with N = 4 plus
// its own zero-fills of the outputs: ~1.1 ms of kernel time per avse1 C2 step).
//
//   y[p][o]  = b[o] + sum_c W[o][c] x[p][c]          (p = pixel of the NHWC raster, c < 64, o < 4)
//   dx[p][c] = sum_o W[o][c] dy[p][o]
//   dW[o][c] = sum_p dy[p][o] x[p][c],  db[o] = sum_p dy[p][o]
//
// Each moves the 256 B per pixel of x (or dx) once: 791 MB per call at C2, the HBM roofline.  Lane layout: 16 lanes
// per pixel, lane q holding channels 4q .. 4q + 3 (one float4), so a wave-instruction reads or writes 4 whole pixels
// = 1 KB contiguous; the 4 output channels of a pixel are reduced over its 16 lanes with xor-shuffles.  The weight
// gradient keeps 16 + 4 partial sums per lane over a grid-stride loop, reduces them over the pixel groups of the wave
// and the waves of the workgroup, writes one partial row per workgroup, and a second kernel sums the rows in a fixed
// order (deterministic).
#include <algorithm>

#include "common.h"

namespace avse {
namespace cvf {

constexpr int CI = 64, CO = 4, THREADS = 256, WAVES = THREADS / 64, UNROLL = 4;
constexpr int PARTS = CO * CI + CO;                 // one workgroup's partial row: dW then db

__device__ inline float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__device__ inline float xsum16(float v) {           // sum over the lane's 16-lane group
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    return v;
}

__global__ __launch_bounds__(THREADS) void fwd_kernel(int64_t npix, const float* __restrict__ x,
                                                      const float* __restrict__ w, const float* __restrict__ b,
                                                      float* __restrict__ y) {
    const int lane = threadIdx.x & 63, q = lane & 15;
    float wr[CO][4];
#pragma unroll
    for (int o = 0; o < CO; ++o) {
        const float4 v = ld4(w + o * CI + 4 * q);
        wr[o][0] = v.x, wr[o][1] = v.y, wr[o][2] = v.z, wr[o][3] = v.w;
    }
    float bias = 0.f;
    if (b != nullptr && q < CO) bias = b[q];
    const int64_t step = (int64_t)gridDim.x * THREADS / 16;
    int64_t p = ((int64_t)blockIdx.x * THREADS + threadIdx.x) / 16;
    for (; p < npix; p += UNROLL * step) {
        float4 xv[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int64_t pu = p + u * step;
            xv[u] = pu < npix ? ld4(x + pu * CI + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            float s[CO];
#pragma unroll
            for (int o = 0; o < CO; ++o)
                s[o] = xsum16(wr[o][0] * xv[u].x + wr[o][1] * xv[u].y + wr[o][2] * xv[u].z + wr[o][3] * xv[u].w);
            const int64_t pu = p + u * step;
            if (q < CO && pu < npix) {
                const float v = q == 0 ? s[0] : q == 1 ? s[1] : q == 2 ? s[2] : s[3];
                y[pu * CO + q] = v + bias;
            }
        }
    }
}

__global__ __launch_bounds__(THREADS) void dgrad_kernel(int64_t npix, const float* __restrict__ dy,
                                                        const float* __restrict__ w, float* __restrict__ dx) {
    const int lane = threadIdx.x & 63, q = lane & 15;
    float wr[CO][4];
#pragma unroll
    for (int o = 0; o < CO; ++o) {
        const float4 v = ld4(w + o * CI + 4 * q);
        wr[o][0] = v.x, wr[o][1] = v.y, wr[o][2] = v.z, wr[o][3] = v.w;
    }
    const int64_t step = (int64_t)gridDim.x * THREADS / 16;
    int64_t p = ((int64_t)blockIdx.x * THREADS + threadIdx.x) / 16;
    for (; p < npix; p += UNROLL * step) {
        float4 g[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int64_t pu = p + u * step;
            g[u] = pu < npix ? ld4(dy + pu * CO) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int64_t pu = p + u * step;
            if (pu < npix) {
                float4 r;
                r.x = wr[0][0] * g[u].x + wr[1][0] * g[u].y + wr[2][0] * g[u].z + wr[3][0] * g[u].w;
                r.y = wr[0][1] * g[u].x + wr[1][1] * g[u].y + wr[2][1] * g[u].z + wr[3][1] * g[u].w;
                r.z = wr[0][2] * g[u].x + wr[1][2] * g[u].y + wr[2][2] * g[u].z + wr[3][2] * g[u].w;
                r.w = wr[0][3] * g[u].x + wr[1][3] * g[u].y + wr[2][3] * g[u].z + wr[3][3] * g[u].w;
                *reinterpret_cast<float4*>(dx + pu * CI + 4 * q) = r;
            }
        }
    }
}

__global__ __launch_bounds__(THREADS) void wgrad_kernel(int64_t npix, const float* __restrict__ x,
                                                        const float* __restrict__ dy, float* __restrict__ part) {
    __shared__ float red[WAVES][PARTS];
    const int lane = threadIdx.x & 63, q = lane & 15, wave = threadIdx.x >> 6;
    float acc[CO][4], dbs[CO];
#pragma unroll
    for (int o = 0; o < CO; ++o) {
        dbs[o] = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[o][j] = 0.f;
    }
    const int64_t step = (int64_t)gridDim.x * THREADS / 16;
    int64_t p = ((int64_t)blockIdx.x * THREADS + threadIdx.x) / 16;
    for (; p < npix; p += UNROLL * step) {
        float4 xv[UNROLL], g[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int64_t pu = p + u * step;
            const bool ok = pu < npix;
            xv[u] = ok ? ld4(x + pu * CI + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
            g[u] = ok ? ld4(dy + pu * CO) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const float gv[CO] = {g[u].x, g[u].y, g[u].z, g[u].w};
#pragma unroll
            for (int o = 0; o < CO; ++o) {
                acc[o][0] += gv[o] * xv[u].x;
                acc[o][1] += gv[o] * xv[u].y;
                acc[o][2] += gv[o] * xv[u].z;
                acc[o][3] += gv[o] * xv[u].w;
                dbs[o] += gv[o];
            }
        }
    }
    // the wave's 4 pixel groups hold the same channels: lanes q, q + 16, q + 32, q + 48
#pragma unroll
    for (int o = 0; o < CO; ++o) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float v = acc[o][j];
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            acc[o][j] = v;
        }
        float v = dbs[o];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        dbs[o] = v;
    }
    if (lane < 16) {
#pragma unroll
        for (int o = 0; o < CO; ++o)
#pragma unroll
            for (int j = 0; j < 4; ++j) red[wave][o * CI + 4 * q + j] = acc[o][j];
        if (q == 0)
#pragma unroll
            for (int o = 0; o < CO; ++o) red[wave][CO * CI + o] = dbs[o];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < PARTS; i += THREADS)
        part[(int64_t)blockIdx.x * PARTS + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
}

// dW (4, 64) and db (4) = the sum of the workgroups' partial rows: workgroup = 64 consecutive elements x 4 row slices
// (coalesced 256-B reads), the slices combined in a fixed order (deterministic)
__global__ __launch_bounds__(THREADS) void wgrad_reduce_kernel(const float* __restrict__ part, int rows,
                                                               float* __restrict__ dw, float* __restrict__ db) {
    __shared__ float red[WAVES][64];
    const int i = blockIdx.x * 64 + (threadIdx.x & 63), sl = threadIdx.x >> 6;
    float s = 0.f;
    if (i < PARTS)
        for (int r = sl; r < rows; r += WAVES) s += part[(int64_t)r * PARTS + i];
    red[sl][threadIdx.x & 63] = s;
    __syncthreads();
    if (sl == 0 && i < PARTS) {
        s = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
        if (i < CO * CI) dw[i] = s;
        else if (db != nullptr) db[i - CO * CI] = s;
    }
}

inline int grid_for(int64_t npix) {
    // 16 lanes per pixel, UNROLL pixels per lane and iteration: enough workgroups to fill 256 CUs several times over
    const int64_t want = (npix * 16 + (int64_t)THREADS * UNROLL - 1) / ((int64_t)THREADS * UNROLL);
    return (int)std::max<int64_t>(1, std::min<int64_t>(want, 4096));
}
constexpr int WG_BLOCKS = 1024;

}  // namespace cvf
}  // namespace avse

using namespace avse::cvf;

extern "C" {

int avse_convf_fwd(int64_t npix, const float* x, const float* w, const float* b, float* y, avse_stream_t stream) {
    if (!x || !w || !y) return AVSE_EINVAL;
    if (npix <= 0 || npix >= (1LL << 40)) return AVSE_ESHAPE;
    if (((uintptr_t)x | (uintptr_t)w) % 16) return AVSE_EINVAL;
    hipLaunchKernelGGL(fwd_kernel, dim3(grid_for(npix)), dim3(THREADS), 0, (hipStream_t)stream, npix, x, w, b, y);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_convf_dgrad(int64_t npix, const float* dy, const float* w, float* dx, avse_stream_t stream) {
    if (!dy || !w || !dx) return AVSE_EINVAL;
    if (npix <= 0 || npix >= (1LL << 40)) return AVSE_ESHAPE;
    if (((uintptr_t)dy | (uintptr_t)w | (uintptr_t)dx) % 16) return AVSE_EINVAL;
    hipLaunchKernelGGL(dgrad_kernel, dim3(grid_for(npix)), dim3(THREADS), 0, (hipStream_t)stream, npix, dy, w, dx);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int64_t avse_convf_wgrad_workspace_bytes(int64_t npix) {
    if (npix <= 0) return -1;
    return (int64_t)WG_BLOCKS * PARTS * 4;
}

int avse_convf_wgrad(int64_t npix, const float* x, const float* dy, float* dw, float* db, float* workspace,
                     avse_stream_t stream) {
    if (!x || !dy || !dw || !workspace) return AVSE_EINVAL;
    if (npix <= 0 || npix >= (1LL << 40)) return AVSE_ESHAPE;
    if (((uintptr_t)x | (uintptr_t)dy) % 16) return AVSE_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(wgrad_kernel, dim3(WG_BLOCKS), dim3(THREADS), 0, st, npix, x, dy, workspace);
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((PARTS + 63) / 64), dim3(THREADS), 0, st, workspace, WG_BLOCKS, dw, db);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
