// Fused residual-add + RMSNorm forward / backward for gfx950.
//
// Replaces the Block pre-norm of /root/reference/Mamba-TasNet/modules/mamba/bimamba.py:447-451
// (residual = hidden + residual; norm(residual)) with the mamba-ssm Triton RMSNorm
// (x * rsqrt(mean(x^2) + eps) * w, un-vendored) and MambaBlocksSequential.norm_f
// (mamba_blocks.py:195-197).  One wave per row (n <= 1024, n % 4 == 0), float4 accesses,
// the sum of squares reduced in registers with cross-lane adds: one HBM pass each way.
// dweight is reduced per workgroup (grid-stride over rows) and summed by a second kernel.
#include "common.h"

namespace avse {
namespace rms {

constexpr int THREADS = 256;
constexpr int WPB = THREADS / 64;
constexpr int MAXV = 4;  // float4 per lane -> n <= 1024

// 4 consecutive elements of a row as a float4: fp32 (one 16-B access) or bf16 (one 8-B access, widened; stores round to
// nearest even).  bf16 rows (round 6): the C5 Block's mixer output enters and the norm output leaves in the autocast
// dtype, so neither needs a torch cast pass (the reference's fused add_norm returns its input's dtype).
template <typename T> struct v4;
template <> struct v4<float> {
    __device__ static inline float4 ld(const float* p, int c) { return reinterpret_cast<const float4*>(p)[c]; }
    __device__ static inline void st(float* p, int c, float4 v) { reinterpret_cast<float4*>(p)[c] = v; }
};
template <> struct v4<bf16_t> {
    __device__ static inline float4 ld(const bf16_t* p, int c) {
        const uint2 q = reinterpret_cast<const uint2*>(p)[c];
        return make_float4(__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u), __uint_as_float(q.y << 16),
                           __uint_as_float(q.y & 0xffff0000u));
    }
    __device__ static inline void st(bf16_t* p, int c, float4 v) {
        bf16_t h[4];
        io<bf16_t>::st(&h[0], v.x), io<bf16_t>::st(&h[1], v.y), io<bf16_t>::st(&h[2], v.z), io<bf16_t>::st(&h[3], v.w);
        reinterpret_cast<uint2*>(p)[c] = make_uint2((uint32_t)h[0].x | ((uint32_t)h[1].x << 16),
                                                    (uint32_t)h[2].x | ((uint32_t)h[3].x << 16));
    }
};

__device__ inline float wave_sum(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

// the workgroup's max |out| -> one atomicMax on the float bits (non-negative floats order like their bits): the
// producer-side max of an operand the split-fp16 projection GEMMs split next (avse_split16_planes_known).  Per
// workgroup, not per wave: the word's atomics serialise at the memory side (~17 ns each).  Called by every thread.
__device__ inline void block_max_out(float m, uint32_t* omax) {
    __shared__ uint32_t red[WPB];
    uint32_t b = __float_as_uint(m);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) b = max(b, (uint32_t)__shfl_xor((int)b, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int w = 0; w < WPB; ++w) b = max(b, red[w]);
        if (b) atomicMax(omax, b);
    }
}

template <typename TH, typename TY>
__global__ __launch_bounds__(THREADS) void fwd_kernel(int rows, int n, const TH* __restrict__ h,
                                                      const float* __restrict__ res_in, const float* __restrict__ w,
                                                      float eps, TY* __restrict__ y, float* __restrict__ res_out,
                                                      float* __restrict__ rstd_out, uint32_t* __restrict__ ymax) {
    const int lane = threadIdx.x & 63;
    const int nv = n / 4;
    float m = 0.f;
    for (int row = blockIdx.x * WPB + (threadIdx.x >> 6); row < rows; row += gridDim.x * WPB) {
        const TH* hr = h + (int64_t)row * n;
        const float4* rr = res_in ? reinterpret_cast<const float4*>(res_in + (int64_t)row * n) : nullptr;
        float4 v[MAXV];
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < MAXV; ++i) {
            const int c = lane + i * 64;
            if (c < nv) {
                float4 a = v4<TH>::ld(hr, c);
                if (rr) {
                    const float4 r = rr[c];
                    a.x += r.x; a.y += r.y; a.z += r.z; a.w += r.w;
                }
                v[i] = a;
                ss += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
            }
        }
        ss = wave_sum(ss);
        const float rs = rsqrtf(ss / n + eps);
        TY* yr = y + (int64_t)row * n;
        float4* ro = reinterpret_cast<float4*>(res_out + (int64_t)row * n);
        const float4* wv = reinterpret_cast<const float4*>(w);
#pragma unroll
        for (int i = 0; i < MAXV; ++i) {
            const int c = lane + i * 64;
            if (c < nv) {
                const float4 ww = wv[c];
                const float4 a = v[i];
                ro[c] = a;
                const float4 o = make_float4(a.x * rs * ww.x, a.y * rs * ww.y, a.z * rs * ww.z, a.w * rs * ww.w);
                v4<TY>::st(yr, c, o);
                m = fmaxf(m, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
            }
        }
        if (lane == 0) rstd_out[row] = rs;
    }
    if (ymax) block_max_out(m, ymax);                      // wave-uniform condition
}

// dx = rstd * (dy*w - xhat * mean(dy*w*xhat)) + dres_out ; dw_partial = sum_rows dy * xhat
template <typename TD>
__global__ __launch_bounds__(THREADS) void bwd_kernel(int rows, int n, const TD* __restrict__ dy,
                                                      const float* __restrict__ dres, const float* __restrict__ x,
                                                      const float* __restrict__ w, const float* __restrict__ rstd,
                                                      float* __restrict__ dx, float* __restrict__ ws,
                                                      uint32_t* __restrict__ dxmax) {
    __shared__ float4 sdw[WPB][256];
    float m = 0.f;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nv = n / 4;
    float4 dwacc[MAXV];
#pragma unroll
    for (int i = 0; i < MAXV; ++i) dwacc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4* wv = reinterpret_cast<const float4*>(w);
    for (int row = blockIdx.x * WPB + wid; row < rows; row += gridDim.x * WPB) {
        const TD* dyr = dy + (int64_t)row * n;
        const float4* xr = reinterpret_cast<const float4*>(x + (int64_t)row * n);
        const float rs = rstd[row];
        float4 g[MAXV], xh[MAXV];
        float dot = 0.f;
#pragma unroll
        for (int i = 0; i < MAXV; ++i) {
            const int c = lane + i * 64;
            if (c < nv) {
                const float4 a = xr[c], d = v4<TD>::ld(dyr, c), ww = wv[c];
                xh[i] = make_float4(a.x * rs, a.y * rs, a.z * rs, a.w * rs);
                g[i] = make_float4(d.x * ww.x, d.y * ww.y, d.z * ww.z, d.w * ww.w);
                dot += g[i].x * xh[i].x + g[i].y * xh[i].y + g[i].z * xh[i].z + g[i].w * xh[i].w;
                dwacc[i].x += d.x * xh[i].x; dwacc[i].y += d.y * xh[i].y;
                dwacc[i].z += d.z * xh[i].z; dwacc[i].w += d.w * xh[i].w;
            }
        }
        dot = wave_sum(dot) / n;
        float4* dxr = reinterpret_cast<float4*>(dx + (int64_t)row * n);
        const float4* drr = dres ? reinterpret_cast<const float4*>(dres + (int64_t)row * n) : nullptr;
#pragma unroll
        for (int i = 0; i < MAXV; ++i) {
            const int c = lane + i * 64;
            if (c < nv) {
                float4 o = make_float4(rs * (g[i].x - xh[i].x * dot), rs * (g[i].y - xh[i].y * dot),
                                       rs * (g[i].z - xh[i].z * dot), rs * (g[i].w - xh[i].w * dot));
                if (drr) {
                    const float4 r = drr[c];
                    o.x += r.x; o.y += r.y; o.z += r.z; o.w += r.w;
                }
                dxr[c] = o;
                m = fmaxf(m, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
            }
        }
    }
    if (dxmax) block_max_out(m, dxmax);                    // wave-uniform condition
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
        const int c = lane + i * 64;
        if (c < nv) sdw[wid][c] = dwacc[i];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < nv; c += THREADS) {
        float4 s = sdw[0][c];
        for (int k = 1; k < WPB; ++k) {
            const float4 t = sdw[k][c];
            s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
        }
        reinterpret_cast<float4*>(ws + (int64_t)blockIdx.x * n)[c] = s;
    }
}

// dweight = sum of the per-workgroup partials: 64 channels per workgroup (lane = channel, coalesced),
// 16 row groups striding over the partials, then a fixed LDS tree (deterministic)
__global__ __launch_bounds__(1024) void reduce_kernel(const float* ws, int nblocks, int n, float* dw) {
    __shared__ float red[16][65];
    const int c = blockIdx.x * 64 + threadIdx.x, gy = threadIdx.y;
    float v = 0.f;
    if (c < n)
        for (int b = gy; b < nblocks; b += 16) v += ws[(int64_t)b * n + c];
    red[gy][threadIdx.x] = v;
    __syncthreads();
    if (gy == 0 && c < n) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) t += red[i][threadIdx.x];
        dw[c] = t;
    }
}

inline int nblocks_for(int64_t rows) {
    int64_t nb = (rows + WPB - 1) / WPB;
    return (int)(nb < 1024 ? nb : 1024);
}

}  // namespace rms
}  // namespace avse

using namespace avse::rms;

extern "C" {

int avse_add_rmsnorm_fwd2(int64_t rows, int64_t n, const void* h, int32_t h_dtype, const float* res_in,
                          const float* weight, float eps, void* y, int32_t y_dtype, float* res_out, float* rstd,
                          uint32_t* y_max, avse_stream_t stream) {
    if (!h || !weight || !y || !res_out || !rstd) return AVSE_EINVAL;
    if (rows <= 0 || n <= 0 || n % 4 || n > 64 * 4 * MAXV || rows > (1LL << 31) - 1) return AVSE_ESHAPE;
    if ((h_dtype != AVSE_F32 && h_dtype != AVSE_BF16) || (y_dtype != AVSE_F32 && y_dtype != AVSE_BF16)) return AVSE_EDTYPE;
    if (y_max && hipMemsetAsync(y_max, 0, 4, (hipStream_t)stream) != hipSuccess) return AVSE_ELAUNCH;
    const dim3 g(nblocks_for(rows)), b(THREADS);
    hipStream_t st = (hipStream_t)stream;
#define AVSE_RMS_FWD(TH, TY) \
    hipLaunchKernelGGL((fwd_kernel<TH, TY>), g, b, 0, st, (int)rows, (int)n, (const TH*)h, res_in, weight, eps, (TY*)y, \
                       res_out, rstd, y_max)
    if (h_dtype == AVSE_F32 && y_dtype == AVSE_F32) AVSE_RMS_FWD(float, float);
    else if (h_dtype == AVSE_F32) AVSE_RMS_FWD(float, avse::bf16_t);
    else if (y_dtype == AVSE_F32) AVSE_RMS_FWD(avse::bf16_t, float);
    else AVSE_RMS_FWD(avse::bf16_t, avse::bf16_t);
#undef AVSE_RMS_FWD
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_add_rmsnorm_fwd(int64_t rows, int64_t n, const float* h, const float* res_in, const float* weight, float eps,
                         float* y, float* res_out, float* rstd, uint32_t* y_max, avse_stream_t stream) {
    return avse_add_rmsnorm_fwd2(rows, n, h, AVSE_F32, res_in, weight, eps, y, AVSE_F32, res_out, rstd, y_max, stream);
}

int64_t avse_rmsnorm_bwd_workspace_bytes(int64_t rows, int64_t n) { return 4 * (int64_t)nblocks_for(rows) * n; }

int avse_rmsnorm_bwd2(int64_t rows, int64_t n, const void* dy, int32_t dy_dtype, const float* dres_out,
                      const float* res_out, const float* weight, const float* rstd, float* dx, float* dweight,
                      float* workspace, uint32_t* dx_max, avse_stream_t stream) {
    if (!dy || !res_out || !weight || !rstd || !dx || !dweight || !workspace) return AVSE_EINVAL;
    if (rows <= 0 || n <= 0 || n % 4 || n > 64 * 4 * MAXV || rows > (1LL << 31) - 1) return AVSE_ESHAPE;
    if (dy_dtype != AVSE_F32 && dy_dtype != AVSE_BF16) return AVSE_EDTYPE;
    const int nb = nblocks_for(rows);
    hipStream_t st = (hipStream_t)stream;
    if (dx_max && hipMemsetAsync(dx_max, 0, 4, st) != hipSuccess) return AVSE_ELAUNCH;
    if (dy_dtype == AVSE_F32)
        hipLaunchKernelGGL(bwd_kernel<float>, dim3(nb), dim3(THREADS), 0, st, (int)rows, (int)n, (const float*)dy,
                           dres_out, res_out, weight, rstd, dx, workspace, dx_max);
    else
        hipLaunchKernelGGL(bwd_kernel<avse::bf16_t>, dim3(nb), dim3(THREADS), 0, st, (int)rows, (int)n,
                           (const avse::bf16_t*)dy, dres_out, res_out, weight, rstd, dx, workspace, dx_max);
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL(reduce_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64, 16), 0, st, workspace, nb, (int)n,
                       dweight);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_rmsnorm_bwd(int64_t rows, int64_t n, const float* dy, const float* dres_out, const float* res_out,
                     const float* weight, const float* rstd, float* dx, float* dweight, float* workspace,
                     uint32_t* dx_max, avse_stream_t stream) {
    return avse_rmsnorm_bwd2(rows, n, dy, AVSE_F32, dres_out, res_out, weight, rstd, dx, dweight, workspace, dx_max,
                             stream);
}

}  // extern "C"
