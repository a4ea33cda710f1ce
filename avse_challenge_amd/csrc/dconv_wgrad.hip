// Weight gradient of the avse1 AudioFeatNet dilated convolutions for gfx950, as an implicit GEMM on the exact-fp32
// MFMA (v_mfma_f32_32x32x2_f32), channels-last (NHWC) activations.
//
// Replaces the weight-gradient half of nn.Conv2d(64, 64, 5, padding=2d, dilation=d), d = 2, 4, 8, 16 — conv2..conv5 of
// /root/reference/baseline/avse1/model.py:199-215 (AudioFeatNet, built in the loop at :202-209).  MIOpen's pick for
// these shapes (igemm_wrw ... bt64x64, group-k-split) ran them at ~0.34 of the fp32 MFMA peak: 47.9 ms of the 170 ms
// avse1 C2 step (profiles/r02d_avse1_timed_window_stats.csv).
//
//   dW[co][ci][kh][kw] = sum_{n,h,w} dY[n][h][w][co] * X[n][h + d (kh - 2)][w + d (kw - 2)][ci]   (0 outside the image)
//
// Work decomposition: the reduction over the B*H*W pixels is cut into chunks = (image n, output row h, piece of the row
// of <= PX_MAX pixels); workgroup (r, kh) accumulates the 5 kw taps of ONE kernel row kh over a contiguous range r of
// chunks, so the 5 workgroups of a range read the same dY pieces (L2) while each stages only its own input row
// h + d (kh - 2).  Per chunk the dY piece [px][co] and the input-row segment [px - 2d, px + len + 2d)[ci] are staged
// in LDS (pixel-major, 256 B per pixel); wave w computes the 32x32 tile (co block w / 2, ci block w % 2) of all 5 taps:
// per K-step (2 pixels: lanes 0-31 pixel 2j, lanes 32-63 pixel 2j + 1) one A read, 5 B reads (the kw-shifted pixel)
// and 5 MFMAs.  The next chunk's tiles are loaded into registers (float4 buffer loads, out-of-range -> 0) while the
// current chunk's MFMAs run.  Per-workgroup partial sums go to a workspace summed by a second kernel (deterministic).
// The bias gradient db[co] = sum dY[.][co] comes along: the kh = 0 workgroups add up the dY pieces they already hold
// in registers (a fixed 4-channel group per thread), so the avse1 step needs no separate reduction pass over dY.
#include <algorithm>

#include "common.h"

namespace avse {
namespace dcw {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int C = 64, KS = 5, THREADS = 256;
constexpr int PX_MAX = 66;                       // pixels per piece, even (a 257-wide row is 64 + 64 + 64 + 65)
constexpr int MAX_DIL = 16;
constexpr int SEG_MAX = PX_MAX + 4 * MAX_DIL;    // staged input pixels per chunk
constexpr int A_V4 = PX_MAX * C / 4 / THREADS + 1;   // float4 loads per thread: dY piece (5)
constexpr int X_V4 = (SEG_MAX * C / 4 + THREADS - 1) / THREADS;   // input segment (9)

struct Shape {
    int N, H, W, dil;
    int npieces, chunks, ranges;
};

__device__ inline float4 ld4(__amdgpu_buffer_rsrc_t r, int voff_elems) {
    float4 v;
    const auto raw = __builtin_amdgcn_raw_buffer_load_b128(r, voff_elems * 4, 0, 0);
    v.x = __uint_as_float(raw[0]);
    v.y = __uint_as_float(raw[1]);
    v.z = __uint_as_float(raw[2]);
    v.w = __uint_as_float(raw[3]);
    return v;
}

__global__ __launch_bounds__(THREADS, 3) void wgrad_kernel(Shape s, const float* __restrict__ x,
                                                           const float* __restrict__ dy, float* __restrict__ part,
                                                           float* __restrict__ dbpart) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = xcd_remap(blockIdx.x, gridDim.x);      // the 5 kh workgroups of a range share an XCD's L2
    const int r = bid / KS, kh = bid % KS;
    const int d = s.dil, seg_px = PX_MAX + 4 * d;
    float* sa = lds;                                       // [PX_MAX + 2][C]   dY piece
    float* sx = lds + (PX_MAX + 2) * C;                    // [seg_px + 2][C]   input row segment
    const int c_lo = (int)((int64_t)r * s.chunks / s.ranges), c_hi = (int)((int64_t)(r + 1) * s.chunks / s.ranges);
    const int c_lo_u = __builtin_amdgcn_readfirstlane(c_lo), c_hi_u = __builtin_amdgcn_readfirstlane(c_hi);

    const int64_t npix = (int64_t)s.N * s.H * s.W;
    const auto rx = make_rsrc(x, npix * C);
    const auto ry = make_rsrc(dy, npix * C);
    const int OOB = (int)(npix * C);                       // element offset past num_records: the load returns 0

    float4 ar[A_V4], xr[X_V4];
    int cur_len = 0;
    // registers <- chunk c: dY pixels [w0, w0 + len) of row (n, h) and input pixels [w0 - 2d, w0 + len + 2d) of row
    // h + d (kh - 2); everything outside the image (and past len / the segment) loads as 0
    auto prefetch = [&](int c, int& len) {
        const int piece = c % s.npieces, row = c / s.npieces;           // row = n * H + h
        const int h = row % s.H;
        const int w0 = piece * s.W / s.npieces, w1 = (piece + 1) * s.W / s.npieces;     // < 2^31 (checked)
        len = w1 - w0;
        const int ybase = (row * s.W + w0) * C;
        const int t4 = threadIdx.x;                                      // float4 index within the tile
#pragma unroll
        for (int i = 0; i < A_V4; ++i) {
            const int e = (t4 + i * THREADS) * 4, px = e / C;
            ar[i] = ld4(ry, px < len ? ybase + e : OOB);
        }
        const int hi = h + d * (kh - 2);
        const bool rowok = hi >= 0 && hi < s.H;
        const int xrow = (row - h + hi) * s.W;                           // pixel index of (n, hi, 0)
#pragma unroll
        for (int i = 0; i < X_V4; ++i) {
            const int e = (t4 + i * THREADS) * 4, px = e / C, wi = w0 - 2 * d + px;
            const bool ok = rowok && px < len + 4 * d && wi >= 0 && wi < s.W;
            xr[i] = ld4(rx, ok ? (xrow + wi) * C + e % C : OOB);
        }
    };

    floatx16 acc[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[k][q] = 0.f;

    const int co = (wave >> 1) * 32 + (lane & 31), ci = (wave & 1) * 32 + (lane & 31), half = lane >> 5;
    const bool want_db = dbpart != nullptr && kh == 0;     // workgroup-uniform
    float4 dsum = {0.f, 0.f, 0.f, 0.f};                    // channels 4 (tid % 16) .. + 3
    if (c_lo_u < c_hi_u) prefetch(c_lo_u, cur_len);
    for (int c = c_lo_u; c < c_hi_u; ++c) {
        const int len = cur_len;
        __syncthreads();                                   // the previous chunk's MFMAs are done with LDS
#pragma unroll
        for (int i = 0; i < A_V4; ++i) {
            const int e = (threadIdx.x + i * THREADS) * 4;
            if (e < PX_MAX * C) *reinterpret_cast<float4*>(&sa[e]) = ar[i];
        }
        if (want_db) {                                     // pixels past the piece loaded as 0
#pragma unroll
            for (int i = 0; i < A_V4; ++i) {
                dsum.x += ar[i].x; dsum.y += ar[i].y; dsum.z += ar[i].z; dsum.w += ar[i].w;
            }
        }
#pragma unroll
        for (int i = 0; i < X_V4; ++i) {
            const int e = (threadIdx.x + i * THREADS) * 4;
            if (e < seg_px * C) *reinterpret_cast<float4*>(&sx[e]) = xr[i];
        }
        __syncthreads();
        if (c + 1 < c_hi_u) prefetch(c + 1, cur_len);
        const int nk = (len + 1) >> 1;
        // operands of K-step j + 1 are read while the MFMAs of step j issue (the LDS tile has one spare pixel row
        // past each array, so the read after the last step stays inside the allocation; its values are unused)
        const float* pa = sa + half * C + co;
        const float* pb = sx + half * C + ci;
        float a0 = pa[0], b0[KS];
#pragma unroll
        for (int k = 0; k < KS; ++k) b0[k] = pb[k * d * C];
        for (int j = 0; j < nk; ++j) {
            pa += 2 * C;
            pb += 2 * C;
            const float a1 = pa[0];
            float b1[KS];
#pragma unroll
            for (int k = 0; k < KS; ++k) b1[k] = pb[k * d * C];
#pragma unroll
            for (int k = 0; k < KS; ++k) acc[k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0[k], acc[k], 0, 0, 0);
            a0 = a1;
#pragma unroll
            for (int k = 0; k < KS; ++k) b0[k] = b1[k];
        }
    }
    if (want_db) {                                         // 16 threads per channel group -> dbpart[r][co]
        __syncthreads();
        reinterpret_cast<float4*>(lds)[threadIdx.x] = dsum;
        __syncthreads();
        if (threadIdx.x < C) {
            const int g = threadIdx.x >> 2, k = threadIdx.x & 3;
            float v = 0.f;
            for (int t = 0; t < THREADS / 16; ++t) v += lds[(t * 16 + g) * 4 + k];
            dbpart[(int64_t)r * C + threadIdx.x] = v;
        }
    }
    // partial tiles out: part[bid][kw][co][ci]; C map col = lane & 31, row = (q & 3) + 8 (q >> 2) + 4 (lane >> 5)
    float* p = part + ((int64_t)r * KS + kh) * KS * C * C;
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int row_co = (wave >> 1) * 32 + (q & 3) + 8 * (q >> 2) + 4 * half;
            p[((int64_t)k * C + row_co) * C + ci] = acc[k][q];
        }
}

// dW[co][ci][kh][kw] = sum over ranges of part[range][kh][kw][co][ci]; db[co] = sum over ranges of dbpart[range][co]
__global__ void reduce_kernel(const float* __restrict__ part, const float* __restrict__ dbpart, int ranges,
                              float* __restrict__ dw, float* __restrict__ db) {
    constexpr int TOTAL = KS * KS * C * C;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= TOTAL) {
        if (db != nullptr && i < TOTAL + C) {
            float v = 0.f;
            for (int g = 0; g < ranges; ++g) v += dbpart[(int64_t)g * C + i - TOTAL];
            db[i - TOTAL] = v;
        }
        return;
    }
    float v = 0.f;
    for (int g = 0; g < ranges; ++g) v += part[(int64_t)g * TOTAL + i];
    const int ci = i % C, co = (i / C) % C, kw = (i / (C * C)) % KS, kh = i / (KS * C * C);
    dw[((co * C + ci) * KS + kh) * KS + kw] = v;
}

inline size_t lds_bytes(int dil) { return 4 * (size_t)(PX_MAX + 2 + PX_MAX + 4 * dil + 2) * C; }

inline int ranges_for(int dil, int chunks) {
    const int per_cu = std::max(1, std::min(3, (int)((160 * 1024) / lds_bytes(dil))));   // <= 168 VGPRs: 3 waves/SIMD
    return std::max(1, std::min(chunks, 256 * per_cu / KS));
}

}  // namespace dcw
}  // namespace avse

using namespace avse::dcw;

extern "C" {

int64_t avse_dconv_wgrad_workspace_bytes(int64_t N, int64_t H, int64_t W, int64_t dil) {
    const int64_t npieces = (W + PX_MAX - 1) / PX_MAX;
    return 4 * (int64_t)ranges_for((int)dil, (int)(N * H * npieces)) * (KS * KS * C * C + C);
}

int avse_dconv_wgrad(int64_t N, int64_t H, int64_t W, int64_t dil, const float* x, const float* dy, float* dw,
                     float* db, float* workspace, avse_stream_t stream) {
    if (!x || !dy || !dw || !workspace) return AVSE_EINVAL;
    if (N <= 0 || H <= 0 || W <= 0 || dil <= 0 || dil > MAX_DIL) return AVSE_ESHAPE;
    const int64_t npieces = (W + PX_MAX - 1) / PX_MAX;
    if (N * H * W * C >= (1LL << 29)) return AVSE_ESHAPE;                 // 32-bit buffer offsets (bytes < 2 GiB)
    if (N * H * 8 >= (1LL << 31) || 8 * W >= (1LL << 31)) return AVSE_ESHAPE;
    Shape s;
    s.N = (int)N; s.H = (int)H; s.W = (int)W; s.dil = (int)dil;
    s.npieces = (int)npieces;
    s.chunks = (int)(N * H * npieces);
    s.ranges = ranges_for(s.dil, s.chunks);
    hipStream_t st = (hipStream_t)stream;
    constexpr int TOTAL = KS * KS * C * C;
    float* dbpart = db ? workspace + (int64_t)s.ranges * TOTAL : nullptr;
    hipLaunchKernelGGL(wgrad_kernel, dim3(s.ranges * KS), dim3(THREADS), lds_bytes(s.dil), st, s, x, dy, workspace,
                       dbpart);
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL(reduce_kernel, dim3((TOTAL + C + 255) / 256), dim3(256), 0, st, workspace, dbpart, s.ranges,
                       dw, db);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
