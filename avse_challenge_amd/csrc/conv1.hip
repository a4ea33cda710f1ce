// AudioFeatNet.conv1 = nn.Conv2d(1, 64, 5, padding=2) (/root/reference/baseline/avse1/model.py:199-215, the first conv
// of the loop at :202-209) on the (B, 1, 376, 257) spectrogram, for gfx950: forward, input gradient and weight / bias
// gradient as direct HBM-streaming kernels.
//
//   y[n][h][w][o] = b[o] + sum_{kh,kw} x[n][h + kh - 2][w + kw - 2] W[o][kh][kw]          (NHWC output, 0 outside)
//   dx[n][h][w]   = sum_{kh,kw} e[n][h + 2 - kh][w + 2 - kw][kh kw],  e[p][t] = sum_o dy[p][o] W[o][t]
//   dW[o][t]      = sum_p dy[p][o] x[p + t - 2],  db[o] = sum_p dy[p][o]
//
// 1600 FMAs per pixel against 256 B of NHWC output / gradient per pixel: all three are bound by streaming y / dy
// (791 MB per call at avse1 C2), not by arithmetic.  Previously im2col GEMMs (a (B H W, 26) row matrix, K = 26 and
// K = B H W library GEMMs, 25 shifted plane adds for dx): several ms per step of memory-inefficient passes.
//   forward: thread = one output pixel, the 25-tap window from an LDS tile of the workgroup's input rows, the weights
//     wave-uniform (scalar loads), 64 accumulators, 16 float4 stores of the pixel's 256 B;
//   input gradient: workgroup = 8 x 32 output pixels of one image; e of the 12 x 36 pixels around them (the 2-pixel
//     halo) into LDS (thread = pixel: 16 float4 loads of dy, 1600 FMAs), then dx = 25 LDS reads per pixel;
//   weight gradient: lane = output channel (a wave reads a pixel's 256 B of dy), the pixel's 25 taps wave-uniform from
//     an LDS tile, 26 accumulators per lane over the workgroup's rows; per-workgroup partials, a fixed-order reduce.
#include <algorithm>

#include "common.h"

namespace avse {
namespace cv1 {

constexpr int CO = 64, KS = 5, TAPS = 25, PAD = 2;

// ------------------------------------------------------------------------------------------------ forward
// workgroup = 256 consecutive raster pixels of one image (up to 3 rows when W >= 128); LDS: the rows they read
constexpr int FT = 256;
constexpr int FROWS = 3 + 4;                   // output rows a tile spans (W >= 128) + the 4 halo rows
constexpr int FCOLS_MAX = 1024 + 4;

__global__ __launch_bounds__(FT) void fwd_kernel(int N, int H, int W, int tiles, const float* __restrict__ x,
                                                 const float* __restrict__ w, const float* __restrict__ b,
                                                 float* __restrict__ y) {
    extern __shared__ float xs[];              // [FROWS][W + 4]
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int n = bid / tiles, tile = bid % tiles;
    const int HW = H * W, WP = W + 4;
    const int p0 = tile * FT, r0 = p0 / W;
    const int nrows = min((min(p0 + FT, HW) - 1) / W - r0 + 1 + 4, FROWS);
    const float* xn = x + (int64_t)n * HW;
    for (int i = threadIdx.x; i < nrows * WP; i += FT) {
        const int rr = i / WP, cc = i % WP;
        const int hi = r0 + rr - PAD, wi = cc - PAD;
        xs[i] = (hi >= 0 && hi < H && wi >= 0 && wi < W) ? xn[hi * W + wi] : 0.f;
    }
    __syncthreads();
    const int p = p0 + (int)threadIdx.x;
    if (p >= HW) return;
    const int h = p / W, wc = p % W;
    float xv[TAPS];
#pragma unroll
    for (int kh = 0; kh < KS; ++kh)
#pragma unroll
        for (int kw = 0; kw < KS; ++kw) xv[kh * KS + kw] = xs[(h - r0 + kh) * WP + wc + kw];
    float* yp = y + ((int64_t)n * HW + p) * CO;
#pragma unroll
    for (int o4 = 0; o4 < CO / 4; ++o4) {
        float acc[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int o = 4 * o4 + k;
            float a = b ? b[o] : 0.f;
#pragma unroll
            for (int t = 0; t < TAPS; ++t) a = fmaf(xv[t], w[o * TAPS + t], a);      // w, b: wave-uniform loads
            acc[k] = a;
        }
        *reinterpret_cast<float4*>(yp + 4 * o4) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    }
}

// ------------------------------------------------------------------------------------------------ input gradient
// workgroup = DR x CW output pixels of one image; e over the (DR + 4) x (CW + 4) pixels around them in LDS
constexpr int DT = 256, DR = 8, CW = 32;
constexpr int ER = DR + 4, EC = CW + 4;

__global__ __launch_bounds__(DT) void dgrad_kernel(int N, int H, int W, int rblocks, int cblocks,
                                                   const float* __restrict__ dy, const float* __restrict__ w,
                                                   float* __restrict__ dx) {
    __shared__ float es[ER * EC * TAPS];       // 43 KB; pixel-major, stride 25 words (distinct banks per lane)
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int cb = bid % cblocks, rb = (bid / cblocks) % rblocks, n = bid / (cblocks * rblocks);
    const int h0 = rb * DR, c0 = cb * CW;
    for (int i = threadIdx.x; i < ER * EC; i += DT) {
        const int rr = i / EC, cc = i % EC;
        const int hh = h0 - PAD + rr, ww = c0 - PAD + cc;
        float e[TAPS];
#pragma unroll
        for (int t = 0; t < TAPS; ++t) e[t] = 0.f;
        if (hh >= 0 && hh < H && ww >= 0 && ww < W) {
            const float4* g = reinterpret_cast<const float4*>(dy + (((int64_t)n * H + hh) * W + ww) * CO);
#pragma unroll
            for (int o4 = 0; o4 < CO / 4; ++o4) {
                const float4 v = g[o4];
                const float gv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int t = 0; t < TAPS; ++t) e[t] = fmaf(gv[k], w[(4 * o4 + k) * TAPS + t], e[t]);
            }
        }
#pragma unroll
        for (int t = 0; t < TAPS; ++t) es[i * TAPS + t] = e[t];
    }
    __syncthreads();
    // dx[h][c] = sum_{kh,kw} e[h + 2 - kh][c + 2 - kw][kh kw]: e tile row r + 4 - kh, column cc + 4 - kw
    for (int i = threadIdx.x; i < DR * CW; i += DT) {
        const int r = i / CW, cc = i % CW, h = h0 + r, c = c0 + cc;
        if (h >= H || c >= W) continue;
        float s = 0.f;
#pragma unroll
        for (int kh = 0; kh < KS; ++kh)
#pragma unroll
            for (int kw = 0; kw < KS; ++kw) s += es[((r + 4 - kh) * EC + cc + 4 - kw) * TAPS + kh * KS + kw];
        dx[((int64_t)n * H + h) * W + c] = s;
    }
}

// ------------------------------------------------------------------------------------------------ weight gradient
constexpr int WT = 256, WROWS = 4;             // threads; image rows per workgroup

// a bounded grid of workgroups, each looping over row blocks (N H / WROWS of them) with its accumulators in registers:
// few partials to reduce (3008 per-row-block partials summed serially took 1.6 ms at avse1 C2)
__global__ __launch_bounds__(WT) void wgrad_kernel(int N, int H, int W, int rblocks, const float* __restrict__ x,
                                                   const float* __restrict__ dy, float* __restrict__ part) {
    extern __shared__ float xs[];              // [WROWS + 4][W + 4]
    const int WP = W + 4, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float acc[TAPS + 1];
#pragma unroll
    for (int t = 0; t <= TAPS; ++t) acc[t] = 0.f;
    for (int rb = blockIdx.x; rb < N * rblocks; rb += gridDim.x) {
        const int n = rb / rblocks, h0 = (rb % rblocks) * WROWS;
        const float* xn = x + (int64_t)n * H * W;
        __syncthreads();                       // the previous row block's tile reads are done
        for (int i = threadIdx.x; i < (WROWS + 4) * WP; i += WT) {
            const int rr = i / WP, cc = i % WP;
            const int hi = h0 - PAD + rr, wi = cc - PAD;
            xs[i] = (hi >= 0 && hi < H && wi >= 0 && wi < W) ? xn[hi * W + wi] : 0.f;
        }
        __syncthreads();
        // lane = output channel; wave w takes the pixels w, w + 4, ... of the row block
        const int np = min(WROWS, H - h0) * W;
        for (int i = wave; i < np; i += WT / 64) {
            const int r = i / W, c = i % W;
            const float g = dy[(((int64_t)n * H + h0 + r) * W + c) * CO + lane];
#pragma unroll
            for (int kh = 0; kh < KS; ++kh)
#pragma unroll
                for (int kw = 0; kw < KS; ++kw) acc[kh * KS + kw] = fmaf(g, xs[(r + kh) * WP + c + kw], acc[kh * KS + kw]);
            acc[TAPS] += g;
        }
    }
    const int bid = blockIdx.x;
    // the 4 waves' partials through LDS (after every wave has finished reading the x tile)
    __syncthreads();
    float* red = xs;                           // [4][26][64]
#pragma unroll
    for (int t = 0; t <= TAPS; ++t) red[(wave * (TAPS + 1) + t) * CO + lane] = acc[t];
    __syncthreads();
    for (int i = threadIdx.x; i < (TAPS + 1) * CO; i += WT)
        part[(int64_t)bid * (TAPS + 1) * CO + i] = red[i] + red[(TAPS + 1) * CO + i] + red[2 * (TAPS + 1) * CO + i] +
                                                   red[3 * (TAPS + 1) * CO + i];
}

// dW[o][t] (= W's (64, 1, 5, 5) layout), db[o]: sum of the workgroups' partials [blk][t][o]; one workgroup per
// output, its threads over the partials, then a fixed tree (deterministic)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int blocks,
                                                           float* __restrict__ dw, float* __restrict__ db) {
    __shared__ float red[4];
    const int i = blockIdx.x;                                   // i = t * 64 + o
    float s = 0.f;
    for (int k = threadIdx.x; k < blocks; k += 256) s += part[(int64_t)k * (TAPS + 1) * CO + i];
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        s = (red[0] + red[1]) + (red[2] + red[3]);
        const int t = i / CO, o = i % CO;
        if (t < TAPS) dw[o * TAPS + t] = s;
        else if (db) db[o] = s;
    }
}

}  // namespace cv1
}  // namespace avse

using namespace avse::cv1;

extern "C" {

int avse_conv1_fwd(int64_t N, int64_t H, int64_t W, const float* x, const float* w, const float* b, float* y,
                   avse_stream_t stream) {
    if (!x || !w || !y) return AVSE_EINVAL;
    if (N <= 0 || H <= 0 || W < 128 || W > FCOLS_MAX - 4 || N * H * W * CO >= (1LL << 40)) return AVSE_ESHAPE;
    if ((uintptr_t)y & 15) return AVSE_EALIGN;
    const int tiles = (int)((H * W + FT - 1) / FT);
    const size_t lds = (size_t)FROWS * (W + 4) * 4;
    hipLaunchKernelGGL(fwd_kernel, dim3((unsigned)(N * tiles)), dim3(FT), lds, (hipStream_t)stream, (int)N, (int)H,
                       (int)W, tiles, x, w, b, y);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_conv1_dgrad(int64_t N, int64_t H, int64_t W, const float* dy, const float* w, float* dx, avse_stream_t stream) {
    if (!dy || !w || !dx) return AVSE_EINVAL;
    if (N <= 0 || H <= 0 || W <= 0) return AVSE_ESHAPE;
    if ((uintptr_t)dy & 15) return AVSE_EALIGN;
    const int rblocks = (int)((H + DR - 1) / DR), cblocks = (int)((W + CW - 1) / CW);
    const int64_t blocks = N * rblocks * cblocks;
    if (blocks >= (1LL << 31)) return AVSE_ESHAPE;
    hipLaunchKernelGGL(dgrad_kernel, dim3((unsigned)blocks), dim3(DT), 0, (hipStream_t)stream, (int)N, (int)H, (int)W,
                       rblocks, cblocks, dy, w, dx);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

constexpr int WG_GRID = 512;

int64_t avse_conv1_wgrad_workspace_bytes(int64_t N, int64_t H, int64_t W) {
    (void)W;
    return std::min<int64_t>(N * ((H + WROWS - 1) / WROWS), WG_GRID) * (TAPS + 1) * CO * 4;
}

int avse_conv1_wgrad(int64_t N, int64_t H, int64_t W, const float* x, const float* dy, float* dw, float* db,
                     float* workspace, avse_stream_t stream) {
    if (!x || !dy || !dw || !workspace) return AVSE_EINVAL;
    if (N <= 0 || H <= 0 || W <= 0 || W > 4096) return AVSE_ESHAPE;
    const int rblocks = (int)((H + WROWS - 1) / WROWS);
    if (N * rblocks >= (1LL << 31)) return AVSE_ESHAPE;
    const int64_t blocks = std::min<int64_t>(N * rblocks, WG_GRID);
    // LDS: the x tile, reused for the 4 x 26 x 64 wave partials
    const size_t lds = std::max<size_t>((size_t)(WROWS + 4) * (W + 4), (size_t)4 * (TAPS + 1) * CO) * 4;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(wgrad_kernel, dim3((unsigned)blocks), dim3(WT), lds, st, (int)N, (int)H, (int)W, rblocks, x, dy,
                       workspace);
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((TAPS + 1) * CO), dim3(256), 0, st, workspace, (int)blocks, dw, db);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
