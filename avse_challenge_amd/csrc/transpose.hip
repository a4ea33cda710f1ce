// Batched 2-D transpose y[n][p][c] = x[n][c][p] (fp32), for the layout changes around the channels-last lip trunk:
// the front-end's (B, C, T, H, W) output -> (B*T, H, W, C) trunk input, and its gradient back
// (avse1 VisualFeatNet.forward; reference model.py:17-58 transposes frames into the batch the same way).
// torch's strided copy moved these 283 MB at ~0.35 TB/s; here a workgroup transposes a 64 x 64 tile through LDS
// (row-coalesced 256-B reads and writes, one padding column against bank conflicts).
#include "common.h"

namespace avse {
namespace tr {

constexpr int T = 64, THREADS = 256;

__global__ __launch_bounds__(THREADS) void transpose_kernel(int64_t C, int64_t P, int tiles_p, int tiles_c,
                                                            const float* __restrict__ x, float* __restrict__ y) {
    __shared__ float tile[T][T + 1];
    const int64_t bid = blockIdx.x;
    const int tp = (int)(bid % tiles_p), tc = (int)((bid / tiles_p) % tiles_c);
    const int64_t n = bid / ((int64_t)tiles_p * tiles_c);
    const int64_t p0 = (int64_t)tp * T, c0 = (int64_t)tc * T;
    const float* xn = x + n * C * P;
    float* yn = y + n * C * P;
    const int lx = threadIdx.x & 63, ly = threadIdx.x >> 6;      // 64 columns x 4 rows per pass
    // unguarded buffer loads, all 16 in flight: rows past C fall outside the resource (read as 0), columns past P read
    // the next row's head, which lands only in tile slots that are never stored
    const auto rx = make_rsrc(xn + c0 * P, (C - c0) * P);
#pragma unroll
    for (int r = 0; r < T; r += 4) tile[r + ly][lx] = bufld<float>::ld(rx, (int)((r + ly) * P + p0 + lx), 0);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < T; r += 4) {
        const int64_t p = p0 + r + ly, c = c0 + lx;
        if (p < P && c < C) yn[p * C + c] = tile[lx][r + ly];
    }
}

}  // namespace tr
}  // namespace avse

extern "C" int avse_transpose_cp(int64_t N, int64_t C, int64_t P, const float* x, float* y, avse_stream_t stream) {
    if (!x || !y) return AVSE_EINVAL;
    if (N <= 0 || C <= 0 || P <= 0) return AVSE_ESHAPE;
    if (P > (1LL << 23)) return AVSE_ESHAPE;          // 32-bit buffer offsets over a 64-row tile
    const int64_t tiles_p = (P + avse::tr::T - 1) / avse::tr::T, tiles_c = (C + avse::tr::T - 1) / avse::tr::T;
    const int64_t blocks = N * tiles_p * tiles_c;
    if (blocks > 0x7FFFFFFFLL || tiles_p > 0x7FFFFFFFLL) return AVSE_ESHAPE;
    hipLaunchKernelGGL(avse::tr::transpose_kernel, dim3((unsigned)blocks), dim3(avse::tr::THREADS), 0,
                       (hipStream_t)stream, C, P, (int)tiles_p, (int)tiles_c, x, y);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}
