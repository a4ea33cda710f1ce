// Weight gradient of the lip front-end Conv3d (Cout 64, small Cin, kernel (KT,KH,KW), stride (1,2,2))
// for gfx950, as an implicit GEMM on the exact-fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the weight-gradient half of nn.Conv3d(3, 64, (5,7,7), stride (1,2,2), pad (2,3,3))
// in /root/reference/baseline/avse1/model.py:29-34 (frontend3D; avse4 utils.py:100-106 is the
// Cin=1 variant).  MIOpen's immediate-mode pick for this shape launched 12 workgroups and took
// 814 ms per call on MI355X (rocprofv3, profiles/); this kernel spreads the 5.5M-long reduction
// over every CU.
//
//   dW[co][n] = sum_k dY[k][co] * Xcol[k][n],  n = ((ci*KT + kt)*KH + kh)*KW + kw,
//   k = (b, t, ho, wo),  Xcol[k][n] = X[b][ci][t - PT + kt][2*ho - PH + kh][2*wo - PW + kw] (0 outside)
//
// One workgroup (4 waves) owns a strided set of output rows (b, t, ho); per row it stages the
// CIN*KT*KH input rows it touches (width 2*(WO-1)+KW) and the 64 x WO gradient row in LDS, then
// every wave runs WO/2 K-steps of 2 x NTW 32x32x2 MFMAs (M = 64 = 2 tiles, N split over waves).
// Partial 64 x N tiles per workgroup go to a workspace; a second kernel sums them (deterministic).
#include "common.h"

namespace avse {
namespace c3w {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int COUT = 64, THREADS = 256, MAX_WO = 64, WIN_MAX = 2 * (MAX_WO - 1) + 8;
constexpr int YS = MAX_WO + 1;      // dY LDS row stride (bank spread for the 32-row A reads)

struct Shape {
    int B, CIN, T, H, W;            // input
    int TO, HO, WO;                 // output
    int KT, KH, KW, PT, PH, PW;
    int N, rows, nparts;
};

template <int NTW>
__global__ __launch_bounds__(THREADS) void wgrad_kernel(Shape s, const float* __restrict__ x, const float* __restrict__ dy,
                                                        float* __restrict__ part) {
    extern __shared__ float lds[];
    const int WIN = 2 * (s.WO - 1) + s.KW;
    const int WINP = WIN + 1;
    const int nxrow = s.CIN * s.KT * s.KH;
    float* xs = lds;                                  // [nxrow][WINP] + zero pad region
    float* zero = xs + nxrow * WINP;                  // 2 * MAX_WO floats of zeros (N padding)
    float* ys = zero + 2 * MAX_WO + 8;                // [64][YS]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 2 * MAX_WO + 8; i += THREADS) zero[i] = 0.f;

    // per-lane B-operand base offsets for this wave's N tiles
    int boff[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int n = (wave * NTW + j) * 32 + (lane & 31);
        if (n < s.N) {
            const int kw = n % s.KW, r = n / s.KW;     // r = (ci*KT + kt)*KH + kh
            boff[j] = r * WINP + kw;
        } else {
            boff[j] = (int)(zero - xs);               // reads 0 (2*k stays inside the zero block)
        }
    }
    floatx16 acc[2][NTW];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][j][r] = 0.f;

    const int64_t plane = (int64_t)s.H * s.W;
    const int64_t yplane = (int64_t)s.HO * s.WO;
    for (int row = blockIdx.x; row < s.rows; row += gridDim.x) {
        const int ho = row % s.HO;
        const int t = (row / s.HO) % s.TO;
        const int b = row / (s.HO * s.TO);
        __syncthreads();
        // stage input rows: xs[(ci*KT + kt)*KH + kh][c] = X[b][ci][t-PT+kt][2ho-PH+kh][c - PW]
        for (int i = threadIdx.x; i < nxrow * WIN; i += THREADS) {
            const int c = i % WIN, r = i / WIN;
            const int kh = r % s.KH, kt = (r / s.KH) % s.KT, ci = r / (s.KH * s.KT);
            const int ti = t - s.PT + kt, hi = 2 * ho - s.PH + kh, wi = c - s.PW;
            float v = 0.f;
            if (ti >= 0 && ti < s.T && hi >= 0 && hi < s.H && wi >= 0 && wi < s.W)
                v = x[(((int64_t)b * s.CIN + ci) * s.T + ti) * plane + (int64_t)hi * s.W + wi];
            xs[r * WINP + c] = v;
        }
        // stage dY row: ys[co][wo] = dY[b][co][t][ho][wo]; zero-pad to an even count
        const int wo2 = (s.WO + 1) & ~1;
        for (int i = threadIdx.x; i < COUT * wo2; i += THREADS) {
            const int wo = i % wo2, co = i / wo2;
            ys[co * YS + wo] = wo < s.WO ? dy[(((int64_t)b * COUT + co) * s.TO + t) * yplane + (int64_t)ho * s.WO + wo] : 0.f;
        }
        __syncthreads();
        const int kh = lane >> 5;
        for (int k0 = 0; k0 < wo2; k0 += 2) {
            const int k = k0 + kh;
            const float a0 = ys[(lane & 31) * YS + k];
            const float a1 = ys[(32 + (lane & 31)) * YS + k];
#pragma unroll
            for (int j = 0; j < NTW; ++j) {
                const float bv = xs[boff[j] + 2 * k];
                acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bv, acc[0][j], 0, 0, 0);
                acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, bv, acc[1][j], 0, 0, 0);
            }
        }
    }
    // partial tile out: C map col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
    float* p = part + (int64_t)blockIdx.x * COUT * s.N;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const int n = (wave * NTW + j) * 32 + (lane & 31);
            if (n < s.N) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int co = m * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    p[(int64_t)co * s.N + n] = acc[m][j][r];
                }
            }
        }
}

__global__ void reduce_kernel(const float* __restrict__ part, int nparts, int total, float* __restrict__ dw, int accumulate) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    float v = 0.f;
    for (int g = 0; g < nparts; ++g) v += part[(int64_t)g * total + i];
    dw[i] = accumulate ? dw[i] + v : v;
}

inline int nparts_for(int rows) { return rows < 1024 ? rows : 1024; }

}  // namespace c3w
}  // namespace avse

using namespace avse::c3w;

extern "C" {

int64_t avse_conv3d_wgrad_workspace_bytes(int64_t B, int64_t TO, int64_t HO, int64_t N) {
    return 4 * (int64_t)nparts_for((int)(B * TO * HO)) * COUT * N;
}

int avse_conv3d_wgrad(int64_t B, int64_t CIN, int64_t T, int64_t H, int64_t W, int64_t KT, int64_t KH, int64_t KW,
                      int64_t PT, int64_t PH, int64_t PW, const float* x, const float* dy, float* dw, int32_t accumulate,
                      float* workspace, avse_stream_t stream) {
    if (!x || !dy || !dw || !workspace) return AVSE_EINVAL;
    Shape s;
    s.B = (int)B; s.CIN = (int)CIN; s.T = (int)T; s.H = (int)H; s.W = (int)W;
    s.KT = (int)KT; s.KH = (int)KH; s.KW = (int)KW; s.PT = (int)PT; s.PH = (int)PH; s.PW = (int)PW;
    s.TO = s.T + 2 * s.PT - s.KT + 1;
    s.HO = (s.H + 2 * s.PH - s.KH) / 2 + 1;
    s.WO = (s.W + 2 * s.PW - s.KW) / 2 + 1;
    s.N = s.CIN * s.KT * s.KH * s.KW;
    if (B <= 0 || CIN <= 0 || s.TO <= 0 || s.HO <= 0 || s.WO <= 0 || s.WO > MAX_WO || s.KW > 8) return AVSE_ESHAPE;
    const int nt = (s.N + 31) / 32;
    const int ntw = (nt + 3) / 4;
    if (ntw > 6) return AVSE_ESHAPE;
    s.rows = s.B * s.TO * s.HO;
    s.nparts = nparts_for(s.rows);
    const int WIN = 2 * (s.WO - 1) + s.KW;
    const size_t lds = 4 * ((size_t)s.CIN * s.KT * s.KH * (WIN + 1) + 2 * MAX_WO + 8 + COUT * YS);
    if (lds > 160 * 1024) return AVSE_ESHAPE;
    hipStream_t st = (hipStream_t)stream;
    dim3 grid(s.nparts), block(THREADS);
    switch (ntw) {
        case 1: hipLaunchKernelGGL(wgrad_kernel<1>, grid, block, lds, st, s, x, dy, workspace); break;
        case 2: hipLaunchKernelGGL(wgrad_kernel<2>, grid, block, lds, st, s, x, dy, workspace); break;
        case 3: hipLaunchKernelGGL(wgrad_kernel<3>, grid, block, lds, st, s, x, dy, workspace); break;
        case 4: hipLaunchKernelGGL(wgrad_kernel<4>, grid, block, lds, st, s, x, dy, workspace); break;
        case 5: hipLaunchKernelGGL(wgrad_kernel<5>, grid, block, lds, st, s, x, dy, workspace); break;
        default: hipLaunchKernelGGL(wgrad_kernel<6>, grid, block, lds, st, s, x, dy, workspace); break;
    }
    AVSE_CHECK_LAUNCH();
    const int total = COUT * s.N;
    hipLaunchKernelGGL(reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, st, workspace, s.nparts, total, dw,
                       (int)accumulate);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
