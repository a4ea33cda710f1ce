// Forward of the lip front-end Conv3d for gfx950, as an implicit GEMM on the exact-fp32 MFMA
// (v_mfma_f32_32x32x2_f32), reading the lips in their stored dtype (uint8 frames or fp32).
//
// Replaces nn.Conv3d(CIN, 64, (5, 7, 7), stride (1, 2, 2), padding (2, 3, 3), bias=False) of
// /root/reference/baseline/avse1/model.py:29-34 (frontend3D, CIN = 3).  MIOpen ran the avse1 C2 shape as a
// Winograd f3x2 Conv2d over frames (time taps folded into 15 input channels by a plane copy, result transposed
// back): 7.1 ms isolated, 14.8 ms per call inside the step (profiles/r03_avse1_default_bench_window_stats.csv).
//
//   y[b][co][t][ho][wo] = sum_{ci, kt, kh, kw} W[co][ci][kt][kh][kw] * x[b][ci][t + kt - 2][2 ho + kh - 3][2 wo + kw - 3]
//
// GEMM view: M = co (64), N = output pixels, K = (ci, kt, kh, kw).  A workgroup owns 384 consecutive output pixels
// of one (b, t) plane (8 rows of 48 at avse1's 96 x 96 lips) and all 64 channels; wave w computes both 32-channel
// tiles of the 3 pixel tiles w * 3 .. w * 3 + 2 (96 accumulators).  The K loop runs over pairs of input planes
// (ci, kt): lanes 0-31 take the pair's first plane, lanes 32-63 its second (the MFMA's two k values), so every
// K-step is one (kh, kw) tap and all 49 taps of a pair are straight-line code with immediate LDS offsets.  Per pair
// the 2 planes' input window (2 * 7 + 7 rows x 101 columns, zero outside the frame / clip) is staged in LDS with even
// and odd columns in separate arrays (the stride-2 pixel walk becomes unit stride: no bank conflicts), and the
// pair's weights as [tap][plane][co]; the next pair is loaded into registers while the current one's MFMAs run.
#include "common.h"

namespace avse {
namespace c3f {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int COUT = 64, KT = 5, KH = 7, KW = 7, PT = 2, PH = 3, PW = 3, THREADS = 256;
constexpr int TAPS = KH * KW;                  // 49 K-steps per plane pair
constexpr int TILES_PER_WAVE = 3, TILE_PX = 4 * TILES_PER_WAVE * 32;   // 384 output pixels per workgroup

template <int CIN, int H, int W>
struct Geo {
    static constexpr int HO = (H + 2 * PH - KH) / 2 + 1, WO = (W + 2 * PW - KW) / 2 + 1;
    static constexpr int PLANE_PX = HO * WO;
    static constexpr int NT = (PLANE_PX + TILE_PX - 1) / TILE_PX;          // workgroups per (b, t)
    static constexpr int NR = (TILE_PX - 1) / WO + 2;                     // output rows a tile can touch
    static constexpr int IR = 2 * (NR - 1) + KH;                          // staged input rows
    static constexpr int IC = 2 * (WO - 1) + KW;                          // staged input columns
    static constexpr int PAR_RAW = (IC + 1) / 2;
    // row stride RS = 2 * PAR with RS % 32 == 16: the two rows a 32-pixel tile can straddle land on disjoint banks
    static constexpr int PAR = ((PAR_RAW + 7) / 16) * 16 + 8;
    static constexpr int RS = 2 * PAR;
    static constexpr int XPLANE = IR * RS;                                // floats per staged plane
    static constexpr int NPL = CIN * KT, NQ = (NPL + 1) / 2;             // planes, plane pairs
    static constexpr int XEL = 2 * IR * IC;                               // staged input elements per pair
    static constexpr int XPT = (XEL + THREADS - 1) / THREADS;
    static constexpr int WEL = TAPS * 2 * COUT;                           // staged weights per pair
    static constexpr int WPT = (WEL / 4 + THREADS - 1) / THREADS;         // float4 per thread
    static constexpr int LDS_FLOATS = 2 * XPLANE + WEL;
    static_assert(RS % 32 == 16 && PAR >= PAR_RAW, "row stride");
    static_assert(WEL % 4 == 0, "weights in float4");
};

// wt[q][tap][h][co] = W[co][plane 2q + h][tap] (0 for the padding plane of an odd plane count)
__global__ void prep_weights_kernel(const float* __restrict__ w, int npl, int nq, float* __restrict__ wt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq * TAPS * 2 * COUT) return;
    const int co = i % COUT, h = (i / COUT) % 2, tap = (i / (2 * COUT)) % TAPS, q = i / (2 * COUT * TAPS);
    const int pl = 2 * q + h;
    wt[i] = pl < npl ? w[((int64_t)co * npl + pl) * TAPS + tap] : 0.f;
}

template <typename T, int CIN, int H, int W>
__global__ __launch_bounds__(THREADS, 2) void fwd_kernel(int B, int TT, const T* __restrict__ x,
                                                         const float* __restrict__ wt, float* __restrict__ y) {
    using G = Geo<CIN, H, W>;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* xs = lds;                          // [2][IR][RS]: plane h, input row, (even | odd) columns
    float* ws = lds + 2 * G::XPLANE;          // [TAPS][2][COUT]
    const int lane = threadIdx.x & 63, half = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = xcd_remap(blockIdx.x, gridDim.x);    // the NT tiles of a frame and the next frames share an L2
    const int tile = bid % G::NT, bt = bid / G::NT;
    const int t = bt % TT, b = bt / TT;
    const int p0 = tile * TILE_PX;
    const int r0 = p0 / G::WO;                // first output row of the tile
    const int hi0 = 2 * r0 - PH;              // input row of staged row 0

    const int64_t nx = (int64_t)B * CIN * TT * H * W;     // < 2^31 elements (checked at launch)
    const auto rx = make_rsrc(x, nx);
    const int OOB = (int)nx;

    // B-operand base per pixel tile: staged row 2 (ho - r0), even-column index wo, plane = half
    int bbase[TILES_PER_WAVE];
#pragma unroll
    for (int j = 0; j < TILES_PER_WAVE; ++j) {
        int p = p0 + (wave * TILES_PER_WAVE + j) * 32 + (lane & 31);
        if (p >= G::PLANE_PX) p = p0;                     // padding pixels of a partial last tile: never stored
        const int ho = p / G::WO, wo = p % G::WO;
        bbase[j] = half * G::XPLANE + 2 * (ho - r0) * G::RS + wo;
    }
    const int abase = half * COUT + (lane & 31);

    float xr[G::XPT];
    float4 wr[G::WPT];
    auto prefetch = [&](int q) {
#pragma unroll
        for (int i = 0; i < G::XPT; ++i) {
            const int e = threadIdx.x + i * THREADS;
            const int c = e % G::IC, row = (e / G::IC) % G::IR, h = e / (G::IC * G::IR);
            const int pl = 2 * q + h, ci = pl / KT, kt = pl % KT;
            const int ti = t + kt - PT, hi = hi0 + row, wi = c - PW;
            const bool ok = e < G::XEL && pl < G::NPL && ti >= 0 && ti < TT && hi >= 0 && hi < H && wi >= 0 && wi < W;
            xr[i] = bufld<T>::ld(rx, ok ? (((b * CIN + ci) * TT + ti) * H + hi) * W + wi : OOB, 0);
        }
        const float4* wq = reinterpret_cast<const float4*>(wt + (int64_t)q * G::WEL);
#pragma unroll
        for (int i = 0; i < G::WPT; ++i) {
            const int e = threadIdx.x + i * THREADS;
            if (e < G::WEL / 4) wr[i] = wq[e];
        }
    };

    floatx16 acc[2][TILES_PER_WAVE];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int j = 0; j < TILES_PER_WAVE; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][j][r] = 0.f;

    prefetch(0);
    for (int q = 0; q < G::NQ; ++q) {
        __syncthreads();                                  // the previous pair's MFMAs are done with LDS
#pragma unroll
        for (int i = 0; i < G::XPT; ++i) {
            const int e = threadIdx.x + i * THREADS;
            const int c = e % G::IC, row = (e / G::IC) % G::IR, h = e / (G::IC * G::IR);
            if (e < G::XEL) xs[h * G::XPLANE + row * G::RS + (c & 1) * G::PAR + (c >> 1)] = xr[i];
        }
#pragma unroll
        for (int i = 0; i < G::WPT; ++i) {
            const int e = threadIdx.x + i * THREADS;
            if (e < G::WEL / 4) reinterpret_cast<float4*>(ws)[e] = wr[i];
        }
        __syncthreads();
        if (q + 1 < G::NQ) prefetch(q + 1);
#pragma unroll
        for (int kh = 0; kh < KH; ++kh)
#pragma unroll
            for (int kw = 0; kw < KW; ++kw) {
                const int tap = kh * KW + kw;
                const int xoff = kh * G::RS + (kw & 1) * G::PAR + (kw >> 1);
                const float a0 = ws[abase + tap * 2 * COUT];
                const float a1 = ws[abase + tap * 2 * COUT + 32];
#pragma unroll
                for (int j = 0; j < TILES_PER_WAVE; ++j) {
                    const float bv = xs[bbase[j] + xoff];
                    acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bv, acc[0][j], 0, 0, 0);
                    acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, bv, acc[1][j], 0, 0, 0);
                }
            }
    }
    // y[b][co][t][p]: C map col = lane & 31 (pixel), row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5) (channel)
    float* yb = y + ((int64_t)b * COUT * TT + t) * G::PLANE_PX;
#pragma unroll
    for (int j = 0; j < TILES_PER_WAVE; ++j) {
        const int p = p0 + (wave * TILES_PER_WAVE + j) * 32 + (lane & 31);
        if (p < G::PLANE_PX) {
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int co = m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                    yb[(int64_t)co * TT * G::PLANE_PX + p] = acc[m][j][r];
                }
        }
    }
}

template <typename T, int CIN, int H, int W>
int launch(int64_t B, int64_t TT, const void* x, const float* w, float* y, float* workspace, hipStream_t st) {
    using G = Geo<CIN, H, W>;
    if ((int64_t)B * CIN * TT * H * W >= (1LL << 31) / (int64_t)sizeof(T)) return AVSE_ESHAPE;   // 32-bit offsets
    if (B * TT * G::NT >= (1LL << 31)) return AVSE_ESHAPE;
    const int nw = G::NQ * G::WEL;
    hipLaunchKernelGGL(prep_weights_kernel, dim3((nw + 255) / 256), dim3(256), 0, st, w, G::NPL, G::NQ, workspace);
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL((fwd_kernel<T, CIN, H, W>), dim3((unsigned)(B * TT * G::NT)), dim3(THREADS),
                       4 * G::LDS_FLOATS, st, (int)B, (int)TT, (const T*)x, workspace, y);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // namespace c3f
}  // namespace avse

using namespace avse::c3f;

extern "C" {

// shapes compiled in: the avse1 front-end (3 x 96 x 96 lips)
int64_t avse_conv3d_fwd_workspace_bytes(int64_t CIN, int64_t H, int64_t W) {
    if (CIN == 3 && H == 96 && W == 96) return 4 * (int64_t)Geo<3, 96, 96>::NQ * Geo<3, 96, 96>::WEL;
    return 0;
}

int avse_conv3d_fwd(int64_t B, int64_t CIN, int64_t T, int64_t H, int64_t W, int32_t x_dtype, const void* x,
                    const float* w, float* y, float* workspace, avse_stream_t stream) {
    if (!x || !w || !y || !workspace) return AVSE_EINVAL;
    if (B <= 0 || T <= 0) return AVSE_ESHAPE;
    hipStream_t st = (hipStream_t)stream;
    if (CIN == 3 && H == 96 && W == 96) {
        if (x_dtype == AVSE_U8) return launch<uint8_t, 3, 96, 96>(B, T, x, w, y, workspace, st);
        if (x_dtype == AVSE_F32) return launch<float, 3, 96, 96>(B, T, x, w, y, workspace, st);
        return AVSE_EDTYPE;
    }
    return AVSE_ESHAPE;
}

}  // extern "C"
