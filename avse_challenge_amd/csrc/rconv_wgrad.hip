// Weight gradient of the ResNet-18 trunk 3x3 convolutions of the lip encoders for gfx950, as an implicit GEMM on the
// exact-fp32 MFMA (v_mfma_f32_32x32x2_f32), NCHW or channels-last (NHWC) activations.
//
// Replaces the weight-gradient half of nn.Conv2d(cin, cout, 3, stride s, padding 1, bias=False) in the BasicBlocks of
// /root/reference/baseline/avse1/utils/resnet.py:26-67 (conv3x3 :11-13; cin, cout in {64, 128, 256, 512}, s in {1, 2})
// as the avse1 VisualFeatNet runs them on B*T lip frames (model.py:48-58), and of the avse4 ResNetLayer convs
// (baseline/avse4/utils.py:40-93).  MIOpen ran the avse1 ones (igemm_wrw ... bt128x128, 21 launches) at ~0.33 of the
// fp32 MFMA peak inside the C2 step: 31.9 ms of 170 ms (profiles/r02d_*).
//
//   dW[co][ci][kh][kw] = sum_{n,ho,wo} dY[n][co][ho][wo] * X[n][ci][s ho - 1 + kh][s wo - 1 + kw]   (0 outside)
//
// GEMM view: M = cout, N = cin * 9, K = frames * HO * WO.  The spatial shape (H, W, stride) is a template parameter
// (the lip encoders have a handful, see the dispatch table at the end), so every index is constant-divided and the
// staging loops unroll.  Workgroup (co block, ci block, kernel row kh, k split) owns a 64 x 64 (co, ci) block for the
// 3 taps of row kh (wave w: the 32 x 32 tile (w / 2, w % 2), 3 accumulators) over a contiguous range of K chunks; a
// chunk is F whole frames or R output rows of one frame (at most P_MAX pixels).  Per chunk the dY pixels [p][co] and
// the zero-padded input rows S r + kh - 1 [frame][row][col][ci] sit in LDS pixel-major with an odd 65-float pixel
// stride: the coalesced global loads (consecutive lanes = consecutive pixels of one channel) write conflict-free and
// the MFMA operand reads (consecutive lanes = consecutive channels of one pixel) read conflict-free.  With 48
// accumulators the next chunk is loaded into registers (raw buffer loads, 32-bit offsets) while the current one's
// MFMAs run.  A K-step takes 2 pixels (lanes 0-31 pixel 2j, 32-63 pixel 2j + 1): one A read, 3 B reads, 3 MFMAs.
// Per-split partial sums go to a workspace summed by a second kernel (deterministic).
#include <algorithm>

#include "common.h"

namespace avse {
namespace rcw {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int THREADS = 256, CB = 64, PS = CB + 1;   // channel block, LDS pixel stride (floats)
constexpr int KS = 3, KK = 9;                        // 3x3 taps; a workgroup owns one kernel row (3 taps)
constexpr int P_MAX = 96;                            // output pixels per chunk
constexpr int LDS_BUDGET = 72 * 1024;                // bytes per workgroup: 2 workgroups per CU (~235 VGPRs)

constexpr int lds_floats(int P, int rows, int WIN) { return (((P + 1) & ~1) + 1) * PS + rows * WIN * PS; }

template <int H, int W, int S>
struct Geo {
    static constexpr int HO = (H - 1) / S + 1, WO = (W - 1) / S + 1, HWO = HO * WO, HW = H * W;
    static constexpr int WIN = (WO - 1) * S + 3;                     // staged input columns (-1 .. )
    static constexpr bool FRAMES = HWO <= P_MAX;                      // chunk = F whole frames, else R rows
    static constexpr int fit_f(int f) { return (f <= 1 || lds_floats(f * HWO, f * HO, WIN) * 4 <= LDS_BUDGET) ? f : fit_f(f - 1); }
    static constexpr int fit_r(int r) { return (r <= 1 || lds_floats(r * WO, r, WIN) * 4 <= LDS_BUDGET) ? r : fit_r(r - 1); }
    static constexpr int F = FRAMES ? fit_f(P_MAX / HWO) : 1;
    static constexpr int R = FRAMES ? HO : fit_r(P_MAX / WO > 0 ? P_MAX / WO : 1);
    static constexpr int P = F * R * WO;                                // pixels of a full chunk
    static constexpr int P2 = (P + 1) & ~1;
    static constexpr int BANDS = (HO + R - 1) / R;                     // row bands per frame (FRAMES: 1)
    static constexpr int NXW = F * R * WIN;                            // staged input pixels per channel (one kh)
    static constexpr int YV = (P2 * CB + THREADS - 1) / THREADS;       // staging registers per thread
    static constexpr int XV = (NXW * CB + THREADS - 1) / THREADS;
    static constexpr int LDSB = lds_floats(P, F * R, WIN) * 4;
    static_assert(P <= P_MAX && LDSB <= LDS_BUDGET, "chunk does not fit");
};

struct Args {
    int N, CIN, COUT, chunks, nci, nco, ksplit;
};

template <int H, int W, int S>
__global__ __launch_bounds__(THREADS, 2) void wgrad_kernel(Args s, const float* __restrict__ x,
                                                           const float* __restrict__ dy, float* __restrict__ part) {
    using G = Geo<H, W, S>;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nblk = s.nco * s.nci;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);       // the 3 kernel rows x co / ci blocks of a split share an XCD
    const int kh = bid % KS, ks = bid / KS / nblk, blk = (bid / KS) % nblk;
    const int cob = blk / s.nci, cib = blk % s.nci;
    const int c_lo = __builtin_amdgcn_readfirstlane((int)((int64_t)ks * s.chunks / s.ksplit));
    const int c_hi = __builtin_amdgcn_readfirstlane((int)((int64_t)(ks + 1) * s.chunks / s.ksplit));

    float* sy = lds;                                        // [P2 + 1][PS]: dY pixels
    float* sx = sy + (G::P2 + 1) * PS;                      // [F * R][WIN][PS]: input rows S * r + kh - 1
    const int xs_n = s.CIN * G::HW, ys_n = s.COUT * G::HWO;     // 32-bit offsets: tensors < 2^29 elements (checked)
    // raw buffer loads with 32-bit element offsets (one VGPR per address; an offset past num_records reads 0)
    const auto rx = make_rsrc(x, (int64_t)s.N * xs_n);
    const auto ry = make_rsrc(dy, (int64_t)s.N * ys_n);
    const int OOBX = s.N * xs_n, OOBY = s.N * ys_n;
    const int xb = cib * CB * G::HW, yb = cob * CB * G::HWO;

    float yv[G::YV], xv[G::XV];
    // chunk c -> registers: dY element e = co * P2 + p, input element e = ci * NXW + q (consecutive threads walk the
    // pixels of one channel: coalesced); everything past the chunk / outside the image is 0
    auto prefetch = [&](int c) {
        int f0, r0, nf, nr;
        if (G::FRAMES) {
            f0 = c * G::F; r0 = 0; nf = min(G::F, s.N - f0); nr = G::HO;
        } else {
            f0 = c / G::BANDS; r0 = (c % G::BANDS) * G::R; nf = 1; nr = min(G::R, G::HO - r0);
        }
        const int ybase = yb + f0 * ys_n + r0 * G::WO, xbase = xb + f0 * xs_n;
#pragma unroll
        for (int i = 0; i < G::YV; ++i) {
            const int e = threadIdx.x + i * THREADS, p = e % G::P2, co = e / G::P2;
            const int f = p / (G::R * G::WO), rem = p % (G::R * G::WO);
            const bool ok = co < CB && f < nf && rem / G::WO < nr;
            yv[i] = bufld<float>::ld(ry, ok ? ybase + f * ys_n + co * G::HWO + rem : OOBY, 0);
        }
#pragma unroll
        for (int i = 0; i < G::XV; ++i) {
            const int e = threadIdx.x + i * THREADS, q = e % G::NXW, ci = e / G::NXW;
            const int fr = q / G::WIN, col = q % G::WIN;                 // staged row fr = f * R + r
            const int f = fr / G::R, r = fr % G::R;
            const int hi = S * (r0 + r) + kh - 1, wi = col - 1;
            const bool ok = ci < CB && f < nf && r < nr && hi >= 0 && hi < H && wi >= 0 && wi < W;
            xv[i] = bufld<float>::ld(rx, ok ? xbase + f * xs_n + ci * G::HW + hi * W + wi : OOBX, 0);
        }
        return nf * nr * G::WO;
    };

    floatx16 acc[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[k][q] = 0.f;
    const int half = lane >> 5;
    const int co_l = (wave >> 1) * 32 + (lane & 31), ci_l = (wave & 1) * 32 + (lane & 31);

    int np = c_lo < c_hi ? prefetch(c_lo) : 0;
    for (int c = c_lo; c < c_hi; ++c) {
        const int npc = np;
        __syncthreads();                                    // previous chunk's MFMAs are done with LDS
#pragma unroll
        for (int i = 0; i < G::YV; ++i) {
            const int e = threadIdx.x + i * THREADS, p = e % G::P2, co = e / G::P2;
            if (co < CB) sy[p * PS + co] = yv[i];
        }
#pragma unroll
        for (int i = 0; i < G::XV; ++i) {
            const int e = threadIdx.x + i * THREADS, q = e % G::NXW, ci = e / G::NXW;
            if (ci < CB) sx[q * PS + ci] = xv[i];
        }
        __syncthreads();
        if (c + 1 < c_hi) np = prefetch(c + 1);             // in flight while this chunk's MFMAs run
        const int nk = (npc + 1) >> 1;
        for (int j = 0; j < nk; ++j) {
            const int p = 2 * j + half;                     // output pixel of this lane half
            const int fr = p / G::WO, w = p % G::WO;        // staged row (f * R + r), column
            const float a = sy[p * PS + co_l];
            const float* pb = sx + (fr * G::WIN + S * w) * PS + ci_l;
            const float b0 = pb[0], b1 = pb[PS], b2 = pb[2 * PS];
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b0, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b1, acc[1], 0, 0, 0);
            acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b2, acc[2], 0, 0, 0);
        }
    }
    // partial out: part[ks][co][ci][kh][kw]; C map col = lane & 31, row = (q & 3) + 8 (q >> 2) + 4 (lane >> 5)
    float* pp = part + (int64_t)ks * s.COUT * s.CIN * KK;
    const int ci = cib * CB + ci_l;
#pragma unroll
    for (int kw = 0; kw < KS; ++kw)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int co = cob * CB + (wave >> 1) * 32 + (q & 3) + 8 * (q >> 2) + 4 * half;
            pp[((int64_t)co * s.CIN + ci) * KK + kh * KS + kw] = acc[kw][q];
        }
}

// Channels-last (NHWC) activations (the avse1 bench's lip trunk): same decomposition; the staged tiles are 64-channel
// slices of contiguous pixel rows, loaded as float4 (16 B per lane, coalesced) and stored as float4 into a 64-float
// pixel stride (ds_write_b128; the MFMA b32 reads of 32 consecutive channels stay conflict-free).
__device__ inline float4 ld4(__amdgpu_buffer_rsrc_t r, int voff_elems) {
    const auto raw = __builtin_amdgcn_raw_buffer_load_b128(r, voff_elems * 4, 0, 0);
    return make_float4(__uint_as_float(raw[0]), __uint_as_float(raw[1]), __uint_as_float(raw[2]), __uint_as_float(raw[3]));
}

template <int H, int W, int S>
__global__ __launch_bounds__(THREADS, 2) void wgrad_nhwc_kernel(Args s, const float* __restrict__ x,
                                                                const float* __restrict__ dy, float* __restrict__ part) {
    using G = Geo<H, W, S>;
    constexpr int PSN = CB;                                 // 64-float pixel stride (16-B aligned rows)
    constexpr int YV4 = (G::P2 * CB / 4 + THREADS - 1) / THREADS, XV4 = (G::NXW * CB / 4 + THREADS - 1) / THREADS;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nblk = s.nco * s.nci;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int kh = bid % KS, ks = bid / KS / nblk, blk = (bid / KS) % nblk;
    const int cob = blk / s.nci, cib = blk % s.nci;
    const int c_lo = __builtin_amdgcn_readfirstlane((int)((int64_t)ks * s.chunks / s.ksplit));
    const int c_hi = __builtin_amdgcn_readfirstlane((int)((int64_t)(ks + 1) * s.chunks / s.ksplit));

    float* sy = lds;                                        // [P2 + 1][64]: dY pixels
    float* sx = sy + (G::P2 + 1) * PSN;                     // [F * R][WIN][64]: input rows S * r + kh - 1
    const auto rx = make_rsrc(x, (int64_t)s.N * G::HW * s.CIN);
    const auto ry = make_rsrc(dy, (int64_t)s.N * G::HWO * s.COUT);
    const int OOBX = s.N * G::HW * s.CIN, OOBY = s.N * G::HWO * s.COUT;

    float4 yv[YV4], xv[XV4];
    auto prefetch = [&](int c) {
        int f0, r0, nf, nr;
        if (G::FRAMES) {
            f0 = c * G::F; r0 = 0; nf = min(G::F, s.N - f0); nr = G::HO;
        } else {
            f0 = c / G::BANDS; r0 = (c % G::BANDS) * G::R; nf = 1; nr = min(G::R, G::HO - r0);
        }
        const int ypix0 = f0 * G::HWO + r0 * G::WO;
#pragma unroll
        for (int i = 0; i < YV4; ++i) {
            const int e = threadIdx.x + i * THREADS, p = e / (CB / 4), c4 = e % (CB / 4);
            const int f = p / (G::R * G::WO), rem = p % (G::R * G::WO);
            const bool ok = p < G::P2 && f < nf && rem / G::WO < nr;
            yv[i] = ld4(ry, ok ? (ypix0 + f * G::HWO + rem) * s.COUT + cob * CB + 4 * c4 : OOBY);
        }
#pragma unroll
        for (int i = 0; i < XV4; ++i) {
            const int e = threadIdx.x + i * THREADS, q = e / (CB / 4), c4 = e % (CB / 4);
            const int fr = q / G::WIN, col = q % G::WIN;
            const int f = fr / G::R, r = fr % G::R;
            const int hi = S * (r0 + r) + kh - 1, wi = col - 1;
            const bool ok = q < G::NXW && f < nf && r < nr && hi >= 0 && hi < H && wi >= 0 && wi < W;
            xv[i] = ld4(rx, ok ? ((f0 + f) * G::HW + hi * W + wi) * s.CIN + cib * CB + 4 * c4 : OOBX);
        }
        return nf * nr * G::WO;
    };

    floatx16 acc[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[k][q] = 0.f;
    const int half = lane >> 5;
    const int co_l = (wave >> 1) * 32 + (lane & 31), ci_l = (wave & 1) * 32 + (lane & 31);

    int np = c_lo < c_hi ? prefetch(c_lo) : 0;
    for (int c = c_lo; c < c_hi; ++c) {
        const int npc = np;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < YV4; ++i) {
            const int e = threadIdx.x + i * THREADS;
            if (e < G::P2 * CB / 4) *reinterpret_cast<float4*>(&sy[e * 4]) = yv[i];
        }
#pragma unroll
        for (int i = 0; i < XV4; ++i) {
            const int e = threadIdx.x + i * THREADS;
            if (e < G::NXW * CB / 4) *reinterpret_cast<float4*>(&sx[e * 4]) = xv[i];
        }
        __syncthreads();
        if (c + 1 < c_hi) np = prefetch(c + 1);
        const int nk = (npc + 1) >> 1;
        for (int j = 0; j < nk; ++j) {
            const int p = 2 * j + half;
            const int fr = p / G::WO, w = p % G::WO;
            const float a = sy[p * PSN + co_l];
            const float* pb = sx + (fr * G::WIN + S * w) * PSN + ci_l;
            const float b0 = pb[0], b1 = pb[PSN], b2 = pb[2 * PSN];
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b0, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b1, acc[1], 0, 0, 0);
            acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b2, acc[2], 0, 0, 0);
        }
    }
    float* pp = part + (int64_t)ks * s.COUT * s.CIN * KK;
    const int ci = cib * CB + ci_l;
#pragma unroll
    for (int kw = 0; kw < KS; ++kw)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int co = cob * CB + (wave >> 1) * 32 + (q & 3) + 8 * (q >> 2) + 4 * half;
            pp[((int64_t)co * s.CIN + ci) * KK + kh * KS + kw] = acc[kw][q];
        }
}

__global__ void reduce_kernel(const float* __restrict__ part, int nparts, int total, float* __restrict__ dw) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    float v = 0.f;
    for (int g = 0; g < nparts; ++g) v += part[(int64_t)g * total + i];
    dw[i] = v;
}

template <int H, int W, int S>
int chunks_of(int N) {
    using G = Geo<H, W, S>;
    return G::FRAMES ? (N + G::F - 1) / G::F : N * G::BANDS;
}

// k splits: about two workgroups per CU over the 256 CUs (3 kernel rows per block), at most one chunk per split
inline int ksplit_for(int chunks, int nblk) { return std::max(1, std::min(chunks, 512 / (KS * nblk))); }

template <int H, int W, int S>
int launch(int N, int CIN, int COUT, bool nhwc, const float* x, const float* dy, float* dw, float* ws, hipStream_t st) {
    using G = Geo<H, W, S>;
    Args a;
    a.N = N; a.CIN = CIN; a.COUT = COUT;
    a.chunks = chunks_of<H, W, S>(N);
    a.nci = CIN / CB; a.nco = COUT / CB;
    a.ksplit = ksplit_for(a.chunks, a.nci * a.nco);
    if (nhwc)
        hipLaunchKernelGGL((wgrad_nhwc_kernel<H, W, S>), dim3(a.ksplit * a.nci * a.nco * KS), dim3(THREADS), G::LDSB, st, a,
                           x, dy, ws);
    else
        hipLaunchKernelGGL((wgrad_kernel<H, W, S>), dim3(a.ksplit * a.nci * a.nco * KS), dim3(THREADS), G::LDSB, st, a, x,
                           dy, ws);
    AVSE_CHECK_LAUNCH();
    const int total = COUT * CIN * KK;
    hipLaunchKernelGGL(reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, st, ws, a.ksplit, total, dw);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

// the lip-encoder trunk shapes: avse1 at 96x96 lips (24 .. 3), avse4 / C5 at 112x112 (28 .. 4), avse2 at 224x224
// (56 .. 7); (H, W, stride) -> kernel.  Returns the number of chunks (0: not a supported shape).
#define AVSE_RCW_SHAPES(X) \
    X(24, 24, 1) X(24, 24, 2) X(12, 12, 1) X(12, 12, 2) X(6, 6, 1) X(6, 6, 2) X(3, 3, 1) \
    X(28, 28, 1) X(28, 28, 2) X(14, 14, 1) X(14, 14, 2) X(7, 7, 1) X(7, 7, 2) X(4, 4, 1) \
    X(56, 56, 1) X(56, 56, 2)

inline int chunks_for(int H, int W, int S, int N) {
#define X_(h, w, s) if (H == h && W == w && S == s) return chunks_of<h, w, s>(N);
    AVSE_RCW_SHAPES(X_)
#undef X_
    return 0;
}

}  // namespace rcw
}  // namespace avse

using namespace avse::rcw;

static bool supported(int64_t N, int64_t CIN, int64_t COUT, int64_t H, int64_t W, int64_t stride) {
    if (N <= 0 || CIN <= 0 || COUT <= 0 || CIN % CB || COUT % CB) return false;
    if (N * CIN * H * W >= (1LL << 29) || N * COUT * H * W >= (1LL << 29)) return false;   // buffer bytes < 2^31
    return chunks_for((int)H, (int)W, (int)stride, 1) > 0;
}

extern "C" {

int64_t avse_rconv_wgrad_workspace_bytes(int64_t N, int64_t CIN, int64_t COUT, int64_t H, int64_t W, int64_t stride) {
    if (!supported(N, CIN, COUT, H, W, stride)) return 0;
    const int nblk = (int)(CIN / CB * (COUT / CB));
    return 4 * (int64_t)ksplit_for(chunks_for((int)H, (int)W, (int)stride, (int)N), nblk) * COUT * CIN * KK;
}

int avse_rconv_wgrad(int64_t N, int64_t CIN, int64_t COUT, int64_t H, int64_t W, int64_t stride, int32_t nhwc,
                     const float* x, const float* dy, float* dw, float* workspace, avse_stream_t stream) {
    if (!x || !dy || !dw || !workspace) return AVSE_EINVAL;
    if (!supported(N, CIN, COUT, H, W, stride)) return AVSE_ESHAPE;
    hipStream_t st = (hipStream_t)stream;
#define X_(h, w, s) \
    if (H == h && W == w && stride == s) \
        return launch<h, w, s>((int)N, (int)CIN, (int)COUT, nhwc != 0, x, dy, dw, workspace, st);
    AVSE_RCW_SHAPES(X_)
#undef X_
    return AVSE_ESHAPE;
}

}  // extern "C"
