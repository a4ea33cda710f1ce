// Forward of the lip front-end Conv3d for gfx950, as an implicit GEMM on the f16 MFMA (v_mfma_f32_32x32x16_f16) with
// split operands, reading the lips in their stored dtype (uint8 frames or fp32).
//
// Replaces nn.Conv3d(CIN, 64, (5, 7, 7), stride (1, 2, 2), padding (2, 3, 3), bias=False) of
// /root/reference/baseline/avse1/model.py:29-34 (frontend3D, CIN = 3) and baseline/avse4/utils.py:97-118 (CIN = 1,
// 112 x 112 normalised grey frames).  MIOpen ran the avse1 C2 shape as a Winograd f3x2 Conv2d over frames (time taps
// folded into 15 input channels by a plane copy, result transposed back): 7.1 ms isolated, 14.8 ms per call inside the
// step (profiles/r03_avse1_default_bench_window_stats.csv).
//
//   y[b][co][t][ho][wo] = sum_{ci, kt, kh, kw} W[co][ci][kt][kh][kw] * x[b][ci][t + kt - 2][2 ho + kh - 3][2 wo + kw - 3]
//
// GEMM view: M = co (64), N = output pixels, K = (ci, kt, kh, kw).  A workgroup owns 384 consecutive output pixels
// of one (b, t) plane and all 64 channels; wave w computes both 32-channel tiles of the 3 pixel tiles w * 3 .. w * 3 + 2
// (96 accumulators).  Round 6: the fp32-frame path moved off the exact-fp32 MFMA (v_mfma_f32_32x32x2_f32, 1/16 of the
// f16 rate: avse4's C4 forward took 2.75 ms per step at 0.55 of that MFMA's peak, 10x its HBM time) onto the f16 kernel
// below with the frames split as well (3 MFMAs per product instead of 2).
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace avse {
namespace c3f {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int COUT = 64, KT = 5, KH = 7, KW = 7, PT = 2, PH = 3, PW = 3, THREADS = 256;
constexpr int TILES_PER_WAVE = 3, TILE_PX = 4 * TILES_PER_WAVE * 32;   // 384 output pixels per workgroup

template <int CIN, int H, int W>
struct Geo {
    static constexpr int HO = (H + 2 * PH - KH) / 2 + 1, WO = (W + 2 * PW - KW) / 2 + 1;
    static constexpr int PLANE_PX = HO * WO;
    static constexpr int NT = (PLANE_PX + TILE_PX - 1) / TILE_PX;          // workgroups per (b, t)
    static constexpr int NR = (TILE_PX - 1) / WO + 2;                     // output rows a tile can touch
    static constexpr int IR = 2 * (NR - 1) + KH;                          // staged input rows
    static constexpr int IC = 2 * (WO - 1) + KW;                          // staged input columns
    static constexpr int NPL = CIN * KT;                                  // input planes (ci, kt)
};

// ------------------------------------------------------------------------------------------------ split f16 MFMA
// The weights are split: W 2^e = hi + lo (fp16 each, 22 bits; max |W| 2^e in [2^14, 2^15)).  uint8 frames are exact in
// fp16, so y = 2^-e (x W_hi + x W_lo): 2 MFMAs per product.  fp32 frames are split too, x 2^f = x_hi + x_lo under the
// scale of max |x| (an absmax pass before the forward), y = 2^-(e + f) (x_hi W_hi + x_hi W_lo + x_lo W_hi): 3 MFMAs
// per product, the lo x lo term (2^-22 relative) dropped -- the products to 22 bits, fp32 accumulation: the fp32 class.
// K per input plane (ci, kt): 8 kernel rows (7 + a zero row) x 8 columns (7 + a zero column) = 4 k16-steps; k-step s,
// lane half h = kernel row 2 s + h, the lane's 8 k = kernel columns 0..7 = input columns 2 wo - 3 .. 2 wo + 4 of input
// row 2 ho + kh - 3: 8 consecutive fp16 of the staged row, two 8-B reads from one of two copies of the row (copy 0
// starts at column -3, copy 1 at column -1, so that either wo parity reads 8-B aligned words).
constexpr int F16_KSTEPS = 4;                    // k16-steps per plane
constexpr int WB_HALF = F16_KSTEPS * COUT * 16 * 2;   // bytes of one plane's hi (or lo) weights
constexpr int XM_GRID = 512;                     // blocks of the x absmax pass (partial maxima in the workspace)
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));

// max |v| over n floats -> *mb (float bits) by one 1024-thread block (the weights; the x pass's partial maxima)
__global__ void wmax16_kernel(const float* __restrict__ w, int n, uint32_t* __restrict__ mb) {
    float m = 0.f;
    for (int i = threadIdx.x; i < n; i += blockDim.x) m = fmaxf(m, fabsf(w[i]));
    uint32_t b = __float_as_uint(m);
    for (int o = 32; o >= 1; o >>= 1) b = max(b, (uint32_t)__shfl_xor((int)b, o, 64));
    __shared__ uint32_t red[16];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < (int)(blockDim.x >> 6); ++k) b = max(b, red[k]);
        *mb = b;
    }
}

// partial max |x| per block over a grid-stride walk (float4 when x is 16-B aligned, 2 loads in flight per thread)
template <bool VEC>
__global__ __launch_bounds__(256) void xmax_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ part) {
    float m0 = 0.f, m1 = 0.f;
    const int64_t stride = (int64_t)gridDim.x * 256;
    const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if constexpr (VEC) {
        const float4* x4 = reinterpret_cast<const float4*>(x);
        const int64_t n4 = n / 4;
        int64_t i = i0;
        for (; i + stride < n4; i += 2 * stride) {
            const float4 a = x4[i], c = x4[i + stride];
            m0 = fmaxf(m0, fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fmaxf(fabsf(a.z), fabsf(a.w))));
            m1 = fmaxf(m1, fmaxf(fmaxf(fabsf(c.x), fabsf(c.y)), fmaxf(fabsf(c.z), fabsf(c.w))));
        }
        if (i < n4) {
            const float4 a = x4[i];
            m0 = fmaxf(m0, fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fmaxf(fabsf(a.z), fabsf(a.w))));
        }
        for (int64_t j = 4 * n4 + i0; j < n; j += stride) m1 = fmaxf(m1, fabsf(x[j]));
    } else {
        for (int64_t j = i0; j < n; j += stride) m0 = fmaxf(m0, fabsf(x[j]));
    }
    uint32_t b = __float_as_uint(fmaxf(m0, m1));
    for (int o = 32; o >= 1; o >>= 1) b = max(b, (uint32_t)__shfl_xor((int)b, o, 64));
    __shared__ uint32_t red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = __uint_as_float(max(max(red[0], red[1]), max(red[2], red[3])));
}

typedef int i4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

__device__ inline i4_t rsrc16(const void* base, int64_t bytes) {
    if (bytes > 0x7FFFFFF0LL) bytes = 0x7FFFFFF0LL;
    const uint64_t a = (uint64_t)base;
    return i4_t{__builtin_amdgcn_readfirstlane((int)(uint32_t)a), __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff)),
                __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000};
}
// one 16-B-per-lane LDS-DMA wave-instruction (inline asm: the builtin makes the compiler wait vmcnt(0) before every
// ds_read of the array).  Nothing else in this kernel uses M0.
__device__ inline void dma16(i4_t r, uint32_t lds_addr, uint32_t voff) {
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(r), "s"(lds_addr)
                 : "memory");
}

__device__ inline int split_exp16(uint32_t mb) {
    const int ef = (int)((mb >> 23) & 0xff);
    if (mb == 0) return 0;
    const int k = ef == 0 ? -127 : ef - 127;
    return min(100, max(-100, 14 - k));
}

__global__ void wprep16_kernel(const float* __restrict__ w, int npl, const uint32_t* __restrict__ mb,
                               uint16_t* __restrict__ wq) {
    const int n = npl * F16_KSTEPS * COUT * 16;
    const float sc = __builtin_ldexpf(1.f, split_exp16(*mb));
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int k = i % 16, co = (i / 16) % COUT, st = (i / (16 * COUT)) % F16_KSTEPS, pl = i / (16 * COUT * F16_KSTEPS);
        const int kh = 2 * st + k / 8, kw = k % 8;
        const float v = (kh < KH && kw < KW) ? w[(((int64_t)co * npl + pl) * KH + kh) * KW + kw] * sc : 0.f;
        const _Float16 hi = (_Float16)v, lo = (_Float16)(v - (float)hi);
        wq[i] = __builtin_bit_cast(uint16_t, hi);
        wq[n + i] = __builtin_bit_cast(uint16_t, lo);
    }
}

// XS: the frames are split too (fp32 frames): a second (lo) image of the staged rows after the hi one
template <int CIN, int H, int W, bool XS>
struct Geo16 {
    using G = Geo<CIN, H, W>;
    static constexpr int RC = ((G::IC + 2 + 3) / 4) * 4;          // staged fp16 per row copy (columns -3 .. IC - 3 + 2)
    static constexpr int IRS = G::IR + 1;                         // staged rows: + a zero row for kernel row 7
    static constexpr int XBH = 2 * IRS * RC * 2;                  // bytes of one image: 2 copies x IRS rows
    static constexpr int XB = XS ? 2 * XBH : XBH;
    static constexpr int WOFF = ((XB + 15) / 16) * 16;            // the weight image inside a stage buffer
    static constexpr int WB = F16_KSTEPS * COUT * 16 * 2 * 2;    // hi + lo
    static constexpr int STG = WOFF + WB;
    static constexpr int XPT = (G::IR * G::IC + THREADS - 1) / THREADS;
    static_assert(2 * STG <= 80 * 1024, "two workgroups per CU");
};

// mb[0]: max |W| bits; mb[1]: max |x| bits (fp32 frames)
template <typename T, int CIN, int H, int W>
__global__ __launch_bounds__(THREADS, 2) void fwd16_kernel(int B, int TT, const T* __restrict__ x,
                                                           const uint16_t* __restrict__ wq, const uint32_t* __restrict__ mb,
                                                           float* __restrict__ y) {
    constexpr bool XS = std::is_same<T, float>::value;
    using G = Geo<CIN, H, W>;
    using G16 = Geo16<CIN, H, W, XS>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * G16::STG];
    const int lane = threadIdx.x & 63, half = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = xcd_remap(blockIdx.x, gridDim.x);    // the NT tiles of a frame and the next frames share an L2
    const int tile = bid % G::NT, bt = bid / G::NT;
    const int t = bt % TT, b = bt / TT;
    const int p0 = tile * TILE_PX;
    const int r0 = p0 / G::WO;                // first output row of the tile
    const int hi0 = 2 * r0 - PH;              // input row of staged row 0
    const int64_t nx = (int64_t)B * CIN * TT * H * W;     // < 2^31 bytes (checked at launch)
    const auto rx = make_rsrc(x, nx);
    const int OOB = (int)nx;
    const float xsc = XS ? __builtin_ldexpf(1.f, split_exp16(mb[1])) : 1.f;

    // B-operand byte offsets (without the k-step row) per pixel tile: copy (wo & 1), row 2 (ho - r0), the word of
    // column 2 wo - 3
    int boff[TILES_PER_WAVE];
#pragma unroll
    for (int j = 0; j < TILES_PER_WAVE; ++j) {
        int p = p0 + (wave * TILES_PER_WAVE + j) * 32 + (lane & 31);
        if (p >= G::PLANE_PX) p = p0;                     // padding pixels of a partial last tile: never stored
        const int ho = p / G::WO, wo = p % G::WO;
        const int cp = wo & 1;                                    // copy 1 starts 2 columns later
        boff[j] = ((cp * G16::IRS + 2 * (ho - r0)) * G16::RC + (2 * wo - 2 * cp)) * 2;
    }
    float xr[G16::XPT];
    const i4_t rwq = rsrc16(wq, (int64_t)2 * G::NPL * WB_HALF);
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const lds_void_t*)lds);
    // x of plane pl into registers; its weights (hi 8 KB, lo 8 KB) by LDS-DMA straight into buffer buf (free: its
    // last readers passed the barrier before this call)
    auto prefetch = [&](int pl, int buf) {
        const int ci = pl / KT, kt = pl % KT, ti = t + kt - PT;
#pragma unroll
        for (int i = 0; i < G16::XPT; ++i) {
            const int e = threadIdx.x + i * THREADS;
            const int c = e % G::IC, row = e / G::IC;
            const int hi = hi0 + row, wi = c - PW;
            const bool ok = e < G::IR * G::IC && ti >= 0 && ti < TT && hi >= 0 && hi < H && wi >= 0 && wi < W;
            xr[i] = bufld<T>::ld(rx, ok ? (((b * CIN + ci) * TT + ti) * H + hi) * W + wi : OOB, 0);
        }
        // 16 pieces of 1 KB (wq: all planes' hi, then all planes' lo), 4 per wave
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = wave * 4 + i, hl = k / 8, kk = k % 8;
            dma16(rwq, lds0 + buf * G16::STG + G16::WOFF + hl * WB_HALF + kk * 1024,
                  (uint32_t)((hl * G::NPL + pl) * WB_HALF + kk * 1024 + lane * 16));
        }
    };
    auto stage = [&](int buf) {
        uint8_t* img = lds + buf * G16::STG;
        _Float16* xs = reinterpret_cast<_Float16*>(img);
        _Float16* xl = reinterpret_cast<_Float16*>(img + G16::XBH);
#pragma unroll
        for (int i = 0; i < G16::XPT; ++i) {
            const int e = threadIdx.x + i * THREADS;
            if (e < G::IR * G::IC) {
                const int c = e % G::IC, row = e / G::IC;
                const float v = xr[i] * xsc;                                    // uint8: exact, xsc = 1
                const _Float16 h = (_Float16)v;
                xs[row * G16::RC + c] = h;                                      // copy 0: column c - 3 at c
                if (c >= 2) xs[(G16::IRS + row) * G16::RC + c - 2] = h;         // copy 1: column c - 3 at c - 2
                if constexpr (XS) {
                    const _Float16 l = (_Float16)(v - (float)h);
                    xl[row * G16::RC + c] = l;
                    if (c >= 2) xl[(G16::IRS + row) * G16::RC + c - 2] = l;
                }
            }
        }
        // zeros: each copy's columns past the window (read by the zero-weight 8th kernel column) and the zero row
        // IR of both copies (the zero-weight 8th kernel row): NaN-free operands for the padded k
        for (int i = threadIdx.x; i < 2 * G16::IRS * 8; i += THREADS) {
            const int cp = i / (G16::IRS * 8), row = (i / 8) % G16::IRS, k = i % 8;
            const int c0 = cp ? G::IC - 2 : G::IC;
#pragma unroll
            for (int im = 0; im < (XS ? 2 : 1); ++im) {
                _Float16* xi = im ? xl : xs;
                if (row == G::IR) {
                    for (int c = k; c < G16::RC; c += 8) xi[(cp * G16::IRS + row) * G16::RC + c] = (_Float16)0.f;
                } else if (c0 + k < G16::RC) {
                    xi[(cp * G16::IRS + row) * G16::RC + c0 + k] = (_Float16)0.f;
                }
            }
        }
    };

    floatx16 acc[2][TILES_PER_WAVE];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int j = 0; j < TILES_PER_WAVE; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][j][r] = 0.f;

    prefetch(0, 0);
    for (int pl = 0; pl < G::NPL; ++pl) {
        const int buf = pl & 1;
        stage(buf);                                 // the buffer last read two planes ago (a barrier in between)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // this wave's weight pieces of plane pl have landed
        __syncthreads();
        if (pl + 1 < G::NPL) prefetch(pl + 1, buf ^ 1);
        const uint8_t* img = lds + buf * G16::STG;
        const uint8_t* wimg = img + G16::WOFF;
#pragma unroll
        for (int st = 0; st < F16_KSTEPS; ++st) {
            half8 ah[2], al[2];
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const int co = 32 * m + (lane & 31);
                ah[m] = *reinterpret_cast<const half8*>(wimg + ((st * COUT + co) * 16 + 8 * half) * 2);
                al[m] = *reinterpret_cast<const half8*>(wimg + WB_HALF + ((st * COUT + co) * 16 + 8 * half) * 2);
            }
            const int rowb = (2 * st + half) * G16::RC * 2;       // kernel row 2 st + half
#pragma unroll
            for (int j = 0; j < TILES_PER_WAVE; ++j) {
                const uint8_t* p = img + boff[j] + rowb;
                const half4 v0 = *reinterpret_cast<const half4*>(p);
                const half4 v1 = *reinterpret_cast<const half4*>(p + 8);
                const half8 bv = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    acc[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[m], bv, acc[m][j], 0, 0, 0);
                    acc[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[m], bv, acc[m][j], 0, 0, 0);
                }
                if constexpr (XS) {
                    const half4 l0 = *reinterpret_cast<const half4*>(p + G16::XBH);
                    const half4 l1 = *reinterpret_cast<const half4*>(p + G16::XBH + 8);
                    const half8 bl = {l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
#pragma unroll
                    for (int m = 0; m < 2; ++m)
                        acc[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[m], bl, acc[m][j], 0, 0, 0);
                }
            }
        }
    }
    // two factors: 2^-(e + f) alone can leave the fp32 range where the product does not
    const float unscale = __builtin_ldexpf(1.f, -split_exp16(mb[0]));
    const float unscale_x = XS ? __builtin_ldexpf(1.f, -split_exp16(mb[1])) : 1.f;
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
                    yb[(int64_t)co * TT * G::PLANE_PX + p] = acc[m][j][r] * unscale * unscale_x;
                }
        }
    }
}

// workspace: wq (2 NPL WB_HALF bytes) | mb[0] = max |W|, mb[1] = max |x| (16 B) | the x pass's partial maxima
template <int CIN, int H, int W>
constexpr int64_t ws_bytes() {
    return 2 * (int64_t)Geo<CIN, H, W>::NPL * WB_HALF + 16 + 4 * XM_GRID;
}

template <typename T, int CIN, int H, int W>
int launch(int64_t B, int64_t TT, const void* x, const float* w, float* y, float* workspace, hipStream_t st) {
    using G = Geo<CIN, H, W>;
    if ((int64_t)B * CIN * TT * H * W >= (1LL << 31) / (int64_t)sizeof(T)) return AVSE_ESHAPE;   // 32-bit offsets
    if (B * TT * G::NT >= (1LL << 31)) return AVSE_ESHAPE;
    uint16_t* wq = reinterpret_cast<uint16_t*>(workspace);
    uint32_t* mb = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(workspace) + 2 * G::NPL * WB_HALF);
    float* part = reinterpret_cast<float*>(mb + 4);
    hipLaunchKernelGGL(wmax16_kernel, dim3(1), dim3(1024), 0, st, w, G::NPL * COUT * KH * KW, mb);
    AVSE_CHECK_LAUNCH();
    const int n = G::NPL * F16_KSTEPS * COUT * 16;
    hipLaunchKernelGGL(wprep16_kernel, dim3((n + 255) / 256), dim3(256), 0, st, w, G::NPL, (const uint32_t*)mb, wq);
    AVSE_CHECK_LAUNCH();
    if constexpr (std::is_same<T, float>::value) {
        const int64_t nx = B * CIN * TT * H * W;
        if (((uintptr_t)x & 15) == 0)
            hipLaunchKernelGGL(xmax_kernel<true>, dim3(XM_GRID), dim3(256), 0, st, (const float*)x, nx, part);
        else
            hipLaunchKernelGGL(xmax_kernel<false>, dim3(XM_GRID), dim3(256), 0, st, (const float*)x, nx, part);
        AVSE_CHECK_LAUNCH();
        hipLaunchKernelGGL(wmax16_kernel, dim3(1), dim3(1024), 0, st, (const float*)part, XM_GRID, mb + 1);
        AVSE_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL((fwd16_kernel<T, CIN, H, W>), dim3((unsigned)(B * TT * G::NT)), dim3(THREADS), 0, st, (int)B,
                       (int)TT, (const T*)x, (const uint16_t*)wq, (const uint32_t*)mb, y);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // namespace c3f
}  // namespace avse

using namespace avse::c3f;

extern "C" {

// shapes compiled in: the avse1 front-end (3 x 96 x 96 lips, uint8 or fp32) and the avse4 one (1 x 112 x 112
// normalised grey frames, fp32: baseline/avse4/utils.py:97-118 frontend3D)
int64_t avse_conv3d_fwd_workspace_bytes(int64_t CIN, int64_t H, int64_t W) {
    if (CIN == 3 && H == 96 && W == 96) return ws_bytes<3, 96, 96>();
    if (CIN == 1 && H == 112 && W == 112) return ws_bytes<1, 112, 112>();
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
    if (CIN == 1 && H == 112 && W == 112) {
        if (x_dtype == AVSE_F32) return launch<float, 1, 112, 112>(B, T, x, w, y, workspace, st);
        return AVSE_EDTYPE;
    }
    return AVSE_ESHAPE;
}

}  // extern "C"
