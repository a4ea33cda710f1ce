// 3x3 convolutions of the lip-encoder ResNet trunks for gfx950: forward, stride-1 input gradient and weight gradient
// as implicit GEMMs on the fp16 MFMA with fp32-accurate split operands (the "fp16x3" scheme of dconv.hip).
//
// Replaces the trunk convolutions nn.Conv2d(cin, cout, 3, stride s in {1, 2}, padding=1, bias=False) of
//   /root/reference/baseline/avse1/utils/resnet.py:9-10 (conv3x3, used by BasicBlock :26-67, ResNet :70-124) and
//   /root/reference/baseline/avse4/utils.py:40-84 (ResNetLayer conv1a / conv2a / conv1b / conv2b),
// channels 64 .. 512 on 2400 (avse1) / 1200 (avse4) lip frames of 3 .. 28 pixels square.  MIOpen ran them in fp32 at
// 0.6-0.8 of the fp32 MFMA peak; they are most of the avse1 lip branch, the critical path of the avse1 C2 step once
// the AudioFeatNet convolutions moved to dconv.hip.
//
//   Y[n][ho][wo][o] = sum_{i,kh,kw} X[n][s ho + kh - 1][s wo + kw - 1][i] W[o][i][kh][kw]          (0 outside)
//   input gradient (s = 1): the same with X = dY and W'[o = ci][i = co][kh][kw] = W[co][ci][2 - kh][2 - kw]
//   weight gradient: dW[o][i][kh][kw] = sum_{n,ho,wo} dY[n][ho][wo][o] X[n][s ho + kh - 1][s wo + kw - 1][i]
//
// Operands are NHWC tensors split once into the Q layout: per pixel, C / 16 chunks of 64 B = [hi 16 ch][lo 16 ch]
// (avse_split16 over the tensor viewed as (pixels C / 64, 64): the same chunk order), hi = fp16(x 2^e),
// lo = fp16(x 2^e - hi), max |x| 2^e in [2^14, 2^15); products hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_f16
// (fp32 accumulation), scaled back by 2^-(e_x + e_w).  Weights: avse_sconv_wprep -> [kh][ci chunk q][kw][o][64 B].
//
// Forward tile: TM consecutive output pixels of the flat (n, ho, wo) raster x TN output channels, 8 waves of
// 64 pixels x 64 channels (2 x 2 MFMA blocks, 64 accumulators per lane): TN = 64, TM = 512 for 64 output channels,
// TN = 128, TM = 256 otherwise.  Reduction in stages (kernel row kh, 16-channel chunk q); a stage stages, by LDS-DMA,
// every input row the tile's output rows read at kernel row kh as a padded segment of RS = s Wo + 2 positions (one
// per input column -1 .. s Wo, zeros outside the image), so output pixel (row k of the tile, column wo) reads position
// k RS + s wo + kw for tap kw: the 3 kw taps share one staged segment.  Per stage and wave: 3 taps x 4 blocks x 3
// products = 36 MFMAs.  Two LDS buffers, the next stage issued right after the barrier that frees its buffer.
#include <algorithm>

#include "common.h"

namespace avse {
namespace scv {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef int i4_t __attribute__((ext_vector_type(4)));
typedef short s4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) s4_t lds_s4_t;

constexpr int ROWB = 64;                 // LDS / Q bytes per staged (position, 16-channel chunk)
constexpr int NPOS_MAX = 720;            // staged positions per forward stage (host-checked)
constexpr int XIMG = NPOS_MAX * ROWB;    // 45 KB
constexpr uint32_t OOB = 0x7FFFFFF0u;    // DMA offset past every buffer range: lands as zeros

__device__ inline int swz(int r) { return (r >> 2) & 3; }

// same function as dconv.hip / projgemm.hip: max |x| 2^e in [2^14, 2^15)
__device__ inline int split_exp(uint32_t mb) {
    const int ef = (int)((mb >> 23) & 0xff);
    if (mb == 0) return 0;
    const int k = ef == 0 ? -127 : ef - 127;
    return min(100, max(-100, 14 - k));
}

__device__ inline i4_t rsrc_of(const void* base, int64_t bytes) {
    if (bytes > 0x7FFFFFF0LL) bytes = 0x7FFFFFF0LL;
    const uint64_t a = (uint64_t)base;
    return i4_t{__builtin_amdgcn_readfirstlane((int)(uint32_t)a), __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff)),
                __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000};
}

// one 16-B-per-lane LDS-DMA wave-instruction (inline asm: the builtin makes the compiler wait vmcnt(0) before every
// ds_read of the array).  Nothing else in these kernels uses M0.
__device__ inline void dma16(i4_t r, uint32_t lds_addr, uint32_t voff) {
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(r), "s"(lds_addr)
                 : "memory");
}

__device__ inline uint32_t lds_u32(const void* p) {
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const lds_void_t*)p);
}

__device__ inline half8 frag(const uint8_t* img, int row, int c) {
    return *reinterpret_cast<const half8*>(img + row * ROWB + 16 * (c ^ swz(row)));
}

// t / d and t % d for 0 <= t < 2^22, d >= 1 (float reciprocal + one correction step)
__device__ inline void divmod_small(int t, int d, float inv_d, int& q, int& r) {
    q = (int)((float)t * inv_d);
    r = t - q * d;
    if (r >= d) { r -= d; ++q; }
    if (r < 0) { r += d; --q; }
}

struct FArgs {
    const void* xq;            // Q-split input (N Hi Wi pixels x Ci 4 B)
    const void* wq;            // avse_sconv_wprep image
    const uint32_t* xmax;
    const uint32_t* wmax;
    float* y;                  // NHWC fp32 (N Ho Wo x Co)
    int N, Hi, Wi, Ci, Ho, Wo, Co;
    int tiles_n;               // Co / TN
    int RS, npos;              // staged segment length, positions per stage (multiple of 16, <= NPOS_MAX)
};

template <int S, int TN>
__global__ __launch_bounds__(512, 1) void fwd_kernel(FArgs a) {
    constexpr int WAVES = 8, WN = TN / 64, WM = WAVES / WN, TM = 64 * WM;
    constexpr int WIMG = 3 * TN * ROWB;
    constexpr int STG = XIMG + WIMG;
    constexpr int PW = WIMG / 1024;                                // W pieces per stage
    constexpr int MP = (NPOS_MAX / 16 + PW + WAVES - 1) / WAVES;   // pieces per wave and stage (upper bound)
    __shared__ __attribute__((aligned(1024))) uint8_t lds[2 * STG];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int tn = bid % a.tiles_n, tm = bid / a.tiles_n;         // the o tiles of one pixel tile run together
    const int p0 = tm * TM, o0 = tn * TN;
    const int NHWo = a.N * a.Ho * a.Wo, NHo = a.N * a.Ho;
    const int g0 = p0 / a.Wo;                                      // first output row (flat n, ho) of the tile
    const int NQ = a.Ci / 16, NSTG = 3 * NQ;
    const i4_t rx = rsrc_of(a.xq, (int64_t)a.N * a.Hi * a.Wi * a.Ci * 4);
    const i4_t rw = rsrc_of(a.wq, (int64_t)9 * a.Ci * a.Co * 4);
    const uint32_t lds0 = lds_u32(lds);
    const int PX = a.npos / 16, PT = PX + PW;
    const int npieces = (PT - wave + WAVES - 1) / WAVES;
    const uint32_t pixb = (uint32_t)a.Ci * 4u;

    // this wave's DMA pieces, everything that does not depend on the stage precomputed: X pieces (position r = 16 k +
    // lane / 4) the byte offset of their input pixel at kernel row 0 plus the lane's source chunk (or OOB for padding
    // columns / rows past the tile) and the valid kernel rows [khlo, khhi); W pieces the lane's byte offset inside a
    // stage's weight rows.  Per stage a piece then costs an add and a compare (round 5 recomputed the pixel with two
    // 32-bit multiplies per piece and stage)
    uint32_t pbase[MP];
    int khlo[MP], khhi[MP];
#pragma unroll
    for (int m = 0; m < MP; ++m) {
        const int k = wave + WAVES * m;
        if (k < PX) {
            const int r = 16 * k + (lane >> 2), c = (lane & 3) ^ swz(r);
            const int rk = r / a.RS, col = r - rk * a.RS, g = g0 + rk;
            const int n = g / a.Ho, ho = g - n * a.Ho, wi = col - 1;
            const bool ok = g < NHo && wi >= 0 && wi < a.Wi;
            const int h0 = S * ho - 1;                                  // input row at kernel row 0
            khlo[m] = ok ? max(0, -h0) : 3;
            khhi[m] = ok ? min(3, a.Hi - h0) : 0;
            pbase[m] = ok ? ((uint32_t)(n * a.Hi + h0) * (uint32_t)a.Wi + (uint32_t)wi) * pixb + 16u * c : 0u;
        } else {
            const int r = 16 * (k - PX) + (lane >> 2), c = (lane & 3) ^ swz(r);    // W row r = kw TN + ol
            const int kw = r / TN, ol = r - kw * TN;
            khlo[m] = khhi[m] = 0;
            pbase[m] = (uint32_t)(kw * a.Co + o0 + ol) * 64u + 16u * c;             // row within the stage's block
        }
    }
    const uint32_t rowb = (uint32_t)a.Wi * pixb, wstage = 3u * (uint32_t)a.Co * 64u;
    auto issue = [&](int s) {
        const int kh = s / NQ, q = s - kh * NQ;
        const uint32_t img = lds0 + (s & 1) * STG;
        const uint32_t xadd = (uint32_t)kh * rowb + (uint32_t)(q * 64), wadd = (uint32_t)s * wstage;
#pragma unroll
        for (int m = 0; m < MP; ++m) {
            if (m >= npieces) break;
            const int k = wave + WAVES * m;
            if (k < PX) {
                const bool ok = kh >= khlo[m] && kh < khhi[m];
                dma16(rx, img + k * 1024, ok ? pbase[m] + xadd : OOB);
            } else {
                dma16(rw, img + XIMG + (k - PX) * 1024, pbase[m] + wadd);
            }
        }
    };

    const int wm = wave / WN, wn = wave % WN;
    // the lane's fragment rows: output pixel p = p0 + 64 wm + 32 i + (lane & 31) reads position pos + kw
    int posA[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int p = min(p0 + 64 * wm + 32 * i + (lane & 31), NHWo - 1);
        const int gr = p / a.Wo, wo = p - gr * a.Wo;
        posA[i] = (gr - g0) * a.RS + S * wo;
    }
    const int hc = lane >> 5;                                       // fragment chunk: hi = hc, lo = 2 + hc

    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    issue(0);
    for (int s = 0; s < NSTG; ++s) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // this wave's stage-s pieces have landed
        __builtin_amdgcn_s_barrier();                              // ... every wave's; stage s - 1's buffer is free
        asm volatile("" ::: "memory");
        if (s + 1 < NSTG) issue(s + 1);
        const uint8_t* ximg = lds + (s & 1) * STG;
        const uint8_t* wimg = ximg + XIMG;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
            half8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int r = posA[i] + kw;
                ah[i] = frag(ximg, r, hc);
                al[i] = frag(ximg, r, 2 + hc);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int r = kw * TN + 64 * wn + 32 * j + (lane & 31);
                bh[j] = frag(wimg, r, hc);
                bl[j] = frag(wimg, r, 2 + hc);
            }
            // product-major: consecutive MFMAs feed the 4 blocks' independent accumulators
#pragma unroll
            for (int pr = 0; pr < 3; ++pr)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(pr == 2 ? al[i] : ah[i], pr == 1 ? bl[j] : bh[j],
                                                                           acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        // the buffer is refilled after the next barrier
    }

    // epilogue: acc[i][j] register 4 g + e = pixel p0 + 64 wm + 32 i + 8 g + 4 (lane >> 5) + e, channel
    // o0 + 64 wn + 32 j + (lane & 31): 32 lanes write 128 contiguous bytes of one pixel
    const float scale = __builtin_ldexpf(1.f, -(split_exp(*a.xmax) + split_exp(*a.wmax)));
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int o = o0 + 64 * wn + 32 * j + (lane & 31);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int p = p0 + 64 * wm + 32 * i + 8 * g + 4 * (lane >> 5) + e;
                    if (p < NHWo) a.y[(int64_t)p * a.Co + o] = acc[i][j][4 * g + e] * scale;
                }
    }
}

// ------------------------------------------------------------------------------------------ stride-2 input gradient
// dX[n][y][x][ci] = sum dY[n][ho][wo][co] W[co][ci][kh][kw] over y = 2 ho + kh - 1, x = 2 wo + kw - 1, split by the
// parity (py, px) of (y, x) into 4 phases, each a stride-1 correlation over dY with only the taps of that parity (no
// zero-inserted dY, no MFMA on zeros): phase pixel (n, a, b) = dX pixel (n, 2a + py, 2b + px), output channel o = ci,
// reduction over i = co.  Row taps th: py = 0 -> kh = 1 at dY row a; py = 1 -> kh = 0 at row a + 1, kh = 2 at row a.
// Column taps tw the same for px.  The forward tile's scheme: stage (th, 16-channel chunk q) stages, per output row
// (n, a) of the tile, the dY row segment of RS = Wb + 1 columns b = 0 .. Wb (zeros past Wo), pixel (row k, column b)
// reads position k RS + b + cofs[tw] for its NTW column taps.  One launch covers the 4 phases (heaviest first).
// Weights: avse_sconv_wprep(transposed = 2): per phase ph = 2 py + px, [th][q][tw][o = ci][64 B] (9 taps in all).
struct DArgs {
    const void* dyq;           // Q-split output gradient (N Ho Wo pixels x Co 4 B)
    const void* wq;            // avse_sconv_wprep(transposed = 2) image
    const uint32_t* dymax;
    const uint32_t* wmax;
    float* dx;                 // NHWC fp32 (N Hi Wi x Ci)
    int N, Hi, Wi, O, I, Ho, Wo;
    int tiles_n;               // O / TN
    int tile0[5];              // launch slot -> first workgroup (prefix sums over the tile counts)
    int py[4], px[4], Ha[4], Wb[4], RS[4], npos[4];
    uint32_t woff[4];          // byte offset of the slot's phase image in wq
};

__host__ __device__ inline uint32_t dg2_tap_off(int ph) {      // taps before phase ph in the image: 0, 1, 3, 5
    return ph == 0 ? 0u : ph == 1 ? 1u : ph == 2 ? 3u : 5u;
}

template <int NTH, int NTW, int TN>
__device__ __forceinline__ void dgrad2_body(const DArgs& a, int slot, int tile, uint8_t* lds) {
    constexpr int WAVES = 8, WN = TN / 64, WM = WAVES / WN, TM = 64 * WM;
    constexpr int WIMG = NTW * TN * ROWB, WIMG_MAX = 2 * TN * ROWB;
    constexpr int STG = XIMG + WIMG_MAX;
    constexpr int PW = WIMG / 1024;
    constexpr int MP = (NPOS_MAX / 16 + PW + WAVES - 1) / WAVES;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int py = a.py[slot], px = a.px[slot], Ha = a.Ha[slot], Wb = a.Wb[slot], RS = a.RS[slot];
    const int tn = tile % a.tiles_n, tm = tile / a.tiles_n;
    const int p0 = tm * TM, o0 = tn * TN;
    const int NP = a.N * Ha * Wb, NHa = a.N * Ha;
    const int g0 = p0 / Wb;
    const int NQ = a.I / 16, NSTG = NTH * NQ;
    const i4_t rx = rsrc_of(a.dyq, (int64_t)a.N * a.Ho * a.Wo * a.I * 4);
    const i4_t rw = rsrc_of(a.wq, (int64_t)9 * a.I * a.O * 4);
    const uint32_t lds0 = lds_u32(lds);
    const int PX = a.npos[slot] / 16, PT = PX + PW;
    const int npieces = (PT - wave + WAVES - 1) / WAVES;
    const uint32_t pixb = (uint32_t)a.I * 4u;
    const uint32_t rowb = (uint32_t)a.Wo * pixb;
    // row tap th reads dY row a + rofs(th): rofs = 1 for (py = 1, th = 0), else 0
    uint32_t pbase[MP];
    int thok[MP];                                                  // bit th: the row exists for tap th
#pragma unroll
    for (int m = 0; m < MP; ++m) {
        const int k = wave + WAVES * m;
        if (k < PX) {
            const int r = 16 * k + (lane >> 2), c = (lane & 3) ^ swz(r);
            const int rk = r / RS, col = r - rk * RS, g = g0 + rk;
            const int n = g / Ha, ar = g - n * Ha;
            const bool ok = g < NHa && col < a.Wo;
            int bits = 0;
            if (ok) bits = (NTH == 2) ? ((ar + 1 < a.Ho ? 1 : 0) | 2) : 1;
            thok[m] = bits;
            pbase[m] = ok ? ((uint32_t)(n * a.Ho + ar) * (uint32_t)a.Wo + (uint32_t)col) * pixb + 16u * c : 0u;
        } else {
            const int r = 16 * (k - PX) + (lane >> 2), c = (lane & 3) ^ swz(r);    // W row r = tw TN + ol
            const int tw = r / TN, ol = r - tw * TN;
            thok[m] = 0;
            pbase[m] = a.woff[slot] + (uint32_t)(tw * a.O + o0 + ol) * 64u + 16u * c;
        }
    }
    const uint32_t wstage = (uint32_t)NTW * (uint32_t)a.O * 64u;
    auto issue = [&](int s) {
        const int th = s / NQ, q = s - th * NQ;
        const uint32_t img = lds0 + (s & 1) * STG;
        const uint32_t xadd = (NTH == 2 && th == 0 ? rowb : 0u) + (uint32_t)(q * 64), wadd = (uint32_t)s * wstage;
#pragma unroll
        for (int m = 0; m < MP; ++m) {
            if (m >= npieces) break;
            const int k = wave + WAVES * m;
            if (k < PX) {
                const bool ok = (thok[m] >> th) & 1;
                dma16(rx, img + k * 1024, ok ? pbase[m] + xadd : OOB);
            } else {
                dma16(rw, img + XIMG + (k - PX) * 1024, pbase[m] + wadd);
            }
        }
    };

    const int wm = wave / WN, wn = wave % WN;
    int posA[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int p = min(p0 + 64 * wm + 32 * i + (lane & 31), NP - 1);
        const int gr = p / Wb, b = p - gr * Wb;
        posA[i] = (gr - g0) * RS + b;
    }
    const int hc = lane >> 5;

    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    issue(0);
    for (int s = 0; s < NSTG; ++s) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (s + 1 < NSTG) issue(s + 1);
        const uint8_t* ximg = lds + (s & 1) * STG;
        const uint8_t* wimg = ximg + XIMG;
#pragma unroll
        for (int tw = 0; tw < NTW; ++tw) {
            const int cofs = (NTW == 2 && tw == 0) ? 1 : 0;         // px = 1: kw = 0 reads column b + 1
            half8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int r = posA[i] + cofs;
                ah[i] = frag(ximg, r, hc);
                al[i] = frag(ximg, r, 2 + hc);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int r = tw * TN + 64 * wn + 32 * j + (lane & 31);
                bh[j] = frag(wimg, r, hc);
                bl[j] = frag(wimg, r, 2 + hc);
            }
#pragma unroll
            for (int pr = 0; pr < 3; ++pr)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(pr == 2 ? al[i] : ah[i], pr == 1 ? bl[j] : bh[j],
                                                                           acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }

    // epilogue: phase pixel p -> dX pixel (n, 2 ar + py, 2 b + px); 4 consecutive phase pixels per (i, g)
    const float scale = __builtin_ldexpf(1.f, -(split_exp(*a.dymax) + split_exp(*a.wmax)));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int pf = p0 + 64 * wm + 32 * i + 8 * g + 4 * (lane >> 5);
            int gr = pf / Wb, b = pf - gr * Wb;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int p = pf + e;
                if (p < NP) {
                    const int n = gr / Ha, ar = gr - n * Ha;
                    const int64_t pix = ((int64_t)n * a.Hi + 2 * ar + py) * a.Wi + 2 * b + px;
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int o = o0 + 64 * wn + 32 * j + (lane & 31);
                        a.dx[pix * a.O + o] = acc[i][j][4 * g + e] * scale;
                    }
                }
                if (++b == Wb) {
                    b = 0;
                    ++gr;
                }
            }
        }
}

template <int TN>
__global__ __launch_bounds__(512, 1) void dgrad2_kernel(DArgs a) {
    __shared__ __attribute__((aligned(1024))) uint8_t lds[2 * (XIMG + 2 * TN * ROWB)];
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    int slot = 0;
    while (slot < 3 && bid >= a.tile0[slot + 1]) ++slot;
    const int tile = bid - a.tile0[slot];
    const int nth = a.py[slot] ? 2 : 1, ntw = a.px[slot] ? 2 : 1;
    if (nth == 2 && ntw == 2) dgrad2_body<2, 2, TN>(a, slot, tile, lds);
    else if (nth == 2) dgrad2_body<2, 1, TN>(a, slot, tile, lds);
    else if (ntw == 2) dgrad2_body<1, 2, TN>(a, slot, tile, lds);
    else dgrad2_body<1, 1, TN>(a, slot, tile, lds);
}

// ------------------------------------------------------------------------------------------------ weight gradient
// Per kernel row kh: dW[o][i][kh][kw] for the 3 kw taps, a GEMM with M = o, N = i and the reduction over output pixels.
// Workgroup (pixel-chunk range, o block of OB = 64 or 128, i block of 64, kh): OB / 32 x 2 waves of 32 x 32 (o, i)
// blocks x 3 taps (48 accumulators).  Per 64-pixel raster chunk: the dY rows (64 pixels x the o block) and the input
// segment rows the chunk reads at kernel row kh (positions as in the forward, 256 B each for the i block) staged by
// LDS-DMA; fragments by ds_read_b64_tr_b16 from pixel rows whose 16-B chunk c sits at c ^ ((r & 3) << 2).  Per chunk
// and wave: 4 k-steps x 3 products x 3 taps = 36 MFMAs, issued product-major so that consecutive MFMAs feed the 3
// taps' independent accumulators.  Per-workgroup partial slabs, summed by a second kernel (deterministic).
constexpr int WG_CHUNK = 64;
constexpr int XROWB = 256;                      // staged input position: the 64-channel i block
constexpr int NPW_MAX = 184;                    // staged input positions per chunk (host-checked)

__device__ inline int tswz(int r, int c) { return c ^ ((r & 3) << 2); }

// 32 channels (block cb of a staged row) x 16 pixels, plane pl (0 hi, 1 lo), rows given per lane (dconv.hip tfrag);
// RB = bytes per staged row
template <int RB>
__device__ inline half8 tfrag(const uint8_t* img, const int (&row)[2], int cb, int pl, int lane) {
    const int g = lane >> 4, i = lane & 15;
    const int q = 2 * cb + (g & 1);
    s4_t v[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int r = row[u];
        const int byte = q * 64 + pl * 32 + 8 * (i & 3);
        const int off = r * RB + 16 * tswz(r, byte >> 4) + (byte & 15);
        v[u] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(img + off));
    }
    const s4_t w0 = v[0], w1 = v[1];
    const short __attribute__((ext_vector_type(8))) w = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
    return __builtin_bit_cast(half8, w);
}

struct WArgs {
    const void* xq;
    const void* dyq;
    const uint32_t* xmax;
    const uint32_t* dymax;
    float* part;                 // [ranges][kh][kw][o][i]
    int N, Hi, Wi, Ci, Ho, Wo, Co;
    int RS, npw;                 // staged segment length, positions staged per chunk (multiple of 4, <= NPW_MAX)
    int chunks, ranges, nob, nib;
    int q64, r64;                // WG_CHUNK = q64 Wo + r64
    float inv_ho, inv_wo;
};

template <int S, int OB>
__global__ __launch_bounds__(512, 1) void wgrad_kernel(WArgs a) {
    // 8 waves; wave = 64 o x 32 i (2 x 1 MFMA blocks) x 3 taps: OB / 32 waves cover the (OB, 64) block, and the
    // KG = 8 / (OB / 32) copies take disjoint k-steps of every chunk (KG partial slabs per range).  Round 5's wave of
    // 32 o x 32 i read and addressed its X fragments for one o block only: with ~900 address / DMA-issue instructions
    // per 36 MFMAs the kernel was instruction-issue bound (MFMA busy 0.24, r06f PMC).
    constexpr int BW = OB / 32, KG = 8 / BW, WAVES = 8, YRB = OB * 4, KS = (WG_CHUNK / 16) / KG;   // KS k-steps per wave
    constexpr int YIMG = WG_CHUNK * YRB, STG = YIMG + NPW_MAX * XROWB;
    constexpr int PY = YIMG / 1024, YPP = 1024 / YRB;             // dY pieces; pixels per piece
    constexpr int MP = (PY + NPW_MAX / 4 + WAVES - 1) / WAVES;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[2 * STG];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    int t = bid;
    const int kh = t % 3;
    t /= 3;
    const int ib = t % a.nib;
    t /= a.nib;
    const int ob = t % a.nob;
    const int r = t / a.nob;
    const int c_lo = (int)((int64_t)r * a.chunks / a.ranges), c_hi = (int)((int64_t)(r + 1) * a.chunks / a.ranges);
    const int NHWo = a.N * a.Ho * a.Wo, NHo = a.N * a.Ho;
    const i4_t rx = rsrc_of(a.xq, (int64_t)a.N * a.Hi * a.Wi * a.Ci * 4);
    const i4_t ry = rsrc_of(a.dyq, (int64_t)NHWo * a.Co * 4);
    const uint32_t lds0 = lds_u32(lds);
    const int PT = PY + a.npw / 4;
    const int npieces = (PT - wave + WAVES - 1) / WAVES;
    const uint32_t xpixb = (uint32_t)a.Ci * 4u, ypixb = (uint32_t)a.Co * 4u;
    const int ypr = lane / (YRB / 16), ypc = lane % (YRB / 16);  // dY piece lane: pixel of the piece, physical chunk
    const int xpr = lane >> 4, xpc = lane & 15;                    // X piece lane: position of the piece, chunk

    // per DMA piece of this wave, everything that does not depend on the chunk: dY pieces: the lane's chunk pixel j and
    // its byte offset within the chunk's dY rows; X pieces: the staged position's row of the chunk's segment list and
    // the byte offset of its input column within an input row (OOB for padding columns and positions past npw)
    int pj[MP];
    uint32_t poff[MP];
#pragma unroll
    for (int m = 0; m < MP; ++m) {
        const int k = wave + WAVES * m;
        if (k < PY) {
            const int j = YPP * k + ypr;
            pj[m] = j;
            poff[m] = (uint32_t)j * ypixb + (uint32_t)(ob * YRB) + 16u * tswz(j, ypc);
        } else {
            const int q = 4 * (k - PY) + xpr;
            const int rk = q / a.RS, wi = q - rk * a.RS - 1;
            const bool ok = q < a.npw && wi >= 0 && wi < a.Wi;
            pj[m] = rk;
            poff[m] = ok ? (uint32_t)wi * xpixb + (uint32_t)(ib * XROWB) + 16u * tswz(q, xpc) : OOB;
        }
    }
    const uint32_t xrowb = (uint32_t)a.Wi * xpixb;                // bytes per input row
    // the chunks' first output row g0 (flat n, ho) and column w0 advance by WG_CHUNK pixels = q64 rows + r64 columns
    struct Cur {
        int g0, w0;
    };
    auto cur_at = [&](int c) {
        Cur cu;
        const int p0 = c * WG_CHUNK;
        cu.g0 = p0 / a.Wo;
        cu.w0 = p0 - cu.g0 * a.Wo;
        return cu;
    };
    auto cur_next = [&](Cur& cu) {
        cu.w0 += a.r64;
        cu.g0 += a.q64;
        if (cu.w0 >= a.Wo) {
            cu.w0 -= a.Wo;
            ++cu.g0;
        }
    };
    auto issue = [&](int c, const Cur& cu, int buf) {
        const int p0 = c * WG_CHUNK, g0 = cu.g0;
        const uint32_t ybase = (uint32_t)p0 * ypixb;
        int n0, ho0;
        divmod_small(g0, a.Ho, a.inv_ho, n0, ho0);
        const uint32_t img = lds0 + buf * STG;
#pragma unroll
        for (int m = 0; m < MP; ++m) {
            if (m >= npieces) break;
            const int k = wave + WAVES * m;
            if (k < PY) {                                        // dY rows: chunk pixel pj
                dma16(ry, img + k * 1024, p0 + pj[m] < NHWo ? ybase + poff[m] : OOB);
            } else {                                             // input position of segment row pj at kernel row kh
                int dn = 0, ho = ho0 + pj[m];
                if (ho >= a.Ho) divmod_small(ho, a.Ho, a.inv_ho, dn, ho);
                const int hi = S * ho - 1 + kh;
                const bool ok = poff[m] != OOB && g0 + pj[m] < NHo && hi >= 0 && hi < a.Hi;
                const uint32_t off = (uint32_t)((n0 + dn) * a.Hi + hi) * xrowb + poff[m];
                dma16(rx, img + YIMG + (k - PY) * 1024, ok ? off : OOB);
            }
        }
    };

    const int kg = wave / BW, lw = wave % BW;
    const int obw = lw >> 1, ibw = lw & 1;                       // this wave's 64 o (blocks 2 obw, 2 obw + 1) x 32 i
    floatx16 acc[2][3];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[t][k][e] = 0.f;

    const int g = lane >> 4, li = lane & 15;
    Cur ci_ = cur_at(c_lo), cc_ = ci_;                           // issue and compute cursors
    if (c_lo < c_hi) {
        issue(c_lo, ci_, 0);
        cur_next(ci_);
    }
    for (int c = c_lo; c < c_hi; ++c) {
        const int it = c - c_lo;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (c + 1 < c_hi) {
            issue(c + 1, ci_, (it + 1) & 1);
            cur_next(ci_);
        }
        const uint8_t* yimg = lds + (it & 1) * STG;
        const uint8_t* ximg = yimg + YIMG;
        const int w0 = cc_.w0;
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            const int s = kg * KS + s2;
            int ry_[2], rx_[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int j = 16 * s + 8 * (g >> 1) + (li >> 2) + 4 * u;       // the lane's pixel of the k-step
                int dr, wo;
                divmod_small(w0 + j, a.Wo, a.inv_wo, dr, wo);
                ry_[u] = j;
                rx_[u] = dr * a.RS + S * wo;
            }
            half8 ah[2], al[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                ah[t] = tfrag<YRB>(yimg, ry_, 2 * obw + t, 0, lane);
                al[t] = tfrag<YRB>(yimg, ry_, 2 * obw + t, 1, lane);
            }
            half8 bh[3], bl[3];
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const int rk[2] = {rx_[0] + kw, rx_[1] + kw};
                bh[kw] = tfrag<XROWB>(ximg, rk, ibw, 0, lane);
                bl[kw] = tfrag<XROWB>(ximg, rk, ibw, 1, lane);
            }
            // product-major over the 6 independent accumulators
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int kw = 0; kw < 3; ++kw)
                    acc[t][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t], bh[kw], acc[t][kw], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int kw = 0; kw < 3; ++kw)
                    acc[t][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t], bl[kw], acc[t][kw], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int kw = 0; kw < 3; ++kw)
                    acc[t][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[t], bh[kw], acc[t][kw], 0, 0, 0);
        }
        cur_next(cc_);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    // partial tiles: acc[t][kw] register 4 q + e = row o = OB ob + 64 obw + 32 t + 8 q + 4 (lane >> 5) + e, column
    // i = 64 ib + 32 ibw + (lane & 31)
    const float sc = __builtin_ldexpf(1.f, -(split_exp(*a.xmax) + split_exp(*a.dymax)));
    float* pp = a.part + ((int64_t)(r * KG + kg) * 9 + kh * 3) * a.Co * a.Ci;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int o = OB * ob + 64 * obw + 32 * t + 8 * q + 4 * (lane >> 5) + e;
                    const int i = 64 * ib + 32 * ibw + (lane & 31);
                    pp[((int64_t)kw * a.Co + o) * a.Ci + i] = acc[t][kw][4 * q + e] * sc;
                }
}

// dW[o][i][kh][kw] = sum over ranges of part[range][kh][kw][o][i]: workgroup = 64 consecutive elements x 4 range
// slices (coalesced 256-B reads per slice and range), the slices combined in a fixed order (deterministic)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int ranges, int Co, int Ci,
                                                           float* __restrict__ dw) {
    __shared__ float red[4][64];
    const int64_t total = (int64_t)9 * Co * Ci;
    const int64_t idx = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const int sl = threadIdx.x >> 6;
    float v = 0.f;
    if (idx < total)
        for (int g = sl; g < ranges; g += 4) v += part[(int64_t)g * total + idx];
    red[sl][threadIdx.x & 63] = v;
    __syncthreads();
    if (sl == 0 && idx < total) {
        v = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
        const int i = (int)(idx % Ci), o = (int)((idx / Ci) % Co), tap = (int)(idx / ((int64_t)Ci * Co));
        dw[((int64_t)o * Ci + i) * 9 + tap] = v;
    }
}

// ------------------------------------------------------------------------------------------------ weights
__global__ void wmax_kernel(const float* w, int n, uint32_t* out) {
    __shared__ uint32_t red[4];
    float m = 0.f;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) m = fmaxf(m, fabsf(w[i]));
    uint32_t b = __float_as_uint(m);
    for (int o = 32; o >= 1; o >>= 1) b = max(b, (uint32_t)__shfl_xor((int)b, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        b = max(max(red[0], red[1]), max(red[2], red[3]));
        if (b) atomicMax(out, b);
    }
}

// W (Co, Ci, 3, 3) fp32 -> [kh][q][kw][o][hi 16 | lo 16]; transposed: the input gradient's W'[o = ci][i = co][kh][kw] =
// W[co][ci][2 - kh][2 - kw] (then o runs over Ci and i over Co of W)
__global__ void wsplit_kernel(const float* w, int Co, int Ci, int transposed, const uint32_t* maxbits, uint16_t* wq) {
    const int O = transposed ? Ci : Co, I = transposed ? Co : Ci, NQ = I / 16;
    const int64_t total = (int64_t)9 * O * I;
    const float sc = __builtin_ldexpf(1.f, split_exp(*maxbits));
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(e % 16);
        const int64_t rrow = e / 16;                            // ((kh NQ + q) 3 + kw) O + o
        const int o = (int)(rrow % O), kw = (int)((rrow / O) % 3), s = (int)(rrow / ((int64_t)O * 3));
        const int kh = s / NQ, q = s % NQ, i = q * 16 + c;
        const float v = transposed ? w[(((int64_t)i * Ci + o) * 3 + (2 - kh)) * 3 + (2 - kw)]
                                   : w[(((int64_t)o * Ci + i) * 3 + kh) * 3 + kw];
        const float sv = v * sc;
        const _Float16 h = (_Float16)sv, l = (_Float16)(sv - (float)h);
        wq[rrow * 32 + c] = __builtin_bit_cast(uint16_t, h);
        wq[rrow * 32 + 16 + c] = __builtin_bit_cast(uint16_t, l);
    }
}

// W (Co, Ci, 3, 3) fp32 -> the stride-2 input gradient's phase images: phase ph = 2 py + px at tap offset
// dg2_tap_off(ph), [th][q][tw][o = ci][hi 16 | lo 16] over i = co (q = co / 16); kh = py ? (th ? 2 : 0) : 1, kw likewise
__global__ void wsplit_dgrad2_kernel(const float* w, int Co, int Ci, const uint32_t* maxbits, uint16_t* wq) {
    const int O = Ci, NQ = Co / 16;
    const int64_t tap = (int64_t)O * Co;                        // (o, i) elements per tap
    const int64_t total = 9 * tap;
    const float sc = __builtin_ldexpf(1.f, split_exp(*maxbits));
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(e % 16);
        const int64_t rrow = e / 16;                            // row of 16 channels over the whole image
        const int64_t t9 = rrow / (tap / 16);                   // global tap index 0 .. 8
        const int ph = t9 < 1 ? 0 : t9 < 3 ? 1 : t9 < 5 ? 2 : 3;
        const int py = ph >> 1, px = ph & 1, ntw = px ? 2 : 1;
        const int64_t lr = rrow - (int64_t)dg2_tap_off(ph) * (tap / 16);     // row within the phase image
        const int o = (int)(lr % O);
        const int64_t u = lr / O;                               // (th NQ + q) NTW + tw
        const int tw = (int)(u % ntw);
        const int64_t sq = u / ntw;
        const int q = (int)(sq % NQ), th = (int)(sq / NQ);
        const int kh = py ? (th ? 2 : 0) : 1, kw = px ? (tw ? 2 : 0) : 1;
        const int i = q * 16 + c;
        const float sv = w[(((int64_t)i * Ci + o) * 3 + kh) * 3 + kw] * sc;
        const _Float16 h = (_Float16)sv, l = (_Float16)(sv - (float)h);
        wq[rrow * 32 + c] = __builtin_bit_cast(uint16_t, h);
        wq[rrow * 32 + 16 + c] = __builtin_bit_cast(uint16_t, l);
    }
}

inline int out_dim(int x, int s) { return (x - 1) / s + 1; }     // k 3, padding 1

// forward geometry: the tile's rows span at most (TM - 1 + Wo - 1) / Wo + 1 output rows
inline int fwd_npos(int TM, int Wo, int RS) {
    const int rows = (TM - 1 + Wo - 1) / Wo + 1;
    return (rows * RS + 15) / 16 * 16;
}
inline int wg_npw(int Wo, int RS) {
    const int rows = (WG_CHUNK - 1 + Wo - 1) / Wo + 1;
    return (rows * RS + 3) / 4 * 4;
}
inline int wg_ranges(int chunks, int blocks_per_range) {
    return std::max(1, std::min(chunks, (512 + blocks_per_range - 1) / blocks_per_range));
}

}  // namespace scv
}  // namespace avse

using namespace avse::scv;

extern "C" {

int64_t avse_sconv_wprep_bytes(int64_t co, int64_t ci) { return 9 * co * ci * 4; }

int avse_sconv_wprep(int64_t co, int64_t ci, const float* w, int32_t transposed, void* wq, uint32_t* wmax,
                     avse_stream_t stream) {
    if (!w || !wq || !wmax) return AVSE_EINVAL;
    if (co <= 0 || ci <= 0 || co % 64 || ci % 64 || co > 4096 || ci > 4096) return AVSE_ESHAPE;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(wmax, 0, 4, st) != hipSuccess) return AVSE_ELAUNCH;
    const int n = (int)(9 * co * ci);
    hipLaunchKernelGGL(wmax_kernel, dim3((unsigned)std::min(256, (n + 255) / 256)), dim3(256), 0, st, w, n, wmax);
    AVSE_CHECK_LAUNCH();
    if (transposed == 2)
        hipLaunchKernelGGL(wsplit_dgrad2_kernel, dim3((unsigned)std::min(2048, (n + 255) / 256)), dim3(256), 0, st, w,
                           (int)co, (int)ci, wmax, reinterpret_cast<uint16_t*>(wq));
    else
        hipLaunchKernelGGL(wsplit_kernel, dim3((unsigned)std::min(2048, (n + 255) / 256)), dim3(256), 0, st, w, (int)co,
                           (int)ci, transposed, wmax, reinterpret_cast<uint16_t*>(wq));
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

// stride-2 input gradient geometry; AVSE_ESHAPE when the kernel does not take the shape
static int dg2_setup(int64_t N, int64_t Hi, int64_t Wi, int64_t ci, int64_t co, DArgs& a, int& TN) {
    if (N <= 0 || Hi <= 0 || Wi <= 0 || ci <= 0 || co <= 0 || ci % 64 || co % 64 || ci > 4096 || co > 4096)
        return AVSE_ESHAPE;
    if (N * Hi * Wi * ci * 4 >= (1LL << 31) - 4096 || N * Hi * Wi * co * 4 >= (1LL << 31) - 4096) return AVSE_ESHAPE;
    a.N = (int)N;
    a.Hi = (int)Hi;
    a.Wi = (int)Wi;
    a.O = (int)ci;
    a.I = (int)co;
    a.Ho = out_dim((int)Hi, 2);
    a.Wo = out_dim((int)Wi, 2);
    TN = ci % 128 ? 64 : 128;
    const int TM = TN == 64 ? 512 : 256;
    a.tiles_n = (int)(ci / TN);
    static const int order[4] = {3, 2, 1, 0};                   // heaviest phase first
    int64_t t0 = 0;
    for (int s = 0; s < 4; ++s) {
        const int ph = order[s], py = ph >> 1, px = ph & 1;
        a.py[s] = py;
        a.px[s] = px;
        a.Ha[s] = ((int)Hi - py + 1) / 2;
        a.Wb[s] = ((int)Wi - px + 1) / 2;
        a.RS[s] = a.Wb[s] + 1;
        a.woff[s] = dg2_tap_off(ph) * (uint32_t)(ci * co * 4);
        a.tile0[s] = (int)t0;
        const int64_t np = N * a.Ha[s] * a.Wb[s];
        a.npos[s] = np > 0 ? fwd_npos(TM, a.Wb[s], a.RS[s]) : 0;
        if (a.npos[s] > NPOS_MAX) return AVSE_ESHAPE;
        t0 += (np + TM - 1) / TM * a.tiles_n;
        if (t0 >= (1LL << 31)) return AVSE_ESHAPE;
    }
    a.tile0[4] = (int)t0;
    return AVSE_OK;
}

int avse_sconv_dgrad2_supported(int64_t N, int64_t Hi, int64_t Wi, int64_t ci, int64_t co) {
    DArgs a;
    int TN;
    return dg2_setup(N, Hi, Wi, ci, co, a, TN) == AVSE_OK ? 1 : 0;
}

int avse_sconv_dgrad2(int64_t N, int64_t Hi, int64_t Wi, int64_t ci, int64_t co, const void* dyq,
                      const uint32_t* dymax, const void* wq, const uint32_t* wmax, float* dx, avse_stream_t stream) {
    if (!dyq || !dymax || !wq || !wmax || !dx) return AVSE_EINVAL;
    DArgs a;
    int TN;
    const int rc = dg2_setup(N, Hi, Wi, ci, co, a, TN);
    if (rc != AVSE_OK) return rc;
    a.dyq = dyq;
    a.wq = wq;
    a.dymax = dymax;
    a.wmax = wmax;
    a.dx = dx;
    if (a.tile0[4] == 0) return AVSE_OK;
    const dim3 grid((unsigned)a.tile0[4]), block(512);
    hipStream_t st = (hipStream_t)stream;
    if (TN == 64) hipLaunchKernelGGL((dgrad2_kernel<64>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((dgrad2_kernel<128>), grid, block, 0, st, a);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_sconv_fwd(int64_t N, int64_t Hi, int64_t Wi, int64_t ci, int64_t co, int64_t stride, const void* xq,
                   const uint32_t* xmax, const void* wq, const uint32_t* wmax, float* y, avse_stream_t stream) {
    if (!xq || !xmax || !wq || !wmax || !y) return AVSE_EINVAL;
    if (N <= 0 || Hi <= 0 || Wi <= 0 || ci <= 0 || co <= 0 || ci % 64 || co % 64 || (stride != 1 && stride != 2))
        return AVSE_ESHAPE;
    if (N * Hi * Wi * ci * 4 >= (1LL << 31) - 4096 || 9 * ci * co * 4 >= (1LL << 31)) return AVSE_ESHAPE;
    FArgs a;
    a.xq = xq;
    a.wq = wq;
    a.xmax = xmax;
    a.wmax = wmax;
    a.y = y;
    a.N = (int)N;
    a.Hi = (int)Hi;
    a.Wi = (int)Wi;
    a.Ci = (int)ci;
    a.Co = (int)co;
    a.Ho = out_dim((int)Hi, (int)stride);
    a.Wo = out_dim((int)Wi, (int)stride);
    a.RS = (int)stride * a.Wo + 2;
    const int TN = co % 128 ? 64 : 128, TM = TN == 64 ? 512 : 256;
    a.npos = fwd_npos(TM, a.Wo, a.RS);
    if (a.npos > NPOS_MAX) return AVSE_ESHAPE;
    const int64_t NHWo = N * a.Ho * a.Wo;
    if (NHWo * co >= (1LL << 31)) return AVSE_ESHAPE;
    a.tiles_n = (int)(co / TN);
    const int64_t tiles = (NHWo + TM - 1) / TM * a.tiles_n;
    if (tiles >= (1LL << 31)) return AVSE_ESHAPE;
    const dim3 grid((unsigned)tiles), block(512);
    hipStream_t st = (hipStream_t)stream;
    if (stride == 1) {
        if (TN == 64) hipLaunchKernelGGL((fwd_kernel<1, 64>), grid, block, 0, st, a);
        else hipLaunchKernelGGL((fwd_kernel<1, 128>), grid, block, 0, st, a);
    } else {
        if (TN == 64) hipLaunchKernelGGL((fwd_kernel<2, 64>), grid, block, 0, st, a);
        else hipLaunchKernelGGL((fwd_kernel<2, 128>), grid, block, 0, st, a);
    }
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

static int wg_setup(int64_t N, int64_t Hi, int64_t Wi, int64_t ci, int64_t co, int64_t stride, WArgs& a) {
    if (N <= 0 || Hi <= 0 || Wi <= 0 || ci <= 0 || co <= 0 || ci % 64 || co % 64 || (stride != 1 && stride != 2))
        return AVSE_ESHAPE;
    if (N * Hi * Wi * ci * 4 >= (1LL << 31) - 4096) return AVSE_ESHAPE;
    a.N = (int)N;
    a.Hi = (int)Hi;
    a.Wi = (int)Wi;
    a.Ci = (int)ci;
    a.Co = (int)co;
    a.Ho = out_dim((int)Hi, (int)stride);
    a.Wo = out_dim((int)Wi, (int)stride);
    a.RS = (int)stride * a.Wo + 2;
    a.npw = wg_npw(a.Wo, a.RS);
    if (a.npw > NPW_MAX) return AVSE_ESHAPE;
    const int64_t NHWo = N * a.Ho * a.Wo;
    if (NHWo * co * 4 >= (1LL << 31) - 4096) return AVSE_ESHAPE;
    a.chunks = (int)((NHWo + WG_CHUNK - 1) / WG_CHUNK);
    a.nob = (int)(co % 128 ? co / 64 : co / 128);               // o blocks of OB = 128 when they tile co, else 64
    a.nib = (int)(ci / 64);
    a.ranges = wg_ranges(a.chunks, 3 * a.nob * a.nib);
    a.inv_ho = 1.f / (float)a.Ho;
    a.inv_wo = 1.f / (float)a.Wo;
    a.q64 = WG_CHUNK / a.Wo;
    a.r64 = WG_CHUNK % a.Wo;
    return AVSE_OK;
}

// k-step groups of the weight-gradient kernel (partial slabs per range): 8 / (OB / 32)
static int wg_kg(int64_t co) { return co % 128 ? 4 : 2; }

int64_t avse_sconv_wgrad_workspace_bytes(int64_t N, int64_t Hi, int64_t Wi, int64_t ci, int64_t co, int64_t stride) {
    WArgs a;
    if (wg_setup(N, Hi, Wi, ci, co, stride, a) != AVSE_OK) return -1;
    return (int64_t)a.ranges * wg_kg(co) * 9 * co * ci * 4;               // KG partial slabs per range
}

int avse_sconv_wgrad(int64_t N, int64_t Hi, int64_t Wi, int64_t ci, int64_t co, int64_t stride, const void* xq,
                     const uint32_t* xmax, const void* dyq, const uint32_t* dymax, float* dw, float* workspace,
                     avse_stream_t stream) {
    if (!xq || !xmax || !dyq || !dymax || !dw || !workspace) return AVSE_EINVAL;
    WArgs a;
    const int rc = wg_setup(N, Hi, Wi, ci, co, stride, a);
    if (rc != AVSE_OK) return rc;
    a.xq = xq;
    a.dyq = dyq;
    a.xmax = xmax;
    a.dymax = dymax;
    a.part = workspace;
    const bool ob128 = co % 128 == 0;
    const dim3 grid((unsigned)(a.ranges * 3 * a.nob * a.nib)), block(512);
    hipStream_t st = (hipStream_t)stream;
    if (ob128) {
        if (stride == 1) hipLaunchKernelGGL((wgrad_kernel<1, 128>), grid, block, 0, st, a);
        else hipLaunchKernelGGL((wgrad_kernel<2, 128>), grid, block, 0, st, a);
    } else {
        if (stride == 1) hipLaunchKernelGGL((wgrad_kernel<1, 64>), grid, block, 0, st, a);
        else hipLaunchKernelGGL((wgrad_kernel<2, 64>), grid, block, 0, st, a);
    }
    AVSE_CHECK_LAUNCH();
    const int64_t total = 9 * co * ci;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((total + 63) / 64)), dim3(256), 0, st, a.part,
                       a.ranges * wg_kg(co), (int)co, (int)ci, dw);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
