// Forward and input gradient of the avse1 AudioFeatNet dilated convolutions for gfx950, as an implicit GEMM on the
// fp16 MFMA with fp32-accurate split operands ("fp16x3").
//
// Replaces the forward and the data-gradient halves of nn.Conv2d(64, 64, 5, padding=2d, dilation=d), d = 2, 4, 8, 16 —
// conv2..conv5 of /root/reference/baseline/avse1/model.py:199-215 (AudioFeatNet, built in the loop at :202-209).  MIOpen
// ran them at 0.6-0.8 of the fp32 MFMA peak (29 + 27 ms of the 145 ms avse1 C2 step, profiles/r04p_*).
//
//   Y[n][h][w][o] = sum_{i,kh,kw} X[n][h + d (kh - 2)][w + d (kw - 2)][i] * W[o][i][kh][kw]      (0 outside the image)
//   input gradient: the same with X = dY and W'[o = ci][i = co][kh][kw] = W[co][ci][4 - kh][4 - kw]
//
// Precision: the fp32 MFMA (v_mfma_f32_32x32x2_f32) runs at 1/16 of the f16 rate.  Each fp32 operand is split into
// two fp16 values after a power-of-two scale 2^e that puts the tensor's max |x| in [2^14, 2^15):
//   hi = fp16(x 2^e), lo = fp16(x 2^e - hi)        (22 significant bits; hi <= 2^15 cannot overflow)
// and each product is formed as hi*hi + hi*lo + lo*hi: three v_mfma_f32_32x32x16_f16 (exact 22-bit products, fp32
// accumulation), dropping lo*lo (2^-22 of the product).  The representation error (2^-22 relative per operand) is below
// the fp32 accumulation error of a K = 1600 dot product, so the result has fp32 accuracy at 16/3 = 5.3x the fp32 MFMA
// rate.  Elements far below the tensor's max keep an absolute error of 2^-25 of the scaled unit (fp16 subnormals).
//
// Operands: X (and dY) are split once into the "Q4" layout: per pixel 4 channel quarters of 64 B = [hi 16 ci][lo 16 ci]
// (avse_split16: absmax pass, then the split; the same 256 B per pixel as fp32).  W is split into
// [stage = kh * 4 + quarter][kw][o][hi 16 | lo 16] (avse_dconv_wprep), 20 KB per stage.
//
// Work decomposition: workgroup = 256 consecutive output pixels of one image in raster order (they span one row or
// the end of one and the start of the next, W = 257 > 256) x all 64 output channels; 4 waves, wave w = pixels
// 64 w .. 64 w + 63 (2 MFMA blocks) x 64 channels (2 blocks): 64 accumulators per lane.  The reduction runs in 20
// stages (kernel row kh x channel quarter q); per stage the input segment is staged once for all 5 kw taps: the tile's
// pixels of row h, shifted by d (kh - 2), with the 2d halo on both sides, at LDS positions 0 .. nA + 4d, and for a
// two-row tile the next row's pixels behind a 4d gap, so that output pixel j reads position pos(j) + d kw for tap kw
// (pos(j) = j, or j + 4d in the second row) and the halo columns outside the image stage as zeros.  Per stage and
// wave: 5 taps x 2 x 2 blocks x 3 products = 60 MFMAs on 8 fragment reads per tap.  Stages are staged HBM/L2 -> LDS
// by LDS-DMA (buffer_load_dwordx4 ... lds, out-of-image pixels read past the buffer range and land as 0) into a ring
// of 3 buffers, issued 2 stages ahead; one barrier per stage.  LDS rows are 64 B with the 16-B chunk c of row r at
// c ^ ((r >> 2) & 3), so the 16 lanes of a ds_read_b128 group read 16 distinct bank slots.
#include <algorithm>

#include "common.h"

namespace avse {
namespace dcf {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef int i4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int C = 64, KS = 5, NQ = 4, TP = 256, THREADS = 256, WAVES = THREADS / 64;
constexpr int ROWB = 64;                       // LDS bytes per staged row (position or W row): hi 16 | lo 16 channels
constexpr int WIMG = KS * C * ROWB;            // one stage's W image: 5 taps x 64 output channels (20 KB)
constexpr int NSTG = KS * NQ;                  // stages per tile
constexpr int MAXD = 16;
constexpr int XIMG_MAX = (TP + 8 * MAXD) * ROWB;
constexpr int STAGE = XIMG_MAX + WIMG;         // ring slot (44 KB)
constexpr int NBUF = 3;
constexpr int MAXP = (XIMG_MAX + WIMG) / 1024 / WAVES + 1;   // LDS-DMA pieces per wave and stage (<= 11)
static_assert(NBUF * STAGE <= 160 * 1024, "LDS");

__device__ inline int swz(int r) { return (r >> 2) & 3; }

// power-of-two scale exponent e for a tensor whose max |x| has the float bits mb: max 2^e in [2^14, 2^15)
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

// one 16-B-per-lane LDS-DMA wave-instruction: LDS[lds_addr + 16 lane] = buffer[voff] (0 past the range).  Inline asm:
// the compiler's LDS-DMA builtin makes it wait vmcnt(0) before every ds_read of the array.  Nothing else uses M0.
__device__ inline void dma16(i4_t r, uint32_t lds_addr, uint32_t voff) {
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(r), "s"(lds_addr)
                 : "memory");
}

__device__ inline uint32_t lds_u32(const void* p) {
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const lds_void_t*)p);
}

// s_waitcnt vmcnt(n) for a wave-uniform n in 0 .. 12 (the immediate must be a constant)
__device__ inline void wait_all_but(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
        case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
        case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    }
}

__device__ inline half8 frag(const uint8_t* img, int row, int c) {
    return *reinterpret_cast<const half8*>(img + row * ROWB + 16 * (c ^ swz(row)));
}

struct Args {
    const void* xq;              // Q4 split input (n_pix x 256 B)
    const void* wq;              // prepped weights (NSTG x WIMG)
    const uint32_t* maxbits;     // [0] = max |x| bits, [1] = max |w| bits
    const float* bias;           // (64) or NULL
    float* y;                    // NHWC fp32
    int N, H, W, tiles;          // tiles per image
};

// NW waves, tile = TP = 64 NW raster pixels spanning up to NSEG rows (W >= 256): row segment k of the tile sits at LDS
// positions S_k .. S_k + n_k + 4 D (its n_k pixels with the 2 D halo each side), S_k = n_0 + .. + n_{k-1} + 4 D k, so
// output pixel j of segment k reads position j + 4 D k + D kw for tap kw.
// WGS workgroups per CU: 2 (NW = 4) takes 2 LDS buffers, so that two workgroups fit; 1: 3 buffers where they fit.
template <int D, int NW, int WGS = 1>
__global__ __launch_bounds__(64 * NW, WGS) void fwd_kernel(Args a) {
    constexpr int TPX = 64 * NW, NSEG = NW == 4 ? 2 : 3;
    constexpr int NP = (TPX + 4 * D * NSEG + 15) / 16 * 16;   // staged positions (whole 1-KB DMA pieces)
    constexpr int XIMG = NP * ROWB;
    constexpr int STG = XIMG + WIMG;
    constexpr int NB = WGS == 2 ? 2 : ((3 * STG <= 160 * 1024) ? 3 : 2);
    constexpr int PX = XIMG / 1024, PT = PX + WIMG / 1024;      // X pieces, all pieces of a stage
    constexpr int MP = PT / NW + 1;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[NB * STG];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int n = bid / a.tiles, t = bid % a.tiles;
    const int HW = a.H * a.W;
    const int p0 = t * TPX;
    const int r0 = p0 / a.W, w0 = p0 - r0 * a.W;
    // pixels of the tile in its first, second and third row, and the segments' first positions
    const int n0 = min(TPX, a.W - w0), n1 = min(TPX - n0, a.W), n2 = TPX - n0 - n1;
    const int S1 = n0 + 4 * D, S2 = n0 + n1 + 8 * D;
    const i4_t rx = rsrc_of(a.xq, (int64_t)a.N * HW * 256);
    const i4_t rw = rsrc_of(a.wq, (int64_t)NSTG * WIMG);
    const uint32_t lds0 = lds_u32(lds);

    // this wave's LDS-DMA pieces of a stage: k = wave + NW m; X pieces (k < PX) carry the lane's position column (or -1
    // outside the image / the segments) and row; W pieces the lane's byte offset in the stage's W image
    int pcol[MP], prow[MP];
    uint32_t pchunk[MP];
    const int npieces = (PT - wave + NW - 1) / NW;
#pragma unroll
    for (int m = 0; m < MP; ++m) {
        const int k = wave + NW * m;
        if (k < PX) {
            const int r = 16 * k + (lane >> 2), c = (lane & 3) ^ swz(r);
            int col, row;
            if (r < S1) {
                col = w0 - 2 * D + r;
                row = r0;
            } else if (r < S2 || NSEG == 2) {
                col = -2 * D + (r - S1);
                row = (n1 > 0 && r < S1 + n1 + 4 * D) ? r0 + 1 : -1000000;
            } else {
                col = -2 * D + (r - S2);
                row = (n2 > 0 && r < S2 + n2 + 4 * D) ? r0 + 2 : -1000000;
            }
            pcol[m] = (col >= 0 && col < a.W) ? col : -1;
            prow[m] = row;
            pchunk[m] = 16u * c;
        } else {
            const int r = 16 * (k - PX) + (lane >> 2), c = (lane & 3) ^ swz(r);
            pcol[m] = 0;
            prow[m] = 0;
            pchunk[m] = (uint32_t)(r * ROWB + 16 * c);
        }
    }
    auto issue = [&](int s) {
        const int kh = s / NQ, q = s % NQ;
        const uint32_t img = lds0 + (s % NB) * STG;
#pragma unroll
        for (int m = 0; m < MP; ++m) {
            if (m >= npieces) break;
            const int k = wave + NW * m;
            if (k < PX) {
                const int row = prow[m] + D * (kh - 2);
                const bool ok = pcol[m] >= 0 && row >= 0 && row < a.H;
                const uint32_t pix = ((uint32_t)n * (uint32_t)a.H + (uint32_t)row) * (uint32_t)a.W + (uint32_t)pcol[m];
                const uint32_t off = ok ? pix * 256u + (uint32_t)(q * 64) + pchunk[m] : 0x7FFFFFF0u;
                dma16(rx, img + k * 1024, off);
            } else {
                dma16(rw, img + XIMG + (k - PX) * 1024, (uint32_t)(s * WIMG) + pchunk[m]);
            }
        }
    };

    // the lane's fragment rows: output pixel j = 64 wave + 32 i + (lane & 31) reads position pos(j) + D kw
    int posA[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int j = 64 * wave + 32 * i + (lane & 31);
        posA[i] = j + 4 * D * ((j >= n0) + (j >= n0 + n1));
    }
    const int hc = lane >> 5;                   // fragment chunk: hi = hc, lo = 2 + hc

    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    issue(0);
    if (NB == 3) issue(1);
    for (int s = 0; s < NSTG; ++s) {
        // this wave's stage-s pieces have landed (with 3 buffers stage s + 1 may still fly); the barrier makes that
        // hold for every wave and releases the buffer of stage s - 1 (3 buffers) or s - 1 = s + 1 (2 buffers)
        if (NB == 3 && s + 1 < NSTG) wait_all_but(npieces);
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (s + NB - 1 < NSTG) issue(s + NB - 1);
        const uint8_t* ximg = lds + (s % NB) * STG;
        const uint8_t* wimg = ximg + XIMG;
#pragma unroll
        for (int kw = 0; kw < KS; ++kw) {
            half8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int r = posA[i] + D * kw;
                ah[i] = frag(ximg, r, hc);
                al[i] = frag(ximg, r, 2 + hc);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int r = kw * C + 32 * j + (lane & 31);
                bh[j] = frag(wimg, r, hc);
                bl[j] = frag(wimg, r, 2 + hc);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
                }
        }
        if (NB == 2) {                                 // the next issue refills this buffer: every wave must be done
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }

    // epilogue: acc[i][j] register 4 g + e = pixel 64 wave + 32 i + 8 g + 4 (lane >> 5) + e, channel 32 j + (lane & 31)
    const float scale = __builtin_ldexpf(1.f, -(split_exp(a.maxbits[0]) + split_exp(a.maxbits[1])));
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int o = 32 * j + (lane & 31);
        const float bv = a.bias ? a.bias[o] : 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int p = p0 + 64 * wave + 32 * i + 8 * g + 4 * (lane >> 5) + e;
                    if (p < HW) a.y[((int64_t)n * HW + p) * C + o] = acc[i][j][4 * g + e] * scale + bv;
                }
    }
}

// ------------------------------------------------------------------------------------------------ weight gradient
// dW[o][i][kh][kw] = sum_{n,h,w} dY[n][h][w][o] X[n][h + d (kh - 2)][w + d (kw - 2)][i] from the two Q4-split operands
// (X split in the forward, dY for the input gradient), scaled back by 2^-(e_dy + e_x).  Per-tap GEMM with M = o, N = i
// and the reduction over pixels: workgroup (chunk range r, kernel row kh) runs over a contiguous range of 64-pixel raster
// chunks; per chunk the dY rows and the input segment of row kh (positions as in the forward: the chunk's pixels of one
// or two rows, 2d halo, 4d gap) are staged by LDS-DMA.  8 waves: wave (half, o block, i block) accumulates the 5 kw tiles
// (80 accumulators per lane) over k-steps {2 half, 2 half + 1} of every chunk, so two waves share each SIMD (one
// wave's fragment reads and DMA issue run under the other's MFMAs; round 5's 4-wave form left one wave per SIMD, whose
// LDS latency and per-chunk address work were exposed: 0.25 of the split peak in the avse1 step).  Both operands are
// contiguous along the GEMM's M / N (channels), so the fragments are read with ds_read_b64_tr_b16 (4 pixels x 16
// channels per 16-lane group, delivered transposed) from 256-B pixel rows whose 16-B chunk c sits at c ^ ((r & 3) << 2).
// The kh = 0 workgroups add one more MFMA pair per k-step against a ones fragment: the bias gradient db[o] = sum dY[.][o].
// The chunk positions advance incrementally (no integer division in the loop).  Per-(workgroup, half) partial slabs,
// summed in a fixed order by a second kernel (deterministic).
constexpr int WG_CHUNK = 64;                     // pixels per chunk (4 k-steps of 16)
constexpr int PIXB = 256;                        // LDS / Q4 bytes per pixel
constexpr int WTHREADS = 512, WWAVES = WTHREADS / 64;

typedef short s4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4_t lds_s4_t;

// 16-B chunk c of staged pixel row r sits at physical chunk tswz(r, c).  A transposed fragment read (tfrag) takes, per
// 32-lane half, 4 consecutive rows x 4 chunks whose logical indices differ in bits 0 and 2; the rows' XOR masks must
// then differ in bits 1 and 3 for the 16 (row, chunk) pairs to land on 16 distinct 4-bank groups (every row starts on
// bank 0: 256-B rows).  Round 5's mask ((r & 3) << 2) moved bits 2-3 only: 2-way conflicts on every read
// (SQ_LDS_BANK_CONFLICT = 0.5 x SQ_LDS_IDX_ACTIVE, gpurun_out/r06f_pmc_dconv); this one is conflict-free.
__device__ inline int tswz(int r, int c) { return c ^ (((r & 1) << 1) | ((r & 2) << 2)); }

// MFMA operand fragment (32 channels x 16 pixels) of the channel block cb (quarters 2 cb, 2 cb + 1), plane pl (0 hi,
// 1 lo), k-step rows rows[0..15] given per lane: lane l (group g = l >> 4, i = l & 15) reads pixel rows
// row(8 (g >> 1) + (i >> 2) + 4 u), channels 16 (g & 1) + 4 (i & 3) .. + 3 of the block
__device__ inline half8 tfrag(const uint8_t* img, const int (&row)[2], int cb, int pl, int lane) {
    const int g = lane >> 4, i = lane & 15;
    const int q = 2 * cb + (g & 1);
    s4_t v[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int r = row[u];
        const int byte = q * 64 + pl * 32 + 8 * (i & 3);                 // within the pixel's 256 B
        const int off = r * PIXB + 16 * tswz(r, byte >> 4) + (byte & 15);
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
    float* part;                 // [ranges][2][kh][kw][o][i]
    float* dbpart;               // [ranges][2][o] (kh = 0 workgroups) or NULL
    int N, H, W, cpi, chunks, ranges;
};

// a chunk's position: image n, first raster pixel p0 in it, its row hA and column wA0
struct ChunkPos {
    int n, p0, hA, wA0;
    __device__ void init(int c, int cpi, int W) {
        n = c / cpi;
        p0 = (c - n * cpi) * WG_CHUNK;
        hA = p0 / W;
        wA0 = p0 - hA * W;
    }
    __device__ void next(int HW, int W) {                // W >= WG_CHUNK
        p0 += WG_CHUNK;
        if (p0 >= HW) {
            ++n;
            p0 = hA = wA0 = 0;
        } else {
            wA0 += WG_CHUNK;
            if (wA0 >= W) {
                wA0 -= W;
                ++hA;
            }
        }
    }
};

template <int D>
__global__ __launch_bounds__(WTHREADS, 1) void wgrad_kernel(WArgs a) {
    constexpr int NP = WG_CHUNK + 8 * D;           // staged input positions per chunk
    constexpr int YIMG = WG_CHUNK * PIXB, XIMG = NP * PIXB, STG = YIMG + XIMG;
    constexpr int NB = (3 * STG <= 160 * 1024) ? 3 : 2;
    constexpr int PY = YIMG / 1024, PT = PY + XIMG / 1024;       // pieces per chunk (4 pixels per 1-KB piece)
    constexpr int MAXPW = PT / WWAVES + 1;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[NB * STG];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = xcd_remap(blockIdx.x, gridDim.x);       // the 5 kh workgroups of a range share an XCD's L2
    const int r = bid / KS, kh = bid % KS;
    const int c_lo = (int)((int64_t)r * a.chunks / a.ranges), c_hi = (int)((int64_t)(r + 1) * a.chunks / a.ranges);
    const int HW = a.H * a.W;
    const i4_t rx = rsrc_of(a.xq, (int64_t)a.N * HW * PIXB);
    const i4_t ry = rsrc_of(a.dyq, (int64_t)a.N * HW * PIXB);
    const uint32_t lds0 = lds_u32(lds);
    const int npieces = (PT - wave + WWAVES - 1) / WWAVES;
    const int pr = lane >> 4, pc = lane & 15;                    // a piece's lane: row (of 4), physical chunk
    // per piece of this wave: the lane's pixel (dY) or position (X) within the chunk and its swizzled chunk byte offset
    int pj[MAXPW];
    uint32_t psw[MAXPW];
#pragma unroll
    for (int m = 0; m < MAXPW; ++m) {
        const int k = wave + WWAVES * m;
        pj[m] = k < PY ? 4 * k + pr : 4 * (k - PY) + pr;
        psw[m] = 16u * tswz(pj[m], pc);
    }

    auto issue = [&](const ChunkPos& cp, int buf) {
        const int nA = min(WG_CHUNK, a.W - cp.wA0);
        const int row1 = cp.hA + D * (kh - 2), row2 = nA < WG_CHUNK ? row1 + 1 : -1000000;
        const int ybase = cp.n * HW + cp.p0;                     // dY pixel of chunk position 0
        const int nHrow = cp.n * a.H;
        const uint32_t img = lds0 + buf * STG;
#pragma unroll
        for (int m = 0; m < MAXPW; ++m) {
            if (m >= npieces) break;
            const int k = wave + WWAVES * m;
            if (k < PY) {                                        // dY rows: chunk pixel j
                const int j = pj[m];
                const uint32_t off = cp.p0 + j < HW ? (uint32_t)(ybase + j) * PIXB + psw[m] : 0x7FFFFFF0u;
                dma16(ry, img + k * 1024, off);
            } else {
                const int q = pj[m];                             // input position
                const bool s1 = q < nA + 4 * D;
                const int col = s1 ? cp.wA0 - 2 * D + q : q - nA - 6 * D;
                const int row = s1 ? row1 : row2;
                const bool ok = (unsigned)col < (unsigned)a.W && (unsigned)row < (unsigned)a.H;
                const uint32_t pix = (uint32_t)((nHrow + row) * a.W + col);
                dma16(rx, img + YIMG + (k - PY) * 1024, ok ? pix * PIXB + psw[m] : 0x7FFFFFF0u);
            }
        }
    };

    const int half = wave >> 2, ob = (wave >> 1) & 1, ib = wave & 1;   // k-steps {2 half, 2 half + 1}, (o, i) block
    const bool want_db = a.dbpart != nullptr && kh == 0 && ib == 0;      // wave-uniform
    floatx16 acc[KS], accb;
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[k][e] = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) accb[e] = 0.f;
    half8 ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (_Float16)1.0f;

    const int g = lane >> 4, li = lane & 15;
    ChunkPos cc, ci;                                             // compute cursor (chunk c), issue cursor
    cc.init(c_lo, a.cpi, a.W);
    ci = cc;
    if (c_lo < c_hi) {
        issue(ci, 0);
        ci.next(HW, a.W);
    }
    if (NB == 3 && c_lo + 1 < c_hi) {
        issue(ci, 1);
        ci.next(HW, a.W);
    }
    for (int c = c_lo; c < c_hi; ++c) {
        const int it = c - c_lo;
        const bool ahead = NB == 3 && c + 1 < c_hi;              // the next chunk's pieces may still fly
        if (ahead) wait_all_but(npieces);
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (c + NB - 1 < c_hi) {
            issue(ci, (it + NB - 1) % NB);
            ci.next(HW, a.W);
        }
        const uint8_t* yimg = lds + (it % NB) * STG;
        const uint8_t* ximg = yimg + YIMG;
        const int nA = min(WG_CHUNK, a.W - cc.wA0);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const int s = 2 * half + s2;
            int ry_[2], rx_[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int j = 16 * s + 8 * (g >> 1) + (li >> 2) + 4 * u;       // the lane's pixel of the k-step
                ry_[u] = j;
                rx_[u] = j < nA ? j : j + 4 * D;
            }
            const half8 ah = tfrag(yimg, ry_, ob, 0, lane), al = tfrag(yimg, ry_, ob, 1, lane);
#pragma unroll
            for (int kw = 0; kw < KS; ++kw) {
                const int rk[2] = {rx_[0] + D * kw, rx_[1] + D * kw};
                const half8 bh = tfrag(ximg, rk, ib, 0, lane), bl = tfrag(ximg, rk, ib, 1, lane);
                acc[kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[kw], 0, 0, 0);
                acc[kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[kw], 0, 0, 0);
                acc[kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[kw], 0, 0, 0);
            }
            if (want_db) {
                accb = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, ones, accb, 0, 0, 0);
                accb = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, ones, accb, 0, 0, 0);
            }
        }
        cc.next(HW, a.W);
    }
    // partial tiles: acc[kw] register 4 q + e = row o = 32 ob + 8 q + 4 (lane >> 5) + e, column i = 32 ib + (lane & 31)
    const float sc = __builtin_ldexpf(1.f, -(split_exp(*a.xmax) + split_exp(*a.dymax)));
    float* pp = a.part + (((int64_t)r * 2 + half) * KS + kh) * KS * C * C;
#pragma unroll
    for (int kw = 0; kw < KS; ++kw)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int o = 32 * ob + 8 * q + 4 * (lane >> 5) + e, i = 32 * ib + (lane & 31);
                pp[((int64_t)kw * C + o) * C + i] = acc[kw][4 * q + e] * sc;
            }
    if (want_db && (lane & 31) == 0) {
        const float sd = __builtin_ldexpf(1.f, -split_exp(*a.dymax));
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e)
                a.dbpart[((int64_t)r * 2 + half) * C + 32 * ob + 8 * q + 4 * (lane >> 5) + e] = accb[4 * q + e] * sd;
    }
}

// dW[o][i][kh][kw] = sum over slabs of part[slab][kh][kw][o][i]; db[o] = sum over slabs of dbpart[slab][o] (slab =
// 2 range + half, summed in order: deterministic)
__global__ void wgrad_reduce_kernel(const float* __restrict__ part, const float* __restrict__ dbpart, int slabs,
                                    float* __restrict__ dw, float* __restrict__ db) {
    constexpr int TOTAL = KS * KS * C * C;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= TOTAL) {
        if (db != nullptr && idx < TOTAL + C) {
            float v = 0.f;
            for (int g = 0; g < slabs; ++g) v += dbpart[(int64_t)g * C + idx - TOTAL];
            db[idx - TOTAL] = v;
        }
        return;
    }
    float v = 0.f;
    for (int g = 0; g < slabs; ++g) v += part[(int64_t)g * TOTAL + idx];
    const int i = idx % C, o = (idx / C) % C, kw = (idx / (C * C)) % KS, kh = idx / (KS * C * C);
    dw[((o * C + i) * KS + kh) * KS + kw] = v;
}

inline int wgrad_ranges(int chunks) { return std::max(1, std::min(chunks, 256 / KS * 1)); }

// ------------------------------------------------------------------------------------------------ operand preparation
// max |x| over n floats -> atomicMax on the float bits (non-negative floats order like their bits; NaN wins).  One
// atomic per 1024-thread workgroup of a 256-workgroup grid: the word's atomics serialise at the memory side (~17 ns
// each), so one per wave of a 2048 x 256 grid cost ~140 us of a 165 us pass (profiles/r05v3_avse1_timed_window_stats.csv)
constexpr int AMAX_NT = 1024, AMAX_GRID = 256;
__global__ __launch_bounds__(AMAX_NT) void absmax_kernel(const float4* x, int64_t n4, uint32_t* out) {
    __shared__ uint32_t red[AMAX_NT / 64];
    float m = 0.f;
    const int64_t stride = (int64_t)gridDim.x * AMAX_NT;
    for (int64_t i0 = blockIdx.x * (int64_t)AMAX_NT + threadIdx.x; i0 < n4; i0 += 4 * stride) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = i0 + u * stride < n4 ? x[i0 + u * stride] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int u = 0; u < 4; ++u) m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
    }
    uint32_t b = __float_as_uint(m);
    for (int o = 32; o >= 1; o >>= 1) b = max(b, (uint32_t)__shfl_xor((int)b, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 0; k < AMAX_NT / 64; ++k) b = max(b, red[k]);
        if (b) atomicMax(out, b);
    }
}

__device__ inline uint32_t split2(float x0, float x1, float sc, uint32_t& lo) {
    const float s0 = x0 * sc, s1 = x1 * sc;
    const _Float16 h0 = (_Float16)s0, h1 = (_Float16)s1;
    const _Float16 l0 = (_Float16)(s0 - (float)h0), l1 = (_Float16)(s1 - (float)h1);
    lo = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
    return (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
}

// NHWC fp32 (n_pix x 64) -> Q4 (n_pix x 4 quarters x [hi 16 | lo 16] fp16); thread = one (pixel, quarter)
__global__ void split_kernel(const float* x, int64_t nq, const uint32_t* maxbits, uint4* xq) {
    const float sc = __builtin_ldexpf(1.f, split_exp(maxbits[0]));
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nq; i += (int64_t)gridDim.x * blockDim.x) {
        const float4* s = reinterpret_cast<const float4*>(x + i * 16);
        uint32_t hi[8], lo[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 v = s[k];
            hi[2 * k] = split2(v.x, v.y, sc, lo[2 * k]);
            hi[2 * k + 1] = split2(v.z, v.w, sc, lo[2 * k + 1]);
        }
        uint4* d = xq + i * 4;
        d[0] = uint4{hi[0], hi[1], hi[2], hi[3]};
        d[1] = uint4{hi[4], hi[5], hi[6], hi[7]};
        d[2] = uint4{lo[0], lo[1], lo[2], lo[3]};
        d[3] = uint4{lo[4], lo[5], lo[6], lo[7]};
    }
}

// W (64 o, 64 i, 5, 5) fp32 -> [kh * 4 + q][kw][o][hi 16 | lo 16]; transposed = the input gradient's W'[o][i][kh][kw] =
// W[i][o][4 - kh][4 - kw].  One workgroup: max |w| first, then the split with that scale.
__global__ __launch_bounds__(1024) void wprep_kernel(const float* w, int transposed, uint32_t* maxbits, uint16_t* wq) {
    __shared__ uint32_t red[16];
    constexpr int TOT = C * C * KS * KS;
    float m = 0.f;
    for (int i = threadIdx.x; i < TOT; i += blockDim.x) m = fmaxf(m, fabsf(w[i]));
    uint32_t b = __float_as_uint(m);
    for (int o = 32; o >= 1; o >>= 1) b = max(b, (uint32_t)__shfl_xor((int)b, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
    __syncthreads();
    b = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) b = max(b, red[k]);
    if (threadIdx.x == 0) maxbits[1] = b;
    const float sc = __builtin_ldexpf(1.f, split_exp(b));
    // destination element e: stage s = kh * 4 + q, kw, o, plane, c (16)
    for (int e = threadIdx.x; e < TOT; e += blockDim.x) {
        const int c = e % 16, o = (e / 16) % C, kw = (e / (16 * C)) % KS, s = e / (16 * C * KS);
        const int kh = s / NQ, q = s % NQ, i = q * 16 + c;
        const float v = transposed ? w[((i * C + o) * KS + (KS - 1 - kh)) * KS + (KS - 1 - kw)]
                                   : w[((o * C + i) * KS + kh) * KS + kw];
        const float sv = v * sc;
        const _Float16 h = (_Float16)sv, l = (_Float16)(sv - (float)h);
        const int64_t row = ((int64_t)s * KS + kw) * C + o;
        wq[row * 32 + c] = __builtin_bit_cast(uint16_t, h);
        wq[row * 32 + 16 + c] = __builtin_bit_cast(uint16_t, l);
    }
}

}  // namespace dcf
}  // namespace avse

using namespace avse::dcf;

extern "C" {

int64_t avse_dconv_wprep_bytes(void) { return (int64_t)NSTG * WIMG; }

int avse_split16(int64_t n_pix, const float* x, void* xq, uint32_t* maxbits, avse_stream_t stream) {
    if (!x || !xq || !maxbits) return AVSE_EINVAL;
    if (n_pix <= 0) return AVSE_ESHAPE;
    if (((uintptr_t)x & 15) || ((uintptr_t)xq & 15)) return AVSE_EALIGN;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(maxbits, 0, 4, st) != hipSuccess) return AVSE_ELAUNCH;
    const int64_t n4 = n_pix * C / 4;
    hipLaunchKernelGGL(absmax_kernel, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(AMAX_GRID, (n4 + AMAX_NT - 1) / AMAX_NT))),
                       dim3(AMAX_NT), 0, st, reinterpret_cast<const float4*>(x), n4, maxbits);
    AVSE_CHECK_LAUNCH();
    const int64_t nq = n_pix * NQ;
    const int blocks = (int)std::min<int64_t>((nq + 255) / 256, 8192);
    hipLaunchKernelGGL(split_kernel, dim3(blocks), dim3(256), 0, st, x, nq, maxbits, reinterpret_cast<uint4*>(xq));
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_split16_known(int64_t n_pix, const float* x, void* xq, const uint32_t* maxbits, avse_stream_t stream) {
    if (!x || !xq || !maxbits) return AVSE_EINVAL;
    if (n_pix <= 0) return AVSE_ESHAPE;
    if (((uintptr_t)x & 15) || ((uintptr_t)xq & 15)) return AVSE_EALIGN;
    const int64_t nq = n_pix * NQ;
    const int blocks = (int)std::min<int64_t>((nq + 255) / 256, 8192);
    hipLaunchKernelGGL(split_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, nq, maxbits,
                       reinterpret_cast<uint4*>(xq));
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_dconv_wprep(const float* w, int32_t transposed, void* wq, uint32_t* maxbits, avse_stream_t stream) {
    if (!w || !wq || !maxbits) return AVSE_EINVAL;
    hipLaunchKernelGGL(wprep_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, w, transposed, maxbits,
                       reinterpret_cast<uint16_t*>(wq));
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int64_t avse_dconv_wgrad16_workspace_bytes(int64_t N, int64_t H, int64_t W) {
    const int64_t chunks = N * ((H * W + WG_CHUNK - 1) / WG_CHUNK);
    return 4 * 2 * (int64_t)wgrad_ranges((int)std::min<int64_t>(chunks, 1 << 30)) * (KS * KS * C * C + C);
}

int avse_dconv_wgrad16(int64_t N, int64_t H, int64_t W, int64_t dil, const void* xq, const uint32_t* xmax,
                       const void* dyq, const uint32_t* dymax, float* dw, float* db, float* workspace,
                       avse_stream_t stream) {
    if (!xq || !xmax || !dyq || !dymax || !dw || !workspace) return AVSE_EINVAL;
    if (N <= 0 || H <= 0 || W < WG_CHUNK || (dil != 2 && dil != 4 && dil != 8 && dil != 16)) return AVSE_ESHAPE;
    if (N * H * W * 256 >= (1LL << 31) - 1024) return AVSE_ESHAPE;
    WArgs a;
    a.xq = xq;
    a.dyq = dyq;
    a.xmax = xmax;
    a.dymax = dymax;
    a.N = (int)N;
    a.H = (int)H;
    a.W = (int)W;
    a.cpi = (int)((H * W + WG_CHUNK - 1) / WG_CHUNK);
    a.chunks = (int)(N * a.cpi);
    a.ranges = wgrad_ranges(a.chunks);
    a.part = workspace;
    a.dbpart = db ? workspace + (int64_t)2 * a.ranges * KS * KS * C * C : nullptr;
    const dim3 grid((unsigned)(a.ranges * KS)), block(WTHREADS);
    hipStream_t st = (hipStream_t)stream;
    switch (dil) {
        case 2: hipLaunchKernelGGL(wgrad_kernel<2>, grid, block, 0, st, a); break;
        case 4: hipLaunchKernelGGL(wgrad_kernel<4>, grid, block, 0, st, a); break;
        case 8: hipLaunchKernelGGL(wgrad_kernel<8>, grid, block, 0, st, a); break;
        default: hipLaunchKernelGGL(wgrad_kernel<16>, grid, block, 0, st, a); break;
    }
    AVSE_CHECK_LAUNCH();
    constexpr int TOTAL = KS * KS * C * C;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((TOTAL + C + 255) / 256), dim3(256), 0, st, a.part, a.dbpart,
                       2 * a.ranges, dw, db);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_dconv_fwd(int64_t N, int64_t H, int64_t W, int64_t dil, const void* xq, const void* wq,
                   const uint32_t* maxbits, const float* bias, float* y, avse_stream_t stream) {
    if (!xq || !wq || !maxbits || !y) return AVSE_EINVAL;
    if (N <= 0 || H <= 0 || W < 256 || (dil != 2 && dil != 4 && dil != 8 && dil != 16)) return AVSE_ESHAPE;
    if (N * H * W * 256 >= (1LL << 31) - 1024) return AVSE_ESHAPE;       // 32-bit byte offsets into the split input
    Args a;
    a.xq = xq;
    a.wq = wq;
    a.maxbits = maxbits;
    a.bias = bias;
    a.y = y;
    a.N = (int)N;
    a.H = (int)H;
    a.W = (int)W;
    // d <= 8: tile = 256 raster pixels on 4 waves, two workgroups per CU (2 LDS buffers of <= 40 KB each): the two
    // workgroups' barriers and DMA phases interleave, 1.61 vs 1.69 ms per launch at C2 against one 8-wave 512-pixel
    // workgroup per CU (profiles/r06g_dconv_fwd_ab.jsonl; one 4-wave workgroup per CU with 3 buffers measured slower in
    // round 5).  d = 16: the 4-wave tile's 4d halos need 89 KB per workgroup, so it keeps the 8-wave form.
    const int nw = dil <= 8 ? 4 : 8;
    a.tiles = (int)((H * W + 64 * nw - 1) / (64 * nw));
    const dim3 grid((unsigned)(N * a.tiles)), block(64 * nw);
    hipStream_t st = (hipStream_t)stream;
    switch (dil) {
        case 2: hipLaunchKernelGGL((fwd_kernel<2, 4, 2>), grid, block, 0, st, a); break;
        case 4: hipLaunchKernelGGL((fwd_kernel<4, 4, 2>), grid, block, 0, st, a); break;
        case 8: hipLaunchKernelGGL((fwd_kernel<8, 4, 2>), grid, block, 0, st, a); break;
        default: hipLaunchKernelGGL((fwd_kernel<16, 8>), grid, block, 0, st, a); break;
    }
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
