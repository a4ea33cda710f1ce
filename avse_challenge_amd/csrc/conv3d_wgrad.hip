// Weight gradient of the lip front-end Conv3d (Cout 64, small Cin, kernel (KT,KH,KW), stride (1,2,2))
// for gfx950, as an implicit GEMM on the exact-fp32 MFMA (v_mfma_f32_32x32x2_f32).  The input is read in its
// stored dtype: fp32, or the uint8 lip frames themselves (avse_conv3d_wgrad_u8: no fp32 copy of the clip).
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
// One workgroup (4 waves) owns a strided set of output rows (b, t, ho) and a slice of N; per row it
// stages the input rows its slice touches (width 2*(WO-1)+KW) and the 64 x WO gradient row in LDS,
// then every wave runs WO/2 K-steps of 2 x NTW 32x32x2 MFMAs (M = 64 = 2 tiles, N split over waves).
// Partial 64 x N tiles per workgroup go to a workspace; a second kernel sums them (deterministic).
#include <algorithm>
#include <type_traits>

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
    int hc;                         // wgrad16: output rows per run
};

// Per workgroup: a strided set of output rows (b, t, ho) and one N slice of 4*NTW 32-wide tiles
// (blockIdx.y), so a slice stages only the input rows its columns touch.  Software pipelined:
// the next row's input window and dY row are loaded into registers (raw buffer loads, out-of-range
// -> 0, no waits at issue) while the MFMAs of the current row run out of LDS.
template <typename T, int NTW, int RPW>
__global__ __launch_bounds__(THREADS, 2) void wgrad_kernel(Shape s, const T* __restrict__ x,
                                                           const float* __restrict__ dy, float* __restrict__ part) {
    extern __shared__ float lds[];
    const int WIN = 2 * (s.WO - 1) + s.KW;
    const int WINP = WIN + 1;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // uniform: row math stays scalar
    const int nxrow = s.CIN * s.KT * s.KH;
    const int n_lo = blockIdx.y * 4 * NTW * 32;
    const int n_hi = min(s.N, n_lo + 4 * NTW * 32);
    const int r_lo = n_lo / s.KW, r_hi = min(nxrow, (n_hi + s.KW - 1) / s.KW);
    const int nrs = r_hi - r_lo;                         // staged input rows (<= 4 * RPW)
    float* xs = lds;                                     // [nrs][WINP]
    float* zero = xs + nrs * WINP;                       // 2 * MAX_WO + 8 zeros (N padding)
    float* ys = zero + 2 * MAX_WO + 8;                   // [64][YS]
    for (int i = threadIdx.x; i < 2 * MAX_WO + 8; i += THREADS) zero[i] = 0.f;

    int boff[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int n = n_lo + (wave * NTW + j) * 32 + (lane & 31);
        boff[j] = n < n_hi ? (n / s.KW - r_lo) * WINP + n % s.KW : (int)(zero - xs);
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
    const int nx = (int)((int64_t)s.B * s.CIN * s.T * plane);     // < 2^29 (checked at launch)
    const int ny = (int)((int64_t)s.B * COUT * s.TO * yplane);
    const auto rx = make_rsrc(x, nx);
    const auto ry = make_rsrc(dy, ny);                    // element offset nx / ny is past num_records -> 0
    float xr[RPW][2], yr[16];
    const int wo2 = (s.WO + 1) & ~1;

    auto prefetch = [&](int row) {
        const int ho = row % s.HO, t = (row / s.HO) % s.TO, b = row / (s.HO * s.TO);
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            const int r = r_lo + wave + 4 * i;           // wave-uniform
            const int kh = r % s.KH, kt = (r / s.KH) % s.KT, ci = r / (s.KH * s.KT);
            const int ti = t - s.PT + kt, hi = 2 * ho - s.PH + kh;
            const bool rowok = r < r_hi && ti >= 0 && ti < s.T && hi >= 0 && hi < s.H;
            const int base = (int)(((int64_t)(b * s.CIN + ci) * s.T + ti) * plane + (int64_t)hi * s.W) - s.PW;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int c = lane + 64 * q, wi = c - s.PW;
                const bool ok = rowok && c < WIN && wi >= 0 && wi < s.W;
                xr[i][q] = bufld<T>::ld(rx, ok ? base + c : nx, 0);
            }
        }
        const int64_t yb = ((int64_t)b * COUT * s.TO + t) * yplane + (int64_t)ho * s.WO;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int co = wave + 4 * i;
            const bool ok = lane < s.WO;
            yr[i] = bufld<float>::ld(ry, ok ? (int)(yb + (int64_t)co * s.TO * yplane) + lane : ny, 0);
        }
    };

    int row = blockIdx.x;
    if (row < s.rows) prefetch(row);
    for (; row < s.rows; row += gridDim.x) {
        __syncthreads();                                 // previous row's MFMAs are done with LDS
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            const int rr = wave + 4 * i;
            if (rr < nrs) {
                if (lane < WIN) xs[rr * WINP + lane] = xr[i][0];          // lanes past the window would
                if (lane + 64 < WIN) xs[rr * WINP + lane + 64] = xr[i][1];  // spill into the next row
                // the pad slot: an odd WO's last k-step (dY = 0 there) reads it, and 0 x stale-LDS NaN is NaN
                if (lane == 0) xs[rr * WINP + WIN] = 0.f;
            }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (lane < wo2) ys[(wave + 4 * i) * YS + lane] = lane < s.WO ? yr[i] : 0.f;
        __syncthreads();
        if (row + (int)gridDim.x < s.rows) prefetch(row + gridDim.x);
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
            const int n = n_lo + (wave * NTW + j) * 32 + (lane & 31);
            if (n < n_hi) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int co = m * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    p[(int64_t)co * s.N + n] = acc[m][j][r];
                }
            }
        }
}

// ------------------------------------------------------------------------------------------------ split f16
// The same decomposition on the f16 MFMA with dY split per element into hi + lo fp16 under one power-of-two scale
// (max |dY| 2^e in [2^14, 2^15): the producing BatchNorm -> act backward reports max |dY|).  uint8 frames are exact in
// fp16: dW = 2^-e (dY_hi X + dY_lo X), 2 MFMAs per product against 1/16-rate fp32 MFMAs.  fp32 frames (round 6, the
// avse4 front-end) are split as well under max |X| (the forward's absmax pass): dW = 2^-(e + f) (dY_hi X_hi + dY_lo X_hi
// + dY_hi X_lo), 3 MFMAs, the lo x lo term dropped (the products to 22 bits, fp32 accumulation).
// Per output row (b, t, ho): K = wo in k16-steps; A = dY (64 co x 16 wo, hi / lo rows in LDS, 16-B reads); B = the
// input columns 2 wo + kw - 3 of the staged rows: stride 2 along wo, so every staged row is kept as its two column
// parities, each twice (the second copy one element later), and a lane's 8 values (8 consecutive wo of one (row,
// kw) tap) are 4 aligned 4-B words of one copy.
// Round 6: a workgroup walks runs of consecutive output rows (b, t, ho0 .. ho1) and keeps each input plane's rows in a
// ring of RING = 8 staged rows (a sliding window over ho): row ho needs input rows 2 ho - PH .. 2 ho - PH + KH - 1 of
// every plane, of which only the last 2 are new after row ho - 1, so a step stages 2 rows per plane (KH at a run's
// start) instead of all KH: the round-5 kernel restaged every row for every output row it served (3.5x the LDS
// writes at KH = 7), and staging, not the MFMAs, set its time.  The ring slot of input row hi is (hi + PH) & 7.
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
constexpr int PARW = MAX_WO + 8;                    // fp16 per parity copy (column pairs of one staged row)
constexpr int YS16 = MAX_WO + 8;                    // fp16 per dY row (hi, lo planes)
constexpr int RING = 8;                             // staged rows per input plane
constexpr int RUN = 16;                             // output rows per run (at most)

__device__ inline int split_exp_w(uint32_t mb) {
    const int ef = (int)((mb >> 23) & 0xff);
    if (mb == 0) return 0;
    const int k = ef == 0 ? -127 : ef - 127;
    return min(100, max(-100, 14 - k));
}

// runs: s.rows = B * TO * nrun units (b, t, run), run r covering output rows r * s.hc .. min(HO, (r + 1) * s.hc) - 1
template <typename XT, int NTW, int RPW>
__global__ __launch_bounds__(THREADS, 2) void wgrad16_kernel(Shape s, const XT* __restrict__ x,
                                                             const uint32_t* __restrict__ xmax,
                                                             const float* __restrict__ dy,
                                                             const uint32_t* __restrict__ dymax,
                                                             float* __restrict__ part) {
    constexpr bool XS = std::is_same<XT, float>::value;         // fp32 frames: a lo image of the staged rows
    extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
    const int WIN = 2 * (s.WO - 1) + s.KW;
    const int lane = threadIdx.x & 63, half = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nxrow = s.CIN * s.KT * s.KH;
    const int n_lo = blockIdx.y * 4 * NTW * 32;
    const int n_hi = min(s.N, n_lo + 4 * NTW * 32);
    const int r_lo = n_lo / s.KW, r_hi = min(nxrow, (n_hi + s.KW - 1) / s.KW);
    const int p_lo = r_lo / s.KH, npl = (r_hi - 1) / s.KH + 1 - p_lo;     // input planes (ci, kt) of the slice
    const int nrs = npl * RING;                                   // staged rows; row nrs: zeros (the N padding)
    const int ks = (s.WO + 15) / 16;                             // k16-steps per output row
    // LDS: dY hi, lo [64][YS16]; staged rows [nrs + 1][parity 2][copy 2][PARW], the lo image after the hi one
    _Float16* yh = reinterpret_cast<_Float16*>(lds8);
    _Float16* yl = yh + COUT * YS16;
    _Float16* xs = yl + COUT * YS16;
    const int XROW = 4 * PARW;                                   // fp16 per staged row
    const int XIMG = (nrs + 1) * XROW;                           // fp16 per image
    for (int i = threadIdx.x; i < XROW; i += THREADS) xs[nrs * XROW + i] = (_Float16)0.f;
    if constexpr (XS)
        for (int i = threadIdx.x; i < XROW; i += THREADS) xs[XIMG + nrs * XROW + i] = (_Float16)0.f;
    // the tail of every copy that staging never writes (copy 0 holds m < 64, copy 1 m < 63) but the k16-steps of the
    // last output columns read (their dY is 0, and 0 x a stale NaN pattern is NaN): zero once, before the first barrier
    for (int i = threadIdx.x; i < (XS ? 2 : 1) * (nrs + 1) * 4 * (PARW - 63); i += THREADS) {
        const int k = i % (PARW - 63), sub = (i / (PARW - 63)) % 4, r = i / ((PARW - 63) * 4);   // r counts both images
        const int m = 63 + k;
        if (m >= 64 - (sub & 1)) xs[r * XROW + sub * PARW + m] = (_Float16)0.f;
    }

    // B fragment per N tile: the plane's ring (row (2 ho + kh) & 7 of it, added per output row), parity p = kw & 1,
    // copy q = (kw >> 1) & 1, element m0 - q with m0 = wo + kw >> 1 (wo added per k-step), so the lane reads words
    // 2 i of copy q: (m0 - q) is even for even wo.  Padding columns read the zero row.
    int bbase[NTW], bshift[NTW], bkh[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int n = n_lo + (wave * NTW + j) * 32 + (lane & 31);
        const bool ok = n < n_hi;
        const int r = ok ? n / s.KW : 0, kw = ok ? n % s.KW : 0;
        const int p = kw & 1, q = (kw >> 1) & 1;
        bbase[j] = (ok ? (r / s.KH - p_lo) * RING * XROW : nrs * XROW) + (2 * p + q) * PARW;
        bshift[j] = (kw >> 1) - q;                               // even
        bkh[j] = ok ? r % s.KH : -1;
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
    const int nx = (int)((int64_t)s.B * s.CIN * s.T * plane);
    const int ny = (int)((int64_t)s.B * COUT * s.TO * yplane);
    const auto rx = make_rsrc(x, nx);
    const auto ry = make_rsrc(dy, ny);
    const float sc = __builtin_ldexpf(1.f, split_exp_w(*dymax));
    const float xsc = XS ? __builtin_ldexpf(1.f, split_exp_w(*xmax)) : 1.f;
    float xr[RPW][2], yr[16];
    const int wo16 = ks * 16;
    const int nrun = (s.HO + s.hc - 1) / s.hc;

    // a step = one output row (unit u, output row ho); first: the run's first row (KH rows per plane staged, else 2)
    struct Step {
        int u, ho, ho_end;
        bool first;
    };
    auto unit_step = [&](int u) {
        const int r = u % nrun;
        return Step{u, r * s.hc, min(s.HO, (r + 1) * s.hc), true};
    };
    auto next_step = [&](const Step& c) {
        if (c.ho + 1 < c.ho_end) return Step{c.u, c.ho + 1, c.ho_end, false};
        return unit_step(c.u + (int)gridDim.x);
    };
    // staged (plane, row) pair i of a step: plane pl = i / cnt, input row v - PH with v = 2 ho + (first ? 0 : KH - 2)
    // + i % cnt, cnt = first ? KH : 2 -- into the ring row pl * RING + (v & 7).  The quotients by KH and KT of these
    // small wave-uniform operands (< 2^8) are multiply-shifts by ceil(2^16 / d) (exact there): a true division per pair
    // and step cost more than the MFMAs (round-6 A/B)
    const uint32_t mkh = (65536u + s.KH - 1) / s.KH, mkt = (65536u + s.KT - 1) / s.KT;
    auto pair = [&](int f, int i, int& pl, int& dv, int& ci, int& kt) {
        const int pi = wave + 4 * i;
        pl = f ? (int)(((uint32_t)pi * mkh) >> 16) : pi >> 1;
        dv = f ? pi - pl * s.KH : s.KH - 2 + (pi & 1);
        const int pg = p_lo + pl;
        ci = (int)(((uint32_t)pg * mkt) >> 16);
        kt = pg - ci * s.KT;
    };
    auto prefetch = [&](const Step& c) {
        const int bt = c.u / nrun, t = bt % s.TO, b = bt / s.TO;
        const int f = c.first ? 1 : 0;
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            int pl, dv, ci, kt;
            pair(f, i, pl, dv, ci, kt);
            const int v = 2 * c.ho + dv;
            const int ti = t - s.PT + kt, hi = v - s.PH;
            const bool rowok = pl < npl && ti >= 0 && ti < s.T && hi >= 0 && hi < s.H;
            const int base = (int)(((int64_t)(b * s.CIN + ci) * s.T + ti) * plane + (int64_t)hi * s.W) - s.PW;
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                const int cc = lane + 64 * qq, wi = cc - s.PW;
                const bool ok = rowok && cc < WIN && wi >= 0 && wi < s.W;
                xr[i][qq] = bufld<XT>::ld(rx, ok ? base + cc : nx, 0);
            }
        }
        const int64_t yb = ((int64_t)b * COUT * s.TO + t) * yplane + (int64_t)c.ho * s.WO;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int co = wave + 4 * i;
            const bool ok = lane < s.WO;
            yr[i] = bufld<float>::ld(ry, ok ? (int)(yb + (int64_t)co * s.TO * yplane) + lane : ny, 0);
        }
    };

    Step cur = unit_step(blockIdx.x);
    if (cur.u < s.rows) prefetch(cur);
    while (cur.u < s.rows) {
        __syncthreads();                                 // previous row's MFMAs are done with LDS
        {
            const int f = cur.first ? 1 : 0;
#pragma unroll
            for (int i = 0; i < RPW; ++i) {
                int pl, dv, ci, kt;
                pair(f, i, pl, dv, ci, kt);
                const int v = 2 * cur.ho + dv;
                if (pl < npl) {
                    const int rr = pl * RING + (v & (RING - 1));
#pragma unroll
                    for (int qq = 0; qq < 2; ++qq) {
                        const int c = lane + 64 * qq;               // staged column c: input column c - PW
                        if (c < 2 * PARW) {
                            // beyond the window: zeros (the zero-weight 8th tap reads up to 2 columns past it)
                            const float f = c < WIN ? xr[i][qq] * xsc : 0.f;          // uint8: exact, xsc = 1
                            const _Float16 hv = (_Float16)f;
                            const int p = c & 1, mm = c >> 1;
                            xs[rr * XROW + (2 * p) * PARW + mm] = hv;                     // copy 0
                            if (mm >= 1) xs[rr * XROW + (2 * p + 1) * PARW + mm - 1] = hv; // copy 1: one element later
                            if constexpr (XS) {
                                const _Float16 l = (_Float16)(f - (float)hv);
                                xs[XIMG + rr * XROW + (2 * p) * PARW + mm] = l;
                                if (mm >= 1) xs[XIMG + rr * XROW + (2 * p + 1) * PARW + mm - 1] = l;
                            }
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (lane < wo16) {
                const float v = (lane < s.WO ? yr[i] : 0.f) * sc;
                const _Float16 h = (_Float16)v;
                yh[(wave + 4 * i) * YS16 + lane] = h;
                yl[(wave + 4 * i) * YS16 + lane] = (_Float16)(v - (float)h);
            }
        }
        __syncthreads();
        const int ho = cur.ho;
        cur = next_step(cur);
        if (cur.u < s.rows) prefetch(cur);
        int boff[NTW];
#pragma unroll
        for (int j = 0; j < NTW; ++j)
            boff[j] = bbase[j] + (bkh[j] >= 0 ? ((2 * ho + bkh[j]) & (RING - 1)) * XROW : 0) + bshift[j];
        for (int kk = 0; kk < ks; ++kk) {
            const int wo0 = 16 * kk + 8 * half;                  // the lane's 8 k = wo0 .. wo0 + 7
            half8 ah[2], al[2];
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const int co = 32 * m + (lane & 31);
                ah[m] = *reinterpret_cast<const half8*>(&yh[co * YS16 + wo0]);
                al[m] = *reinterpret_cast<const half8*>(&yl[co * YS16 + wo0]);
            }
#pragma unroll
            for (int j = 0; j < NTW; ++j) {
                const _Float16* src = xs + boff[j] + wo0;
                const uint32_t* w32 = reinterpret_cast<const uint32_t*>(src);
                const uint32_t u0 = w32[0], u1 = w32[1], u2 = w32[2], u3 = w32[3];
                const uint32_t __attribute__((ext_vector_type(4))) u = {u0, u1, u2, u3};
                const half8 bv = __builtin_bit_cast(half8, u);
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    acc[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[m], bv, acc[m][j], 0, 0, 0);
                    acc[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[m], bv, acc[m][j], 0, 0, 0);
                }
                if constexpr (XS) {
                    const uint32_t* l32 = reinterpret_cast<const uint32_t*>(src + XIMG);
                    const uint32_t __attribute__((ext_vector_type(4))) ul = {l32[0], l32[1], l32[2], l32[3]};
                    const half8 bl = __builtin_bit_cast(half8, ul);
#pragma unroll
                    for (int m = 0; m < 2; ++m)
                        acc[m][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[m], bl, acc[m][j], 0, 0, 0);
                }
            }
        }
    }
    const float unscale = __builtin_ldexpf(1.f, -split_exp_w(*dymax));
    const float unscale_x = XS ? __builtin_ldexpf(1.f, -split_exp_w(*xmax)) : 1.f;
    float* pp = part + (int64_t)blockIdx.x * COUT * s.N;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const int n = n_lo + (wave * NTW + j) * 32 + (lane & 31);
            if (n < n_hi) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int co = m * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    pp[(int64_t)co * s.N + n] = acc[m][j][r] * unscale * unscale_x;
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

inline int cu_count() {
    static int n = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return cus;
    }();
    return n;
}

}  // namespace c3w
}  // namespace avse

using namespace avse::c3w;

template <typename XT>
static int conv3d_wgrad_impl(int64_t B, int64_t CIN, int64_t T, int64_t H, int64_t W, int64_t KT, int64_t KH,
                             int64_t KW, int64_t PT, int64_t PH, int64_t PW, const XT* x, const float* dy, float* dw,
                             int32_t accumulate, float* workspace, avse_stream_t stream,
                             const uint32_t* dymax = nullptr, const uint32_t* xmax = nullptr) {
    if (!x || !dy || !dw || !workspace) return AVSE_EINVAL;
    Shape s;
    s.B = (int)B; s.CIN = (int)CIN; s.T = (int)T; s.H = (int)H; s.W = (int)W;
    s.KT = (int)KT; s.KH = (int)KH; s.KW = (int)KW; s.PT = (int)PT; s.PH = (int)PH; s.PW = (int)PW;
    s.TO = s.T + 2 * s.PT - s.KT + 1;
    s.HO = (s.H + 2 * s.PH - s.KH) / 2 + 1;
    s.WO = (s.W + 2 * s.PW - s.KW) / 2 + 1;
    s.N = s.CIN * s.KT * s.KH * s.KW;
    if (B <= 0 || CIN <= 0 || s.TO <= 0 || s.HO <= 0 || s.WO <= 0 || s.WO > MAX_WO || s.KW > 8) return AVSE_ESHAPE;
    constexpr int NTW = 3, RPW = 16;
    const int nt = (s.N + 31) / 32;
    const int nsplit = (nt + 4 * NTW - 1) / (4 * NTW);
    s.rows = s.B * s.TO * s.HO;
    s.nparts = nparts_for(s.rows);
    const int WIN = 2 * (s.WO - 1) + s.KW;
    if (WIN > 128) return AVSE_ESHAPE;
    // 32-bit buffer offsets: both tensors must stay under 2 GiB
    if ((int64_t)s.B * s.CIN * s.T * s.H * s.W * (int64_t)sizeof(XT) >= (1LL << 31) ||
        (int64_t)s.B * COUT * s.TO * s.HO * s.WO >= (1LL << 29))
        return AVSE_ESHAPE;
    // staged rows of the widest slice must fit the RPW registers per wave
    int max_nrs = 0;
    for (int y = 0; y < nsplit; ++y) {
        const int n_lo = y * 4 * NTW * 32, n_hi = std::min(s.N, n_lo + 4 * NTW * 32);
        const int nrs = std::min(s.CIN * s.KT * s.KH, (n_hi + s.KW - 1) / s.KW) - n_lo / s.KW;
        max_nrs = std::max(max_nrs, nrs);
    }
    hipStream_t st = (hipStream_t)stream;
    dim3 grid(s.nparts, nsplit), block(THREADS);
    constexpr bool XS = std::is_same<XT, float>::value;
    if (dymax && (!XS || xmax)) {               // the f16 MFMA with dY (and fp32 X) split under the given maxima
        if (2 * ((s.KW - 1) / 2) + 2 * MAX_WO > 2 * PARW || WIN > 128 || s.KH > RING) return AVSE_ESHAPE;
        // units (b, t, run of <= RUN output rows) over one round of resident workgroups (2 per CU, the nsplit N
        // slices side by side), each taking every nparts-th unit: a partial round of a longer grid cost more
        // than the imbalance of one unit in ~30 (round-6 A/B: 1800 workgroups of 8 units, 4.81 ms, vs 512)
        const int nrun = (s.HO + RUN - 1) / RUN;
        s.hc = (s.HO + nrun - 1) / nrun;
        s.rows = s.B * s.TO * nrun;
        s.nparts = std::max(1, std::min(s.rows, std::min(1024, 2 * cu_count() / nsplit)));
        // input planes (ci, kt) of the widest slice: the ring rows, and the (plane, row) pairs a run's first step stages
        int max_npl = 0;
        for (int y = 0; y < nsplit; ++y) {
            const int n_lo = y * 4 * NTW * 32, n_hi = std::min(s.N, n_lo + 4 * NTW * 32);
            const int r_lo = n_lo / s.KW, r_hi = std::min(s.CIN * s.KT * s.KH, (n_hi + s.KW - 1) / s.KW);
            max_npl = std::max(max_npl, (r_hi - 1) / s.KH + 1 - r_lo / s.KH);
        }
        const int pairs = max_npl * s.KH;
        if (pairs > 4 * RPW) return AVSE_ESHAPE;
        const size_t lds16 = 2 * ((size_t)2 * COUT * YS16 + (XS ? 2 : 1) * (size_t)(max_npl * RING + 1) * 4 * PARW);
        if (lds16 > 160 * 1024) return AVSE_ESHAPE;
        dim3 grid16(s.nparts, nsplit);
        // fp32 frames with few planes (avse4: 5 x 7 pairs): 12 prefetch rows per wave keep the kernel within 256
        // VGPRs (16 spill with the lo image's fragments)
        bool launched = false;
        if constexpr (XS) {
            if (pairs <= 4 * 12) {
                static const bool big12 = hipFuncSetAttribute(
                    reinterpret_cast<const void*>(&wgrad16_kernel<XT, NTW, 12>), hipFuncAttributeMaxDynamicSharedMemorySize,
                    160 * 1024) == hipSuccess;
                if (lds16 > 64 * 1024 && !big12) return AVSE_ESHAPE;
                hipLaunchKernelGGL((wgrad16_kernel<XT, NTW, 12>), grid16, block, lds16, st, s, x, xmax, dy, dymax,
                                   workspace);
                launched = true;
            }
        }
        if (!launched) {
            static const bool big = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad16_kernel<XT, NTW, RPW>),
                                                        hipFuncAttributeMaxDynamicSharedMemorySize,
                                                        160 * 1024) == hipSuccess;
            if (lds16 > 64 * 1024 && !big) return AVSE_ESHAPE;
            hipLaunchKernelGGL((wgrad16_kernel<XT, NTW, RPW>), grid16, block, lds16, st, s, x, xmax, dy, dymax,
                               workspace);
        }
        AVSE_CHECK_LAUNCH();
        const int total = COUT * s.N;
        hipLaunchKernelGGL(reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, st, workspace, s.nparts, total, dw,
                           (int)accumulate);
        AVSE_CHECK_LAUNCH();
        return AVSE_OK;
    }
    if (max_nrs > 4 * RPW) return AVSE_ESHAPE;
    const size_t lds = 4 * ((size_t)max_nrs * (WIN + 1) + 2 * MAX_WO + 8 + COUT * YS);
    if (lds > 64 * 1024) return AVSE_ESHAPE;
    hipLaunchKernelGGL((wgrad_kernel<XT, NTW, RPW>), grid, block, lds, st, s, x, dy, workspace);
    AVSE_CHECK_LAUNCH();
    const int total = COUT * s.N;
    hipLaunchKernelGGL(reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, st, workspace, s.nparts, total, dw,
                       (int)accumulate);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

extern "C" {

int64_t avse_conv3d_wgrad_workspace_bytes(int64_t B, int64_t TO, int64_t HO, int64_t N) {
    return 4 * (int64_t)nparts_for((int)(B * TO * HO)) * COUT * N;
}

int avse_conv3d_wgrad(int64_t B, int64_t CIN, int64_t T, int64_t H, int64_t W, int64_t KT, int64_t KH, int64_t KW,
                      int64_t PT, int64_t PH, int64_t PW, const float* x, const float* dy, float* dw,
                      int32_t accumulate, float* workspace, avse_stream_t stream) {
    return conv3d_wgrad_impl<float>(B, CIN, T, H, W, KT, KH, KW, PT, PH, PW, x, dy, dw, accumulate, workspace, stream);
}

int avse_conv3d_wgrad_u8_split(int64_t B, int64_t CIN, int64_t T, int64_t H, int64_t W, int64_t KT, int64_t KH,
                               int64_t KW, int64_t PT, int64_t PH, int64_t PW, const uint8_t* x, const float* dy,
                               const uint32_t* dymax, float* dw, int32_t accumulate, float* workspace,
                               avse_stream_t stream) {
    if (!dymax) return AVSE_EINVAL;
    return conv3d_wgrad_impl<uint8_t>(B, CIN, T, H, W, KT, KH, KW, PT, PH, PW, x, dy, dw, accumulate, workspace, stream,
                                      dymax);
}

int avse_conv3d_wgrad_split(int64_t B, int64_t CIN, int64_t T, int64_t H, int64_t W, int64_t KT, int64_t KH,
                            int64_t KW, int64_t PT, int64_t PH, int64_t PW, const float* x, const uint32_t* xmax,
                            const float* dy, const uint32_t* dymax, float* dw, int32_t accumulate, float* workspace,
                            avse_stream_t stream) {
    if (!xmax || !dymax) return AVSE_EINVAL;
    return conv3d_wgrad_impl<float>(B, CIN, T, H, W, KT, KH, KW, PT, PH, PW, x, dy, dw, accumulate, workspace, stream,
                                    dymax, xmax);
}

int avse_conv3d_wgrad_u8(int64_t B, int64_t CIN, int64_t T, int64_t H, int64_t W, int64_t KT, int64_t KH, int64_t KW,
                         int64_t PT, int64_t PH, int64_t PW, const uint8_t* x, const float* dy, float* dw,
                         int32_t accumulate, float* workspace, avse_stream_t stream) {
    return conv3d_wgrad_impl<uint8_t>(B, CIN, T, H, W, KT, KH, KW, PT, PH, PW, x, dy, dw, accumulate, workspace, stream);
}

}  // extern "C"
