// dt_proj with the selective scan's softplus folded into its epilogue, for gfx950.
//
// Replaces the step-size projection of MambaInnerFnNoOutProj
//   delta = delta_proj_weight @ x_dbl[:, :delta_rank].t()          Mamba-TasNet/modules/mamba/selective_scan_interface.py:187
// together with the `delta = softplus(delta + delta_bias)` that selective_scan_cuda applies per element inside the
// scan (semantics: selective_scan_ref, :110-112).  The scan kernels then read the final step sizes (mode
// delta_softplus = 2 of avse_scan_fwd / avse_scan_bwd) and evaluate no softplus per element.
//
//   delta[b][d][t] = softplus(sum_r W[d][r] * x[b][r][t] + bias[d])        (torch's threshold: x > 20 -> x)
//
// A GEMM with M = D, N = L and a short reduction K = R (dt_rank = 8 .. 32 at every Mamba-TasNet size) whose output
// (b, D, l) is the bulk of its bytes: the kernel has to stream at HBM rate, and 2R fp32 FMAs per output element on
// the VALU did not (round-5 first version: 0.28 of HBM at C3, 0.16 at C5, VALU-bound).  So the products run on the
// MFMA (v_mfma_f32_32x32x16_*), fp32 accumulation:
//   - bf16 operands: bf16 MFMA on the values as they are (bf16 x bf16 products are exact in fp32);
//   - fp32 operands: the split of dconv.hip / projgemm.hip with per-TILE power-of-two scales (the tile's x slab and
//     W rows are in LDS anyway): hi = fp16(v 2^e), lo = fp16(v 2^e - hi), products hi*hi + hi*lo + lo*hi on the f16
//     MFMA, scaled back by 2^-(e_x + e_w) (22-bit operands: the fp32 class).
// Workgroup = 64 channels x 256 steps of one batch row, 4 waves of 64 channels x 64 steps (2 x 2 MFMA blocks); the
// output tile goes out through LDS in 1-KB coalesced rows (stores straight from the accumulators -- 32-B runs per
// row -- ran the C3 call at 0.60 ms against 0.48 for the VALU version).  x rows
// [0, R) x 256 steps are staged in LDS as 16-bit k-rows of 512 B (16-B chunk c of k-row r at c ^ ((r & 3) << 2),
// fragments by ds_read_b64_tr_b16), W's 64 rows as R-long 16-bit rows padded by 16 B (conflict-free 16-B reads).
// The workgroups of one x slab (its D / 64 channel tiles) are consecutive, so the slab is re-read from L2.
// bias + softplus in the epilogue; the bf16 output is rounded once.
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace avse {
namespace dtp {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef short s4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4_t lds_s4_t;

constexpr int THREADS = 256, CH = 64, TT = 256, RMAX = 64;

struct Args {
    int D, R, RP, L, nt, nd;
    const void* w;
    int64_t w_ds;
    const void* x;
    int64_t x_bs, x_rs;
    const float* bias;
    void* out;
    int64_t o_bs, o_ds;
    int softplus;
};

// same function as dconv.hip: max |v| 2^e in [2^14, 2^15)
__device__ inline int split_exp(uint32_t mb) {
    const int ef = (int)((mb >> 23) & 0xff);
    if (mb == 0) return 0;
    const int k = ef == 0 ? -127 : ef - 127;
    return min(100, max(-100, 14 - k));
}

template <typename T> struct ld4;
template <> struct ld4<float> {
    __device__ static inline float4 ld(__amdgpu_buffer_rsrc_t r, int e) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, e * 4, 0, 0);
        return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
    }
};
template <> struct ld4<bf16_t> {
    __device__ static inline float4 ld(__amdgpu_buffer_rsrc_t r, int e) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, e * 2, 0, 0);
        return make_float4(__uint_as_float(v[0] << 16), __uint_as_float(v[0] & 0xffff0000u),
                           __uint_as_float(v[1] << 16), __uint_as_float(v[1] & 0xffff0000u));
    }
};

__device__ inline uint16_t h16(float v) { return __builtin_bit_cast(uint16_t, (_Float16)v); }

// x image: k-row r (512 B = 256 steps of 16 bits), step t at r 512 + 16 ((t >> 3) ^ ((r & 3) << 2)) + 2 (t & 7)
__device__ inline int ximg_off(int r, int t) { return r * 512 + 16 * ((t >> 3) ^ ((r & 3) << 2)) + 2 * (t & 7); }

// B operand fragment (32 steps x 16 k) of steps cb .. cb + 31, k-substep s: lane l holds step cb + (l & 31),
// k = 16 s + 8 (l >> 5) + 0..7 — two transposed 4 x 16 reads per 16-lane group (projgemm.hip frag_raw, MN image)
__device__ inline s4_t tr(const uint8_t* img, int off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(img + off));
}
__device__ inline half8 xfrag(const uint8_t* img, int cb, int s, int lane) {
    const int g = lane >> 4, i = lane & 15;
    const int col = cb + 16 * (g & 1) + 4 * (i & 3);
    const int kb = 16 * s + 8 * (g >> 1) + (i >> 2);
    const s4_t v0 = tr(img, ximg_off(kb, col)), v1 = tr(img, ximg_off(kb + 4, col));
    const short __attribute__((ext_vector_type(8))) w = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    return __builtin_bit_cast(half8, w);
}
// A operand fragment (32 channels x 16 k) of channels rb .. rb + 31: lane l holds channel rb + (l & 31),
// k = 16 s + 8 (l >> 5) + 0..7 (one 16-B read of the channel's row)
__device__ inline half8 wfrag(const uint8_t* img, int wrow, int rb, int s, int lane) {
    return *reinterpret_cast<const half8*>(img + (rb + (lane & 31)) * wrow + 2 * (16 * s + 8 * (lane >> 5)));
}

template <typename T>
__global__ __launch_bounds__(THREADS) void dtproj_kernel(Args a) {
    constexpr bool F32 = std::is_same<T, float>::value;
    constexpr int NPL = F32 ? 2 : 1;                          // planes: hi, lo (fp32) or the bf16 values
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ uint32_t red[2][4];
    const int XB = a.RP * 512, wrow = 2 * a.RP + 16, WB = CH * wrow;
    uint8_t* ximg = lds;                                      // [plane][RP k-rows][512 B]
    uint8_t* wimg = lds + NPL * XB;                           // [plane][64 rows][wrow]
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int db = bid % a.nd, tb = (bid / a.nd) % a.nt, b = bid / (a.nd * a.nt);
    const int t0 = tb * TT, d0 = db * CH;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    // x slab: thread -> (k-row r, 4 steps); steps past L read 0 (the range ends at the row's last element) or row
    // padding (inside the range): either way they feed only unstored outputs
    const T* xb = reinterpret_cast<const T*>(a.x) + (int64_t)b * a.x_bs;
    const auto rx = make_rsrc(xb, (int64_t)(a.R - 1) * a.x_rs + a.L);
    constexpr int XPT = RMAX * (TT / 4) / THREADS;            // float4 per thread (upper bound: R <= 64)
    float4 xv[XPT];
    float mx = 0.f;
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
        const int i = tid + k * THREADS, r = i / (TT / 4), c4 = i % (TT / 4);
        xv[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r < a.R) {
            const int t = t0 + 4 * c4;
            if (t + 3 < a.L) {
                xv[k] = ld4<T>::ld(rx, (int)(r * a.x_rs) + t);
            } else if (t < a.L) {                             // the row's last partial quad
                const T* p = xb + (int64_t)r * a.x_rs + t;
                xv[k].x = io<T>::ld(p);
                xv[k].y = t + 1 < a.L ? io<T>::ld(p + 1) : 0.f;
                xv[k].z = t + 2 < a.L ? io<T>::ld(p + 2) : 0.f;
            }
        }
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(xv[k].x), fabsf(xv[k].y)), fmaxf(fabsf(xv[k].z), fabsf(xv[k].w))));
    }
    // W rows of the tile: thread -> (row, 4 k); rows past D and k past R are 0
    const T* w = reinterpret_cast<const T*>(a.w);
    constexpr int WPT = CH * RMAX / 4 / THREADS;
    float4 wv[WPT];
#pragma unroll
    for (int k = 0; k < WPT; ++k) {
        const int i = tid + k * THREADS, row = i / (RMAX / 4), k4 = 4 * (i % (RMAX / 4)), d = d0 + row;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (d < a.D && k4 + e < a.R) ? io<T>::ld(w + (int64_t)d * a.w_ds + k4 + e) : 0.f;
        wv[k] = make_float4(v[0], v[1], v[2], v[3]);
    }
    float sx = 1.f, sw = 1.f, unscale = 1.f;
    if constexpr (F32) {
        float mw = 0.f;
#pragma unroll
        for (int k = 0; k < WPT; ++k)
            mw = fmaxf(mw, fmaxf(fmaxf(fabsf(wv[k].x), fabsf(wv[k].y)), fmaxf(fabsf(wv[k].z), fabsf(wv[k].w))));
        uint32_t bx = __float_as_uint(mx), bw = __float_as_uint(mw);
        for (int o = 32; o >= 1; o >>= 1) {
            bx = max(bx, (uint32_t)__shfl_xor((int)bx, o, 64));
            bw = max(bw, (uint32_t)__shfl_xor((int)bw, o, 64));
        }
        if (lane == 0) {
            red[0][wave] = bx;
            red[1][wave] = bw;
        }
        __syncthreads();
        bx = max(max(red[0][0], red[0][1]), max(red[0][2], red[0][3]));
        bw = max(max(red[1][0], red[1][1]), max(red[1][2], red[1][3]));
        const int ex = split_exp(bx), ew = split_exp(bw);
        sx = __builtin_ldexpf(1.f, ex);
        sw = __builtin_ldexpf(1.f, ew);
        unscale = __builtin_ldexpf(1.f, -(ex + ew));
    }
    // LDS images (k-rows R .. RP - 1 of x are zero: their thread slots loaded 0)
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
        const int i = tid + k * THREADS, r = i / (TT / 4), c4 = i % (TT / 4);
        if (r >= a.RP) continue;
        const float v[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
        uint16_t h[4], l[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if constexpr (F32) {
                const float sv = v[e] * sx;
                const _Float16 hh = (_Float16)sv;
                h[e] = __builtin_bit_cast(uint16_t, hh);
                l[e] = h16(sv - (float)hh);
            } else {
                h[e] = (uint16_t)(__float_as_uint(v[e]) >> 16);        // the bf16 value as loaded
            }
        }
        const int off = ximg_off(r, 4 * c4);
        *reinterpret_cast<uint2*>(ximg + off) = make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
        if constexpr (F32)
            *reinterpret_cast<uint2*>(ximg + XB + off) = make_uint2(l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16));
    }
#pragma unroll
    for (int k = 0; k < WPT; ++k) {
        const int i = tid + k * THREADS, row = i / (RMAX / 4), k4 = 4 * (i % (RMAX / 4));
        if (k4 >= a.RP) continue;
        const float v[4] = {wv[k].x, wv[k].y, wv[k].z, wv[k].w};
        uint16_t h[4], l[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if constexpr (F32) {
                const float sv = v[e] * sw;
                const _Float16 hh = (_Float16)sv;
                h[e] = __builtin_bit_cast(uint16_t, hh);
                l[e] = h16(sv - (float)hh);
            } else {
                h[e] = (uint16_t)(__float_as_uint(v[e]) >> 16);
            }
        }
        const int off = row * wrow + 2 * k4;
        *reinterpret_cast<uint2*>(wimg + off) = make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
        if constexpr (F32)
            *reinterpret_cast<uint2*>(wimg + WB + off) = make_uint2(l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16));
    }
    __syncthreads();

    floatx16 acc[2][2];                                       // [channel block i][step block j]
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    const int tc = 64 * wave;                                 // this wave's steps tc .. tc + 63 of the tile
    for (int s = 0; s < a.RP / 16; ++s) {
        half8 wh[2], xh[2], wl[2], xl[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            wh[i] = wfrag(wimg, wrow, 32 * i, s, lane);
            if constexpr (F32) wl[i] = wfrag(wimg + WB, wrow, 32 * i, s, lane);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            xh[j] = xfrag(ximg, tc + 32 * j, s, lane);
            if constexpr (F32) xl[j] = xfrag(ximg + XB, tc + 32 * j, s, lane);
        }
#pragma unroll
        for (int pr = 0; pr < (F32 ? 3 : 1); ++pr)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if constexpr (F32) {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(pr == 2 ? wl[i] : wh[i], pr == 1 ? xl[j] : xh[j],
                                                                           acc[i][j], 0, 0, 0);
                    } else {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, wh[i]),
                                                                            __builtin_bit_cast(bf16x8, xh[j]), acc[i][j],
                                                                            0, 0, 0);
                    }
                }
    }

    // epilogue through LDS, 32 channels at a time: acc[i][j] register 4 g + e = channel d0 + 32 i + 8 g + 4 (lane >> 5)
    // + e, step t0 + tc + 32 j + (lane & 31) -> ot[channel][step] (rows padded by 4 floats: the two half-waves' rows
    // land on different banks), then every thread stores whole 16-B pieces of 32 rows x 256 steps (1 KB per wave
    // instruction, coalesced): the output is the kernel's bytes
    float* ot = reinterpret_cast<float*>(lds);                // [32][OS]
    constexpr int OS = TT + 4;
    T* ob = reinterpret_cast<T*>(a.out) + (int64_t)b * a.o_bs;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        __syncthreads();                                      // the images / the previous half's reads are done
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int dl = 8 * g + 4 * (lane >> 5) + e, d = d0 + 32 * i + dl;
                const float bv = (a.bias && d < a.D) ? a.bias[d] : 0.f;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    float v = acc[i][j][4 * g + e] * unscale + bv;
                    if (a.softplus) v = softplus2(v);
                    ot[dl * OS + tc + 32 * j + (lane & 31)] = v;
                }
            }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 32 * TT / 4 / THREADS; ++k) {
            const int idx = tid + k * THREADS, row = idx / (TT / 4), c4 = idx % (TT / 4);
            const int d = d0 + 32 * i + row, t = t0 + 4 * c4;
            if (d >= a.D || t >= a.L) continue;
            const float4 v4 = *reinterpret_cast<const float4*>(&ot[row * OS + 4 * c4]);
            T* o = ob + (int64_t)d * a.o_ds + t;
            const float v[4] = {v4.x, v4.y, v4.z, v4.w};
            if constexpr (F32) {
                if (t + 3 < a.L && ((uintptr_t)o & 15) == 0) {
                    *reinterpret_cast<float4*>(o) = v4;
                    continue;
                }
            } else {
                if (t + 3 < a.L && ((uintptr_t)o & 7) == 0) {
                    bf16_t h[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) io<bf16_t>::st(&h[e], v[e]);
                    *reinterpret_cast<uint2*>(o) = make_uint2((uint32_t)h[0].x | ((uint32_t)h[1].x << 16),
                                                              (uint32_t)h[2].x | ((uint32_t)h[3].x << 16));
                    continue;
                }
            }
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (t + e < a.L) io<T>::st(o + e, v[e]);
        }
    }
}

}  // namespace dtp
}  // namespace avse

using namespace avse::dtp;

extern "C" {

int avse_dtproj(int64_t batch, int64_t dim, int64_t rank, int64_t seqlen, int32_t dtype, const void* w, int64_t w_ds,
                const void* x, int64_t x_bs, int64_t x_rs, const float* bias, int32_t softplus, void* delta,
                int64_t delta_bs, int64_t delta_ds, avse_stream_t stream) {
    if (!w || !x || !delta) return AVSE_EINVAL;
    if (batch <= 0 || dim <= 0 || rank <= 0 || seqlen <= 0 || rank > RMAX) return AVSE_ESHAPE;
    if (dtype != AVSE_F32 && dtype != AVSE_BF16) return AVSE_EDTYPE;
    const int64_t es = dtype == AVSE_F32 ? 4 : 2;
    if (((uintptr_t)x % es) || x_rs < seqlen || x_bs < (rank - 1) * x_rs + seqlen || delta_ds < seqlen ||
        w_ds < rank)
        return AVSE_ESHAPE;
    // 32-bit buffer offsets within one batch row of x
    if (((rank - 1) * x_rs + seqlen + TT) * es >= (1LL << 31)) return AVSE_ESHAPE;
    Args a;
    a.D = (int)dim;
    a.R = (int)rank;
    a.RP = (int)((rank + 15) / 16 * 16);
    a.L = (int)seqlen;
    a.nt = (int)((seqlen + TT - 1) / TT);
    a.nd = (int)((dim + CH - 1) / CH);
    a.w = w;
    a.w_ds = w_ds;
    a.x = x;
    a.x_bs = x_bs;
    a.x_rs = x_rs;
    a.bias = bias;
    a.out = delta;
    a.o_bs = delta_bs;
    a.o_ds = delta_ds;
    a.softplus = softplus;
    const int64_t nblocks = batch * a.nt * a.nd;
    if (nblocks >= (1LL << 31)) return AVSE_ESHAPE;
    const int npl = dtype == AVSE_F32 ? 2 : 1;
    // the operand images, later the 32 x (256 + 4)-float output staging
    const size_t lds = std::max<size_t>((size_t)npl * (a.RP * 512 + CH * (2 * a.RP + 16)), (size_t)32 * (TT + 4) * 4);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == AVSE_F32)
        hipLaunchKernelGGL(dtproj_kernel<float>, dim3((unsigned)nblocks), dim3(THREADS), lds, st, a);
    else
        hipLaunchKernelGGL(dtproj_kernel<avse::bf16_t>, dim3((unsigned)nblocks), dim3(THREADS), lds, st, a);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
