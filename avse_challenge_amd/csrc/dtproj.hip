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
// (b, D, l) is nearly all of its bytes: a write stream.  The products run on the MFMA (v_mfma_f32_32x32x16_*, fp32
// accumulation):
//   - bf16 operands: bf16 MFMA on the values as they are (bf16 x bf16 products are exact in fp32);
//   - fp32 operands: the split of dconv.hip / projgemm.hip with power-of-two scales per x tile and per W tile:
//     hi = fp16(v 2^e), lo = fp16(v 2^e - hi), products hi*hi + hi*lo + lo*hi on the f16 MFMA, scaled back by
//     2^-(e_x + e_w) (22-bit operands: the fp32 class).
// Schedule (round 5, fourth version): one workgroup per (batch row, 256-step tile) walks ALL channels.  The x slab
// (R rows x 256 steps) is staged once through LDS (16-bit k-rows of 512 B, 16-B chunk c of k-row r at
// c ^ ((r & 3) << 2), read by ds_read_b64_tr_b16) into per-wave MFMA A fragments (steps as the rows) that stay in
// registers; the channel loop then reads no LDS and has no barrier: W fragments (lane = channel, 8 consecutive k: one
// or two 16-B loads) are loaded one 32-channel tile ahead, so a tile's stores drain while the next one multiplies.
// Each lane ends with 4 consecutive steps of one channel: one 16-B (fp32) / 8-B (bf16) store.  bias + softplus in
// the epilogue; the bf16 output is rounded once.  <= 128 VGPRs (4 waves per SIMD at dt_rank <= 32).
// Isolated (tools/dtproj_bench.py, profiles/r05v_dtproj_ab.jsonl): C5 bf16 0.18 ms (the VALU version 0.28, the
// earlier MFMA versions with one workgroup per (64 channels, 256 steps) 0.31-0.34), C3 fp32 0.43 (VALU 0.41).
#include "common.h"

namespace avse {
namespace dtp {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef short s4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4_t lds_s4_t;

constexpr int THREADS = 256, CH = 32, TT = 256, RMAX = 64;

struct Args {
    int D, R, L, nt, nd;
    bool wvec;
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
// One lane's 8 W values of an MFMA B fragment: channel d, k = k0 .. k0 + 7 (0 past D or R).  wvec: rows of 8-element
// multiples, 16-B aligned, R % 8 == 0 (the model's dt_proj.weight) -> 16-B loads; otherwise element loads.
template <typename T>
__device__ inline void wload(const T* __restrict__ w, int64_t w_ds, int D, int R, int d, int k0, bool wvec, float (&o)[8]) {
    if (d < D && k0 < R && wvec) {
        const T* p = w + (int64_t)d * w_ds + k0;
        if constexpr (std::is_same<T, float>::value) {
            const float4 v0 = *reinterpret_cast<const float4*>(p), v1 = *reinterpret_cast<const float4*>(p + 4);
            o[0] = v0.x; o[1] = v0.y; o[2] = v0.z; o[3] = v0.w;
            o[4] = v1.x; o[5] = v1.y; o[6] = v1.z; o[7] = v1.w;
        } else {
            const uint4 v = *reinterpret_cast<const uint4*>(p);
            const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                o[2 * e] = __uint_as_float(u[e] << 16);
                o[2 * e + 1] = __uint_as_float(u[e] & 0xffff0000u);
            }
        }
        return;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (d < D && k0 + e < R) ? io<T>::ld(w + (int64_t)d * w_ds + k0 + e) : 0.f;
}

template <typename T, int NKS>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(4))) void dtproj_kernel(Args a) {
    constexpr bool F32 = std::is_same<T, float>::value;
    constexpr int RP = 16 * NKS;
    constexpr int XB = RP * 512;                              // one plane of the x image
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ uint32_t red[4];
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int tb = bid % a.nt, b = bid / a.nt;
    const int t0 = tb * TT;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    // x slab: thread -> (k-row r, 4 steps); steps past L and rows past R are 0 (the tile's split scale sees only data)
    const T* xb = reinterpret_cast<const T*>(a.x) + (int64_t)b * a.x_bs;
    const auto rx = make_rsrc(xb, (int64_t)(a.R - 1) * a.x_rs + a.L);
    constexpr int XPT = RP * (TT / 4) / THREADS;
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
    float sx = 1.f;
    int ex = 0;
    if constexpr (F32) {
        uint32_t bx = __float_as_uint(mx);
        for (int o = 32; o >= 1; o >>= 1) bx = max(bx, (uint32_t)__shfl_xor((int)bx, o, 64));
        if (lane == 0) red[wave] = bx;
        __syncthreads();
        bx = max(max(red[0], red[1]), max(red[2], red[3]));
        ex = split_exp(bx);
        sx = __builtin_ldexpf(1.f, ex);
    }
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
        const int i = tid + k * THREADS, r = i / (TT / 4), c4 = i % (TT / 4);
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
        *reinterpret_cast<uint2*>(lds + off) = make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
        if constexpr (F32)
            *reinterpret_cast<uint2*>(lds + XB + off) = make_uint2(l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16));
    }
    __syncthreads();
    // the wave's x fragments (steps tc .. tc + 63 as the MFMA rows) stay in registers for every channel tile: the
    // loop below reads no LDS and has no barrier, so one tile's stores drain while the next one computes
    const int tc = 64 * wave;
    half8 xh[2][NKS], xl[2][NKS];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
            xh[j][s] = xfrag(lds, tc + 32 * j, s, lane);
            if constexpr (F32) xl[j][s] = xfrag(lds + XB, tc + 32 * j, s, lane);
        }

    const T* w = reinterpret_cast<const T*>(a.w);
    T* ob = reinterpret_cast<T*>(a.out) + (int64_t)b * a.o_bs;
    const int kl = 8 * (lane >> 5);
    // channel tiles of 32 (one MFMA column block): 32 accumulators, the x fragments and the next tile's W in flight
    // fit ~100 VGPRs, i.e. 4+ waves per SIMD to cover the loads' and stores' latency
    float wn[NKS][8];                                         // this tile's W fragment (loaded one tile ahead)
#pragma unroll
    for (int s = 0; s < NKS; ++s) wload<T>(w, a.w_ds, a.D, a.R, lane & 31, 16 * s + kl, a.wvec, wn[s]);
    for (int d0 = 0; d0 < a.D; d0 += CH) {
        const int d = d0 + (lane & 31);
        // B fragments (lane = channel d, k = 16 s + kl .. + 7); fp32: split with the tile's scale (every wave holds
        // all 32 x RP W values of the tile: one wave max)
        half8 wh[NKS], wl[NKS];
        float unscale = 1.f;
        if constexpr (F32) {
            float mw = 0.f;
#pragma unroll
            for (int s = 0; s < NKS; ++s)
#pragma unroll
                for (int e = 0; e < 8; ++e) mw = fmaxf(mw, fabsf(wn[s][e]));
            uint32_t bw = __float_as_uint(mw);
            for (int o = 32; o >= 1; o >>= 1) bw = max(bw, (uint32_t)__shfl_xor((int)bw, o, 64));
            const int ew = split_exp(bw);
            const float sw = __builtin_ldexpf(1.f, ew);
            unscale = __builtin_ldexpf(1.f, -(ex + ew));
#pragma unroll
            for (int s = 0; s < NKS; ++s)
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float sv = wn[s][e] * sw;
                    const _Float16 hh = (_Float16)sv;
                    wh[s][e] = hh;
                    wl[s][e] = (_Float16)(sv - (float)hh);
                }
        } else {
#pragma unroll
            for (int s = 0; s < NKS; ++s)
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    wh[s][e] = __builtin_bit_cast(_Float16, (uint16_t)(__float_as_uint(wn[s][e]) >> 16));
        }
        if (d0 + CH < a.D) {                                  // the next tile's W, in flight during this tile
#pragma unroll
            for (int s = 0; s < NKS; ++s) wload<T>(w, a.w_ds, a.D, a.R, d + CH, 16 * s + kl, a.wvec, wn[s]);
        }
        floatx16 acc[2];                                      // [step block j]
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
        if constexpr (F32) {
            // C^T = W x: the W fragment as the A operand (its rows are the channels), the x fragment as B (its columns
            // are the steps), so a lane ends with ONE step of 16 channels and a store instruction writes whole 128-B
            // rows: per register a wave instruction writes 32 consecutive steps of two channel rows.  Round 5's order
            // (a lane = one channel, 4 steps; 32 rows x 32 B per instruction) ran the C3 call in 0.439 ms, this one in
            // 0.327 (profiles/r06k_dtproj_ab.jsonl).  bf16 keeps that order: 2-B stores per lane would write 64-B
            // half rows (0.243 vs 0.177 ms at C5).
#pragma unroll
            for (int s = 0; s < NKS; ++s)
#pragma unroll
                for (int pr = 0; pr < 3; ++pr)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(pr == 1 ? wl[s] : wh[s],
                                                                        pr == 2 ? xl[j][s] : xh[j][s], acc[j], 0, 0, 0);
            // acc[j] register 4 g + e = channel d0 + 8 g + 4 (lane >> 5) + e at step ts + 32 j
            const int ts = t0 + tc + (lane & 31);
            float bv[4][4];
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int dd = d0 + 8 * g + 4 * (lane >> 5) + e;
                    bv[g][e] = (a.bias && dd < a.D) ? a.bias[dd] : 0.f;
                }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int t = ts + 32 * j;
                if (t >= a.L) continue;
#pragma unroll
                for (int g = 0; g < 4; ++g)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int dd = d0 + 8 * g + 4 * (lane >> 5) + e;
                        if (dd >= a.D) continue;
                        float v = acc[j][4 * g + e] * unscale + bv[g][e];
                        if (a.softplus) v = softplus2(v);
                        ob[(int64_t)dd * a.o_ds + t] = v;
                    }
            }
        } else {
#pragma unroll
            for (int s = 0; s < NKS; ++s)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xh[j][s]),
                                                                     __builtin_bit_cast(bf16x8, wh[s]), acc[j], 0, 0, 0);
            // acc[j] register 4 g + e = step tl + 32 j + 8 g + e of channel d: four consecutive steps per lane -> one
            // 8-B store
            if (d >= a.D) continue;
            const float bvd = a.bias ? a.bias[d] : 0.f;
            const int tl = t0 + tc + 4 * (lane >> 5);
            T* orow = ob + (int64_t)d * a.o_ds;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int t = tl + 32 * j + 8 * g;
                    if (t >= a.L) continue;
                    float v[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v[e] = acc[j][4 * g + e] * unscale + bvd;
                        if (a.softplus) v[e] = softplus2(v[e]);
                    }
                    T* o = orow + t;
                    if (t + 3 < a.L && ((uintptr_t)o & 7) == 0) {
                        bf16_t h[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) io<bf16_t>::st(&h[e], v[e]);
                        *reinterpret_cast<uint2*>(o) = make_uint2((uint32_t)h[0].x | ((uint32_t)h[1].x << 16),
                                                                  (uint32_t)h[2].x | ((uint32_t)h[3].x << 16));
                        continue;
                    }
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (t + e < a.L) io<T>::st(o + e, v[e]);
                }
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
    a.L = (int)seqlen;
    a.nt = (int)((seqlen + TT - 1) / TT);
    a.nd = (int)((dim + CH - 1) / CH);
    a.w = w;
    a.w_ds = w_ds;
    // 16-B W fragment loads: rows of 8-element multiples (bf16: 16 B; fp32: two 16-B halves), 16-B aligned base
    a.wvec = (rank % 8 == 0) && ((uintptr_t)w % 16 == 0) && ((w_ds * es) % 16 == 0);
    a.x = x;
    a.x_bs = x_bs;
    a.x_rs = x_rs;
    a.bias = bias;
    a.out = delta;
    a.o_bs = delta_bs;
    a.o_ds = delta_ds;
    a.softplus = softplus;
    // one workgroup per (batch row, 256-step tile), looping over the channel tiles
    const int64_t nblocks = batch * a.nt;
    if (nblocks >= (1LL << 31)) return AVSE_ESHAPE;
    const int nks = (int)((rank + 15) / 16);
    const size_t lds = (size_t)(dtype == AVSE_F32 ? 2 : 1) * nks * 16 * 512;   // the x image (hi, lo planes)
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)nblocks), blk(THREADS);
#define AVSE_DTP_LAUNCH(T)                                                          \
    switch (nks) {                                                                  \
        case 1: hipLaunchKernelGGL((dtproj_kernel<T, 1>), grid, blk, lds, st, a); break; \
        case 2: hipLaunchKernelGGL((dtproj_kernel<T, 2>), grid, blk, lds, st, a); break; \
        case 3: hipLaunchKernelGGL((dtproj_kernel<T, 3>), grid, blk, lds, st, a); break; \
        default: hipLaunchKernelGGL((dtproj_kernel<T, 4>), grid, blk, lds, st, a); break; \
    }
    if (dtype == AVSE_F32) {
        AVSE_DTP_LAUNCH(float)
    } else {
        AVSE_DTP_LAUNCH(avse::bf16_t)
    }
#undef AVSE_DTP_LAUNCH
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
