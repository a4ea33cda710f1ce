// dt_proj with the selective scan's softplus folded into its epilogue, for gfx950.
//
// Replaces the step-size projection of MambaInnerFnNoOutProj
//   delta = delta_proj_weight @ x_dbl[:, :delta_rank].t()          Mamba-TasNet/modules/mamba/selective_scan_interface.py:187
// together with the `delta = softplus(delta + delta_bias)` that selective_scan_cuda applies per element inside the
// scan (semantics: selective_scan_ref, :110-112).  The scan kernels then read the final step sizes (mode
// delta_softplus = 2 of avse_scan_fwd / avse_scan_bwd) and evaluate no softplus per element: that staging was about a
// quarter of the scan forward's VALU cycles, and the backward re-evaluated it a second time.
//
//   delta[b][d][t] = softplus(sum_r W[d][r] * x[b][r][t] + bias[d])        (torch's threshold: x > 20 -> x)
//
// The reduction is short (R = dt_rank = 8 .. 32 at every Mamba-TasNet size) and the output is (b, d, l): the kernel
// is a write stream with 2R FMAs per element, so it runs on the VALU with both operands from LDS.
// Workgroup = 64 channels x 256 steps: x[b][0..R)[t0 .. t0+256) and W^T of the 64 channels are staged in LDS once;
// wave w owns channels 16 w .. 16 w + 15, lane l the steps t0 + 4 l .. + 3, so per r a lane reads one float4 of x and
// four broadcast float4 of W (all lanes the same address) for 64 FMAs.  fp32 accumulation for either dtype; bf16
// output is rounded once, after the softplus.
#include <type_traits>

#include "common.h"

namespace avse {
namespace dtp {

constexpr int THREADS = 256, CH = 64, TT = 256, RMAX = 64;

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

struct Args {
    int D, R, L, nt, nd;
    const void* w;
    int64_t w_ds;
    const void* x;
    int64_t x_bs, x_rs;
    const float* bias;
    void* out;
    int64_t o_bs, o_ds;
    int softplus;
};

template <typename T>
__global__ __launch_bounds__(THREADS) void dtproj_kernel(Args a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* sx = lds;                         // [R][TT]
    float* sw = lds + a.R * TT;              // [R][CH]: W^T of the block's channels
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int tb = bid % a.nt, db = (bid / a.nt) % a.nd, b = bid / (a.nt * a.nd);
    const int t0 = tb * TT, d0 = db * CH;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    // x rows (4 steps per load; steps past L read row padding or 0 past the buffer: they feed unstored outputs only)
    const T* xb = reinterpret_cast<const T*>(a.x) + (int64_t)b * a.x_bs;
    const auto rx = make_rsrc(xb, (int64_t)(a.R - 1) * a.x_rs + a.L);
    for (int i = tid; i < a.R * (TT / 4); i += THREADS) {
        const int r = i / (TT / 4), c4 = i % (TT / 4);
        const int t = t0 + 4 * c4;
        float4 v;
        if (t + 3 < a.L) {
            v = ld4<T>::ld(rx, (int)(r * a.x_rs) + t);
        } else {                             // the row's last partial quad: element loads, steps past L as 0
            const T* p = xb + (int64_t)r * a.x_rs + t;
            v.x = t < a.L ? io<T>::ld(p) : 0.f;
            v.y = t + 1 < a.L ? io<T>::ld(p + 1) : 0.f;
            v.z = t + 2 < a.L ? io<T>::ld(p + 2) : 0.f;
            v.w = 0.f;
        }
        *reinterpret_cast<float4*>(&sx[r * TT + 4 * c4]) = v;
    }
    const T* w = reinterpret_cast<const T*>(a.w);
    for (int i = tid; i < a.R * CH; i += THREADS) {
        const int c = i % CH, r = i / CH, d = d0 + c;
        sw[r * CH + c] = d < a.D ? io<T>::ld(w + (int64_t)d * a.w_ds + r) : 0.f;
    }
    __syncthreads();

    float4 acc[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    const float* wrow = sw + wave * 16;
#pragma unroll 4
    for (int r = 0; r < a.R; ++r) {
        const float4 xv = *reinterpret_cast<const float4*>(&sx[r * TT + 4 * lane]);
        float wv[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 w4 = *reinterpret_cast<const float4*>(&wrow[r * CH + 4 * q]);
            wv[4 * q] = w4.x; wv[4 * q + 1] = w4.y; wv[4 * q + 2] = w4.z; wv[4 * q + 3] = w4.w;
        }
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            acc[c].x = __builtin_fmaf(wv[c], xv.x, acc[c].x);
            acc[c].y = __builtin_fmaf(wv[c], xv.y, acc[c].y);
            acc[c].z = __builtin_fmaf(wv[c], xv.z, acc[c].z);
            acc[c].w = __builtin_fmaf(wv[c], xv.w, acc[c].w);
        }
    }

    const int t = t0 + 4 * lane;
    if (t >= a.L) return;
    const bool full = t + 3 < a.L;
    T* ob = reinterpret_cast<T*>(a.out) + (int64_t)b * a.o_bs + t;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        const int d = d0 + wave * 16 + c;
        if (d >= a.D) break;
        const float bv = a.bias ? a.bias[d] : 0.f;
        float v[4] = {acc[c].x + bv, acc[c].y + bv, acc[c].z + bv, acc[c].w + bv};
        if (a.softplus) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = softplus2(v[e]);
        }
        T* o = ob + (int64_t)d * a.o_ds;
        if constexpr (std::is_same<T, float>::value) {
            if (full && ((uintptr_t)o & 15) == 0) {
                *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
                continue;
            }
        } else {
            if (full && ((uintptr_t)o & 7) == 0) {
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
    const size_t lds = (size_t)rank * (TT + CH) * 4;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == AVSE_F32)
        hipLaunchKernelGGL(dtproj_kernel<float>, dim3((unsigned)nblocks), dim3(THREADS), lds, st, a);
    else
        hipLaunchKernelGGL(dtproj_kernel<avse::bf16_t>, dim3((unsigned)nblocks), dim3(THREADS), lds, st, a);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
