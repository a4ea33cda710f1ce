// Persistent single-layer LSTM recurrence for gfx950 (MI355X): avse1 FusionNet and the avse2 DPRNN LSTMs.
//
// Replaces the per-time-step cuDNN/MIOpen LSTM the reference runs through nn.LSTM
// (/root/reference/baseline/avse1/model.py:88 `nn.LSTM(1540, 257, num_layers=1, batch_first=True)`,
//  /root/reference/baseline/avse2/model.py:101-102 bidirectional DPRNN LSTMs).  PyTorch gate order i, f, g, o;
// h0 = c0 = 0; c_t = f c_{t-1} + i g; h_t = o tanh(c_t).
//
// Split of the work (the caller does the dense parts as GEMMs):
//   forward:  gx = X W_ih^T + b_ih + b_hh for ALL steps is one GEMM (caller); this kernel runs the recurrence
//             g_t = gx_t + W_hh h_{t-1} and the cell update for every step inside ONE launch — one workgroup per
//             sequence, thread j owning gate rows 4j..4j+3 (float4 rows of W_hh^T, coalesced across the wave) and
//             hidden unit j; h_{t-1} is broadcast from LDS.  W_hh (1 MB fp32 at H = 257) stays L2-resident and is
//             streamed once per step per sequence.  Saves h, c and the gate activations for the backward.
//   backward: the adjoint recurrence dh_{t-1} = W_hh^T dg_t (dg = pre-activation gate gradients), again one launch,
//             the 4H-long dot products split over 4 row slices per float4 column group; the caller forms
//             dX = dg W_ih, dW_ih = dg^T X, dW_hh = dg^T h_{t-1}, db = sum dg as GEMMs.
// No atomics, no grid synchronisation, deterministic.
#include "common.h"

namespace avse {
namespace lstm {

constexpr int MAXH = 512;

__device__ inline float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__global__ void fwd_kernel(int T, int H, int reverse, const float* __restrict__ gx, const float* __restrict__ whhT,
                           float* __restrict__ hout, int64_t hout_bs, int64_t hout_ts, float* __restrict__ c_all,
                           float* __restrict__ gates) {
    extern __shared__ float sm[];
    float* s_h = sm;                 // h_{t-1}  [H]
    float* s_gp = sm + ((H + 3) & ~3);   // pre-activation gates [4H] (16-B aligned)
    const int b = blockIdx.x, j = threadIdx.x;
    const bool act = j < H;
    const int H4 = 4 * H;
    float c = 0.f;
    if (act) s_h[j] = 0.f;
    __syncthreads();
    const float4* W4 = reinterpret_cast<const float4*>(whhT);     // row k = H float4 (gate rows 4m..4m+3)
    for (int s = 0; s < T; ++s) {
        const int t = reverse ? T - 1 - s : s;
        const int64_t bt = (int64_t)b * T + t;
        if (act) {
            float4 acc = reinterpret_cast<const float4*>(gx + bt * H4)[j];
            int k = 0;
#pragma unroll 8
            for (; k < H; ++k) {
                const float4 w = W4[(int64_t)k * H + j];
                const float hk = s_h[k];
                acc.x = fmaf(w.x, hk, acc.x);
                acc.y = fmaf(w.y, hk, acc.y);
                acc.z = fmaf(w.z, hk, acc.z);
                acc.w = fmaf(w.w, hk, acc.w);
            }
            reinterpret_cast<float4*>(s_gp)[j] = acc;
        }
        __syncthreads();
        if (act) {
            const float ig = sigm(s_gp[j]), fg = sigm(s_gp[H + j]), gg = tanhf(s_gp[2 * H + j]),
                        og = sigm(s_gp[3 * H + j]);
            c = fmaf(fg, c, ig * gg);
            const float h = og * tanhf(c);
            s_h[j] = h;                                  // every read of h_{t-1} finished before the barrier
            hout[(int64_t)b * hout_bs + (int64_t)t * hout_ts + j] = h;
            c_all[bt * H + j] = c;
            float* gt = gates + bt * H4;
            gt[j] = ig;
            gt[H + j] = fg;
            gt[2 * H + j] = gg;
            gt[3 * H + j] = og;
        }
        __syncthreads();
    }
}

__global__ void bwd_kernel(int T, int H, int Hp, int reverse, const float* __restrict__ dh_out, int64_t dh_bs,
                           int64_t dh_ts, const float* __restrict__ gates, const float* __restrict__ c_all,
                           const float* __restrict__ whh_pad, float* __restrict__ dgp) {
    extern __shared__ float sm[];
    const int H4 = 4 * H;
    float* s_dg = sm;                        // [4H] pre-activation gate gradients of the step
    float* s_part = sm + ((H4 + 3) & ~3);    // [4][Hp] partial dh over the 4 gate-row slices
    float* s_dh = s_part + 4 * Hp;           // [Hp] dh_{t-1} contribution W_hh^T dg_t
    const int b = blockIdx.x, q = threadIdx.x;
    const bool act = q < H;
    const int ncg = Hp / 4;                  // float4 column groups of the padded W_hh rows
    const int cg = q % ncg, rs = q / ncg;    // GEMV role: column group, row slice (4 slices of H rows)
    const bool gemv = q < 4 * ncg;
    if (q < Hp) s_dh[q] = 0.f;
    float dc_carry = 0.f;
    __syncthreads();
    const float4* W4 = reinterpret_cast<const float4*>(whh_pad);   // row r = Hp/4 float4
    for (int s = 0; s < T; ++s) {
        const int t = reverse ? s : T - 1 - s;                        // reverse order of the forward
        const int tp = reverse ? t + 1 : t - 1;                        // the forward's previous step
        const int64_t bt = (int64_t)b * T + t;
        if (act) {
            const float* gt = gates + bt * H4;
            const float ig = gt[q], fg = gt[H + q], gg = gt[2 * H + q], og = gt[3 * H + q];
            const float c = c_all[bt * H + q];
            const float cp = (tp >= 0 && tp < T) ? c_all[((int64_t)b * T + tp) * H + q] : 0.f;
            const float dh = dh_out[(int64_t)b * dh_bs + (int64_t)t * dh_ts + q] + s_dh[q];
            const float tc = tanhf(c);
            const float dc = fmaf(dh * og, 1.f - tc * tc, dc_carry);
            const float di = dc * gg * ig * (1.f - ig);
            const float df = dc * cp * fg * (1.f - fg);
            const float dg = dc * ig * (1.f - gg * gg);
            const float dO = dh * tc * og * (1.f - og);
            dc_carry = dc * fg;
            s_dg[q] = di;
            s_dg[H + q] = df;
            s_dg[2 * H + q] = dg;
            s_dg[3 * H + q] = dO;
            float* o = dgp + bt * H4;
            o[q] = di;
            o[H + q] = df;
            o[2 * H + q] = dg;
            o[3 * H + q] = dO;
        }
        __syncthreads();
        if (gemv) {
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
            const int r0 = rs * H;
#pragma unroll 8
            for (int r = r0; r < r0 + H; ++r) {
                const float4 w = W4[(int64_t)r * ncg + cg];
                const float d = s_dg[r];
                acc.x = fmaf(w.x, d, acc.x);
                acc.y = fmaf(w.y, d, acc.y);
                acc.z = fmaf(w.z, d, acc.z);
                acc.w = fmaf(w.w, d, acc.w);
            }
            reinterpret_cast<float4*>(s_part + rs * Hp)[cg] = acc;
        }
        __syncthreads();
        if (q < Hp) s_dh[q] = (s_part[q] + s_part[Hp + q]) + (s_part[2 * Hp + q] + s_part[3 * Hp + q]);
        __syncthreads();
    }
}

}  // namespace lstm
}  // namespace avse

using namespace avse;

extern "C" {

int64_t avse_lstm_padded_hidden(int64_t H) { return (H + 3) & ~(int64_t)3; }

int avse_lstm_fwd(int64_t B, int64_t T, int64_t H, int32_t reverse, const float* gx, const float* whhT, float* hout,
                  int64_t hout_bs, int64_t hout_ts, float* c_all, float* gates, avse_stream_t stream) {
    if (!gx || !whhT || !hout || !c_all || !gates) return AVSE_EINVAL;
    if (B <= 0 || T <= 0 || H <= 0 || H > lstm::MAXH || B > 0x7FFFFFFF) return AVSE_ESHAPE;
    if (((uintptr_t)gx | (uintptr_t)whhT) & 15) return AVSE_EALIGN;
    const int threads = (int)((H + 63) / 64 * 64);
    const size_t lds = sizeof(float) * (size_t)(((H + 3) & ~3) + 4 * H);
    hipLaunchKernelGGL(lstm::fwd_kernel, dim3((unsigned)B), dim3(threads), lds, (hipStream_t)stream, (int)T, (int)H,
                       (int)reverse, gx, whhT, hout, hout_bs, hout_ts, c_all, gates);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_lstm_bwd(int64_t B, int64_t T, int64_t H, int32_t reverse, const float* dh_out, int64_t dh_bs, int64_t dh_ts,
                  const float* gates, const float* c_all, const float* whh_pad, float* dgates, avse_stream_t stream) {
    if (!dh_out || !gates || !c_all || !whh_pad || !dgates) return AVSE_EINVAL;
    if (B <= 0 || T <= 0 || H <= 0 || H > lstm::MAXH || B > 0x7FFFFFFF) return AVSE_ESHAPE;
    if ((uintptr_t)whh_pad & 15) return AVSE_EALIGN;
    const int Hp = (int)avse_lstm_padded_hidden(H);
    const int threads = (int)((H + 63) / 64 * 64);
    if (threads < Hp) return AVSE_ESHAPE;                 // H in (60, 64] etc.: Hp = H rounded to 4 <= threads always
    const size_t lds = sizeof(float) * (size_t)(((4 * H + 3) & ~3) + 5 * Hp);
    hipLaunchKernelGGL(lstm::bwd_kernel, dim3((unsigned)B), dim3(threads), lds, (hipStream_t)stream, (int)T, (int)H,
                       Hp, (int)reverse, dh_out, dh_bs, dh_ts, gates, c_all, whh_pad, dgates);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
