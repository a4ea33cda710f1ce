// bf16 MFMA GEMM for the Mamba projections on gfx950 (v_mfma_f32_32x32x16_bf16, fp32 accumulation).
//
// Replaces the bf16 GEMMs that BiMamba v2 runs under autocast (BASELINE configs[4]):
//   in_proj   xz = W_in h^T                      Mamba-TasNet/modules/mamba/bimamba.py:190-196
//   out_proj  out = (0.5 f + 0.5 b)^T W_out^T    bimamba.py:250-253
// and their input gradients (the backward of the same torch.nn.functional.linear calls).  The model keeps every
// (b, channels, l) activation in the scan's layout with a padded time stride, so the four GEMMs see operands whose
// contiguous dimension is either the reduction (K-contiguous: h (b, l, d_model), the weights' rows) or the output
// dimension (MN-contiguous: xz / y (b, channels, l) read along channels).  One kernel template covers all of them:
//
//   C[b][q][p] = alpha * sum_k P[b][p][k] * Q[b][q][k]        (p contiguous in C; batch stride 0 = a shared weight)
//
// P feeds the MFMA's rows, so each lane's accumulator holds 4 consecutive p (one 8-byte bf16 store).
//
// Tiling: 256 threads, 128 (p) x 128 (q) per workgroup, 2 x 2 waves of 64 x 64 (2 x 2 MFMA blocks of 32 x 32),
// K in stages of 64 staged HBM -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds: out-of-range reads land as 0), two
// stage buffers (64 KB: 2 workgroups per CU, the other one's MFMAs cover a stage's load latency).
// LDS images per operand and stage (16 KB):
//   K-contiguous: 128 rows x 128 B (64 k); 16-B chunk c of row r stored at c ^ ((r >> 1) & 7), so the fragment
//     reads (ds_read_b128, lane = row) of a 16-lane group hit 16 distinct 16-B bank slots;
//   MN-contiguous: 64 k-rows x 256 B (128 p or q); chunk c of k-row r at c ^ ((r & 3) << 2); fragments by
//     ds_read_b64_tr_b16 (4 k-rows x 16 columns per 16-lane group, delivered column-major), conflict-free per half.
// The swizzle is applied to the DMA's per-lane SOURCE address (the LDS side of an LDS-DMA is lane-linear).
// Workgroup order: the tile index of the shared weight (batch stride 0) runs fastest and neighbouring ids share an
// XCD (xcd_remap), so an activation tile is fetched from HBM once and re-read from that XCD's L2.
#include "common.h"

namespace avse {
namespace pg {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s4_t __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) s4_t lds_s4_t;

constexpr int BP = 128, BQ = 128, BK = 64, THREADS = 256;
constexpr int IMG = 16384;                 // one operand's image of one stage
constexpr int STAGE = 2 * IMG;
constexpr int NSTAGE = 2;

struct Args {
    const uint16_t* p;
    const uint16_t* q;
    void* c;
    int64_t p_bs, q_bs, c_bs;              // batch strides (elements)
    int64_t p_ext, q_ext;                  // elements addressable from p / q (for the buffer range)
    int32_t p_sx, q_sx;                    // stride of the p / q index (K-contiguous operand) or of k (MN-contiguous)
    int32_t c_sq;
    int32_t mp, mq, k, batch;
    int32_t tp, tq;                        // tile counts
    int32_t q_fast;                        // q tile index runs fastest in the workgroup order
    float alpha;
};

__device__ inline __amdgpu_buffer_rsrc_t rsrc_from(const uint16_t* base, int64_t elems) {
    int64_t bytes = elems * 2;
    if (bytes > 0x7FFFFFF0LL) bytes = 0x7FFFFFF0LL;
    if (bytes < 0) bytes = 0;
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

// One operand's stage (BK k x 128 rows) HBM -> LDS image.  KC: the operand is K-contiguous (row x0 + r has stride sx,
// k is contiguous); otherwise k-row k0 + r has stride sx and the 128 rows are contiguous.  Rows past mx are clamped
// (KC) or read whatever lies there / 0 past the buffer (MN); they only feed outputs that are never stored.
template <bool KC>
__device__ inline void stage_load(__amdgpu_buffer_rsrc_t r, uint8_t* img, int x0, int k0, int sx, int mx, int wave,
                                  int lane) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int piece = wave * 4 + j;                        // 1 KB of the image per wave-instruction
        uint32_t voff;
        if constexpr (KC) {
            const int row = piece * 8 + (lane >> 3);
            const int xr = min(x0 + row, mx - 1);
            const int c = (lane & 7) ^ ((row >> 1) & 7);
            voff = (uint32_t)(xr * sx + k0 + c * 8) * 2u;
        } else {
            const int krow = piece * 4 + (lane >> 4);
            const int c = (lane & 15) ^ ((krow & 3) << 2);
            voff = (uint32_t)((k0 + krow) * sx + x0 + c * 8) * 2u;
        }
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(img + piece * 1024), 16, voff, 0, 0, 0);
    }
}

// The 32 x 16 (row x k) MFMA operand fragment of rows rb .. rb + 31, k-substep s (k = 16 s .. 16 s + 15):
// lane l holds row rb + (l & 31), k = 16 s + 8 (l >> 5) + 0..7.
template <bool KC>
__device__ inline bf16x8 frag(const uint8_t* img, int rb, int s, int lane) {
    if constexpr (KC) {
        const int row = rb + (lane & 31);
        const int ch = 2 * s + (lane >> 5);
        return *reinterpret_cast<const bf16x8*>(img + row * 128 + 16 * (ch ^ ((row >> 1) & 7)));
    } else {
        const int g = lane >> 4, i = lane & 15;
        const int col = rb + 16 * (g & 1) + 4 * (i & 3);
        const int kb = 16 * s + 8 * (g >> 1) + (i >> 2);
        s4_t v[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int kr = kb + 4 * u;
            const int off = kr * 256 + 16 * ((col >> 3) ^ ((kr & 3) << 2)) + (col & 7) * 2;
            v[u] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(img + off));
        }
        typedef short s8_t __attribute__((ext_vector_type(8)));
        const s8_t w = {v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3]};
        return __builtin_bit_cast(bf16x8, w);
    }
}

__device__ inline uint32_t pack_bf16x2(float a, float b) {
    bf16_t x, y;
    io<bf16_t>::st(&x, a);
    io<bf16_t>::st(&y, b);
    return (uint32_t)x.x | ((uint32_t)y.x << 16);
}

template <bool P_KC, bool Q_KC>
__global__ __launch_bounds__(THREADS, 2) void gemm_kernel(Args a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[NSTAGE * STAGE];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nwg = gridDim.x;
    const int id = xcd_remap(blockIdx.x, nwg);
    const int per_b = a.tp * a.tq;
    const int b = id / per_b, t = id % per_b;
    const int tpi = a.q_fast ? t / a.tq : t % a.tp;
    const int tqi = a.q_fast ? t % a.tq : t / a.tp;
    const int p0 = tpi * BP, q0 = tqi * BQ;

    const uint16_t* pb = a.p + (int64_t)b * a.p_bs;
    const uint16_t* qb = a.q + (int64_t)b * a.q_bs;
    const auto rp = rsrc_from(pb, a.p_ext - (int64_t)b * a.p_bs);
    const auto rq = rsrc_from(qb, a.q_ext - (int64_t)b * a.q_bs);

    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int wp = (wave >> 1) * 64, wq = (wave & 1) * 64;
    const int nt = a.k / BK;
    stage_load<P_KC>(rp, lds, p0, 0, a.p_sx, a.mp, wave, lane);
    stage_load<Q_KC>(rq, lds + IMG, q0, 0, a.q_sx, a.mq, wave, lane);
    for (int kt = 0; kt < nt; ++kt) {
        const uint8_t* img = lds + (kt & 1) * STAGE;
        if (kt + 1 < nt) {
            uint8_t* nxt = lds + ((kt + 1) & 1) * STAGE;
            stage_load<P_KC>(rp, nxt, p0, (kt + 1) * BK, a.p_sx, a.mp, wave, lane);
            stage_load<Q_KC>(rq, nxt + IMG, q0, (kt + 1) * BK, a.q_sx, a.mq, wave, lane);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");          // this stage's 8 DMAs landed, the next 8 fly
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
#pragma unroll
        for (int s = 0; s < BK / 16; ++s) {
            bf16x8 fa[2], fb[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) fa[i] = frag<P_KC>(img, wp + 32 * i, s, lane);
#pragma unroll
            for (int j = 0; j < 2; ++j) fb[j] = frag<Q_KC>(img + IMG, wq + 32 * j, s, lane);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                                  // the buffer is re-filled next iteration
        asm volatile("" ::: "memory");
    }

    // epilogue: lane holds C rows p = p0 + wp + 32 i + 8 g + 4 (lane >> 5) + 0..3 at column q = q0 + wq + 32 j + (lane & 31)
    uint16_t* cb = reinterpret_cast<uint16_t*>(a.c) + (int64_t)b * a.c_bs;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int q = q0 + wq + 32 * j + (lane & 31);
        if (q >= a.mq) continue;
        uint16_t* crow = cb + (int64_t)q * a.c_sq;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int p = p0 + wp + 32 * i + 8 * g + 4 * (lane >> 5);
                const float v0 = a.alpha * acc[i][j][4 * g], v1 = a.alpha * acc[i][j][4 * g + 1];
                const float v2 = a.alpha * acc[i][j][4 * g + 2], v3 = a.alpha * acc[i][j][4 * g + 3];
                if (p + 3 < a.mp) {
                    uint2 w;
                    w.x = pack_bf16x2(v0, v1);
                    w.y = pack_bf16x2(v2, v3);
                    *reinterpret_cast<uint2*>(crow + p) = w;
                } else {
                    const float v[4] = {v0, v1, v2, v3};
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (p + e < a.mp) io<bf16_t>::st(reinterpret_cast<bf16_t*>(crow + p + e), v[e]);
                }
            }
    }
}

}  // namespace pg
}  // namespace avse

using namespace avse::pg;

extern "C" {

int avse_gemm_bf16(const avse_gemm_bf16_args* g, avse_stream_t stream) {
    if (!g || !g->p || !g->q || !g->c) return AVSE_EINVAL;
    if (g->c_dtype != AVSE_BF16) return AVSE_EDTYPE;
    if (g->batch <= 0 || g->mp <= 0 || g->mq <= 0 || g->k <= 0) return AVSE_ESHAPE;
    if (g->k % BK) return AVSE_ESHAPE;
    const bool p_kc = g->p_sk == 1, q_kc = g->q_sk == 1;
    if (!p_kc && g->p_sx != 1) return AVSE_ESHAPE;
    if (!q_kc && g->q_sx != 1) return AVSE_ESHAPE;
    const int64_t p_s = p_kc ? g->p_sx : g->p_sk, q_s = q_kc ? g->q_sx : g->q_sk;
    if (p_s % 8 || q_s % 8 || ((uintptr_t)g->p & 15) || ((uintptr_t)g->q & 15) || ((uintptr_t)g->c & 7) || g->c_sq % 4)
        return AVSE_EALIGN;
    const int64_t tp = (g->mp + BP - 1) / BP, tq = (g->mq + BQ - 1) / BQ;
    // 32-bit per-batch byte offsets: the farthest element a stage reads, and the output's
    const int64_t p_far = p_kc ? (tp * BP) * p_s + g->k : (g->k) * p_s + tp * BP;
    const int64_t q_far = q_kc ? (tq * BQ) * q_s + g->k : (g->k) * q_s + tq * BQ;
    if (p_far * 2 >= (1LL << 31) || q_far * 2 >= (1LL << 31)) return AVSE_ESHAPE;
    if (g->mp >= (1 << 30) || g->mq >= (1 << 30) || g->batch * tp * tq >= (1LL << 31)) return AVSE_ESHAPE;
    Args a;
    a.p = (const uint16_t*)g->p;
    a.q = (const uint16_t*)g->q;
    a.c = g->c;
    a.p_bs = g->p_bs;
    a.q_bs = g->q_bs;
    a.c_bs = g->c_bs;
    a.p_ext = g->p_extent;
    a.q_ext = g->q_extent;
    a.p_sx = (int32_t)p_s;
    a.q_sx = (int32_t)q_s;
    a.c_sq = (int32_t)g->c_sq;
    a.mp = (int32_t)g->mp;
    a.mq = (int32_t)g->mq;
    a.k = (int32_t)g->k;
    a.batch = (int32_t)g->batch;
    a.tp = (int32_t)tp;
    a.tq = (int32_t)tq;
    // the shared weight's tiles vary fastest; otherwise the operand with fewer tiles
    a.q_fast = (g->q_bs == 0) ? 1 : (g->p_bs == 0) ? 0 : (tq <= tp);
    a.alpha = g->alpha;
    const dim3 grid((unsigned)(g->batch * tp * tq)), block(THREADS);
    hipStream_t st = (hipStream_t)stream;
    if (p_kc && q_kc) hipLaunchKernelGGL((gemm_kernel<true, true>), grid, block, 0, st, a);
    else if (p_kc) hipLaunchKernelGGL((gemm_kernel<true, false>), grid, block, 0, st, a);
    else if (q_kc) hipLaunchKernelGGL((gemm_kernel<false, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((gemm_kernel<false, false>), grid, block, 0, st, a);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
