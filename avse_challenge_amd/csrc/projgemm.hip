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
// Shape of the work: K is short (512 .. 2048), so a 128 x 128 tile spends more time fetching its operands from L2
// than multiplying them (256 KB per 16.8 MFLOP = 75 GB/s per CU at half the MFMA peak, the L2's per-CU rate), and a
// non-persistent workgroup's epilogue leaves the MFMAs idle.  Hence:
//   - 256 x 256 tiles, 8 waves (2 per SIMD) of 128 (p) x 64 (q) each: 4 x 2 MFMA blocks, 128 accumulators per lane;
//     37 GB/s of L2 reads per CU at half the peak;
//   - persistent workgroups (one per CU) walking a flat sequence of (tile, k-stage) pairs; stages of 32 k staged
//     HBM/L2 -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds; reads past the operand's extent land as 0) into a ring of
//     4 buffers (128 KB), issued 3 stages ahead — across tile boundaries, so the next tile's first stages load while
//     this tile's epilogue stores;
//   - one barrier per stage: after it, every wave has finished the stage that last used the buffer being refilled.
// LDS images per operand and stage (16 KB):
//   K-contiguous: 256 rows x 64 B (32 k); 16-B chunk c of row r stored at c ^ ((r >> 2) & 3): the fragment reads
//     (ds_read_b128, lane = row) of each 16-lane group hit 16 distinct 16-B bank slots;
//   MN-contiguous: 32 k-rows x 512 B (256 p or q); chunk c of k-row r at c ^ ((r & 3) << 2); fragments by
//     ds_read_b64_tr_b16 (4 k-rows x 16 columns per 16-lane group, delivered column-major), conflict-free per half.
// The swizzle is applied to the DMA's per-lane SOURCE address (the LDS side of an LDS-DMA is lane-linear).
// Tile order: the shared weight's tile index runs fastest, and the 32 workgroups of an XCD take 32 consecutive tiles
// per round, so an activation block is fetched from HBM once and re-read from that XCD's L2.
#include <algorithm>

#include "common.h"

namespace avse {
namespace pg {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s4_t __attribute__((ext_vector_type(4)));
typedef short s8_t __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) s4_t lds_s4_t;

constexpr int BT = 256, THREADS = 512, WAVES = THREADS / 64;
constexpr int BK = 32;                     // k per stage
constexpr int IMG = BT * BK * 2;           // one operand's image of one stage
constexpr int STAGE = 2 * IMG;
constexpr int NBUF = 4, AHEAD = NBUF - 1;   // LDS ring; stages in flight ahead of the one computed
// Waves 0..LWAVES-1 issue every LDS-DMA, waves LWAVES.. every global store of the bf16 epilogue: a loader wave never
// has a store outstanding, so its counted vmcnt waits for a stage are exact (vmcnt also counts stores, and loads and
// stores may complete out of order), and a store wave never waits on vmcnt at all.
constexpr int LWAVES = 4;
constexpr int PIECES = IMG / 1024 / LWAVES; // LDS-DMA wave-instructions per operand, stage and loader wave
constexpr int LOADS = 2 * PIECES;          // per stage and loader wave
// K-contiguous image: rows of RB bytes (CPR 16-B chunks), RPL rows per 256-B bank line
constexpr int RB = 2 * BK, CPR = BK / 8, RPL = 256 / RB;
static_assert(NBUF * STAGE <= 160 * 1024, "LDS");
static_assert(AHEAD >= 2 && AHEAD <= 4, "ring depth: stage s + 1 is issued before iteration s");

__device__ inline int kc_swz(int row) { return (row / RPL) % CPR; }

struct Args {
    const uint16_t* p;
    const uint16_t* q;
    void* c;
    int64_t p_bs, q_bs, c_bs;              // batch strides (elements)
    int64_t p_ext, q_ext;                  // elements addressable from p / q (for the buffer range)
    int32_t p_sx, q_sx;                    // stride of the p / q index (K-contiguous operand) or of k (MN-contiguous)
    int32_t c_sq;
    int32_t mp, mq, k, batch;
    int32_t tp, tq;                        // tile counts per batch group
    int32_t ntiles, ntb;                   // tiles in all; k-stages per batch
    int32_t fold;                          // batches summed into one output (weight gradients), batch % fold == 0
    int32_t kv_last;                       // valid k in a batch's last stage (BK unless k % BK)
    int32_t q_fast;                        // q tile index runs fastest in the tile order
    int32_t c_vec16;                       // bf16 out: rows 16-B aligned (c and c_sq * 2 multiples of 16)
    float alpha;
    // split mode (fp32 GEMM on fp16 hi / lo planes): the lo planes (same strides as p / q) and the device max-|x| bits
    // the planes were scaled by (dconv.hip split_exp)
    const uint16_t* p_lo;
    const uint16_t* q_lo;
    const uint32_t* p_max;
    const uint32_t* q_max;
    // nsub > 1: batch b sits at (b / nsub) bs + (b % nsub) bs2 (a reduction split into nsub chunks of k per batch, e.g.
    // the time chunks of a 1x1-conv weight gradient, folded and summed as batches); otherwise at b bs
    int32_t nsub;
    int64_t p_bs2, q_bs2;
};

__device__ inline int64_t batch_off(int b, int nsub, int64_t bs, int64_t bs2) {
    return nsub > 1 ? (int64_t)(b / nsub) * bs + (int64_t)(b % nsub) * bs2 : (int64_t)b * bs;
}

// power-of-two split scale of a tensor with max |x| bits mb (the same function as dconv.hip's / gemmsplit's)
__device__ inline int split_exp_pg(uint32_t mb) {
    const int ef = (int)((mb >> 23) & 0xff);
    if (mb == 0) return 0;
    const int k = ef == 0 ? -127 : ef - 127;
    return min(100, max(-100, 14 - k));
}

typedef int i4_t __attribute__((ext_vector_type(4)));

// Buffer resource (wave-uniform) over [base, base + elems): reads past it return 0.
__device__ inline i4_t rsrc_from(const uint16_t* base, int64_t elems) {
    int64_t bytes = elems * 2;
    if (bytes > 0x7FFFFFF0LL) bytes = 0x7FFFFFF0LL;
    if (bytes < 0) bytes = 0;
    const uint64_t a = (uint64_t)base;
    return i4_t{__builtin_amdgcn_readfirstlane((int)(uint32_t)a), __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff)),
                __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000};
}

// One 16-B-per-lane LDS-DMA wave-instruction: LDS[lds_addr + 16 lane] = buffer[voff].  Inline asm on purpose: the
// compiler tracks its own LDS-DMA builtins as pending writes to the whole staging array and then waits vmcnt(0)
// before every ds_read of it, which drains the stages in flight; the ring's counted waits are done by hand instead.
// Nothing else in these kernels uses M0.
__device__ inline void dma16(i4_t r, uint32_t lds_addr, uint32_t voff) {
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(r), "s"(lds_addr)
                 : "memory");
}

__device__ inline uint32_t lds_u32(const void* p) {
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const lds_void_t*)p);
}

struct Tile {
    int b, p0, q0;
};

// b: the batch group (the output batch); its batches are b * fold .. b * fold + fold - 1
__device__ inline Tile tile_of(const Args& a, int T) {
    const int per_b = a.tp * a.tq;
    const int b = T / per_b, t = T - b * per_b;
    const int tpi = a.q_fast ? t / a.tq : t % a.tp;
    const int tqi = a.q_fast ? t % a.tq : t / a.tp;
    return Tile{b, tpi * BT, tqi * BT};
}

// One operand's stage (BK k x 256 rows) -> LDS image.  KC: the operand is K-contiguous (row x0 + r has stride sx, k
// is contiguous); otherwise k-row k0 + r has stride sx and the 256 rows are contiguous.  Rows past mx are clamped
// (KC) or read whatever lies there / 0 past the buffer (MN); they only feed outputs that are never stored.
// piece_offsets: this lane's byte offsets of its PIECES wave-instructions for k0 = 0; stage kt adds kt * stage_step.
template <bool KC>
__device__ inline void piece_offsets(uint32_t (&vo)[PIECES], int x0, int sx, int mx, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < PIECES; ++j) {
        const int piece = wave * PIECES + j;                  // 1 KB of the image per wave-instruction
        if constexpr (KC) {
            const int row = piece * (1024 / RB) + lane / CPR;
            const int xr = min(x0 + row, mx - 1);
            const int c = (lane % CPR) ^ kc_swz(row);
            vo[j] = (uint32_t)(xr * sx + c * 8) * 2u;
        } else {
            const int krow = piece * 2 + (lane >> 5);
            const int c = (lane & 31) ^ ((krow & 3) << 2);
            vo[j] = (uint32_t)(krow * sx + x0 + c * 8) * 2u;
        }
    }
}
template <bool KC>
__device__ inline uint32_t stage_step(int sx) { return KC ? (uint32_t)(BK * 2) : (uint32_t)(BK * sx * 2); }

template <bool KC>
__device__ inline void stage_load(i4_t r, uint32_t img, const uint32_t (&vo)[PIECES], uint32_t koff, int wave) {
#pragma unroll
    for (int j = 0; j < PIECES; ++j) dma16(r, img + (wave * PIECES + j) * 1024, vo[j] + koff);
}

// The 32 x 16 (row x k) MFMA operand fragment of rows rb .. rb + 31, k-substep s (k = 16 s .. 16 s + 15):
// lane l holds row rb + (l & 31), k = 16 s + 8 (l >> 5) + 0..7 (element e <-> k = 16 s + 8 (l >> 5) + e).
template <bool KC>
__device__ inline bf16x8 frag_raw(const uint8_t* img, int rb, int s, int lane) {
    if constexpr (KC) {
        const int row = rb + (lane & 31);
        const int ch = 2 * s + (lane >> 5);
        return *reinterpret_cast<const bf16x8*>(img + row * RB + 16 * (ch ^ kc_swz(row)));
    } else {
        const int g = lane >> 4, i = lane & 15;
        const int col = rb + 16 * (g & 1) + 4 * (i & 3);
        const int kb = 16 * s + 8 * (g >> 1) + (i >> 2);
        s4_t v[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int kr = kb + 4 * u;
            const int off = kr * 512 + 16 * ((col >> 3) ^ ((kr & 3) << 2)) + (col & 7) * 2;
            v[u] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(img + off));
        }
        const s8_t w = {v[0][0], v[0][1], v[0][2], v[0][3], v[1][0], v[1][1], v[1][2], v[1][3]};
        return __builtin_bit_cast(bf16x8, w);
    }
}

// Zero the k >= kv part of one operand's stage image (the reduction's last, partial stage: what lies past k is
// another row's data, pad columns or 0, and a non-finite value there must not reach the sums as 0 * inf), so both
// operands are cleared.  KC image: 16-B chunk c of row r (k = 8 c .. 8 c + 7) at c ^ kc_swz(r); MN image: whole
// k-rows.
template <bool KC>
__device__ inline void zero_tail(uint8_t* img, int kv, int tid) {
    if constexpr (KC) {
        for (int i = tid; i < BT * CPR; i += THREADS) {
            const int row = i / CPR, pos = i % CPR, c = pos ^ kc_swz(row);
            if (8 * c + 8 <= kv) continue;
            s8_t* ptr = reinterpret_cast<s8_t*>(img + row * RB + 16 * pos);
            s8_t w = *ptr;
#pragma unroll
            for (int e = 0; e < 8; ++e) w[e] = (8 * c + e < kv) ? w[e] : (short)0;
            *ptr = w;
        }
    } else {
        for (int i = tid; i < BK * 32; i += THREADS) {          // 32 16-B chunks per 512-B k-row
            const int kr = i >> 5;
            if (kr >= kv) *reinterpret_cast<uint4*>(img + kr * 512 + 16 * (i & 31)) = uint4{0u, 0u, 0u, 0u};
        }
    }
}

__device__ inline uint32_t pack_bf16x2(float a, float b) {
    bf16_t x, y;
    io<bf16_t>::st(&x, a);
    io<bf16_t>::st(&y, b);
    return (uint32_t)x.x | ((uint32_t)y.x << 16);
}

// Wave (wr, wc) = (wave >> 2, wave & 3) owns the p blocks 32 (2 i + wr), i = 0..3 (so an epilogue round i covers the
// 64 contiguous p of 64 i .. 64 i + 63 over both wave rows) and the q columns 64 wc .. 64 wc + 63 (blocks j = 0, 1).
struct Frags {
    bf16x8 a[4], b[2];
};
template <bool P_KC, bool Q_KC>
__device__ inline void read_frags(Frags& f, const uint8_t* img, int ks, int wr, int wq, int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i) f.a[i] = frag_raw<P_KC>(img, 32 * (2 * i + wr), ks, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j) f.b[j] = frag_raw<Q_KC>(img + IMG, wq + 32 * j, ks, lane);
}
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
template <bool F16>
__device__ inline void mma(floatx16 (&acc)[4][2], const Frags& f) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if constexpr (F16)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, f.a[i]),
                                                                   __builtin_bit_cast(half8, f.b[j]), acc[i][j], 0, 0, 0);
            else
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[i], f.b[j], acc[i][j], 0, 0, 0);
        }
}

// Pipeline (one barrier per stage).  Stage s is certified readable by the barrier of iteration s - 1 (its DMAs'
// counted vmcnt wait precedes that barrier), so its first k-substep's fragments are read at the end of iteration s - 1,
// across the barrier, and iteration s starts on MFMAs.  Iteration s: wait for stage s + 1's DMAs -> barrier (also: every
// wave has finished reading stage s - 1) -> DMA stage s + AHEAD into stage s - 1's buffer -> MFMAs of stage s with the
// next substep's / stage's fragment reads interleaved.  Before the barrier each wave's reads of the stage leaving the
// ring have completed: an lgkmcnt(0) sits between the last read of stage s and the first prefetch read of stage s + 1.
// EPI: 0 = bf16 out, LDS-staged 128-B lines; 1 = fp32 out straight from the accumulators (weight gradients: small
// outputs); 2 = fp32 out, LDS-staged 128-B lines (large outputs).  SPLIT: the fp32 GEMM on fp16 hi / lo planes of both
// operands (gemmsplit.hip): the k-stage sequence of a tile runs three segments, P_hi Q_hi, P_hi Q_lo, P_lo Q_hi, on the
// f16 MFMA, and the epilogue scales by 2^-(e_p + e_q).
template <bool P_KC, bool Q_KC, int EPI, bool SPLIT = false>
__global__ __launch_bounds__(THREADS, 1) void gemm_kernel(Args a) {
    constexpr bool OUT_F32 = EPI != 0;
    constexpr int NSEG = SPLIT ? 3 : 1;
    __shared__ __attribute__((aligned(16))) uint8_t lds[NBUF * STAGE];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // tiles of this workgroup: round r takes tile r * G + xcd * (G / 8) + slot (G % 8 == 0), so the workgroups of
    // one XCD (blockIdx % 8) work on consecutive tiles
    const int G = gridDim.x;
    const int base = (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8;
    const int my_tiles = base < a.ntiles ? (a.ntiles - base + G - 1) / G : 0;
    const int per_tile = NSEG * a.ntb * a.fold;
    const int total = my_tiles * per_tile;
    if (total == 0) return;                                    // workgroup-uniform: no barrier is skipped by part
    const int wr = wave >> 2, wc = wave & 3, wq = wc * 64;
    const uint32_t lds0 = lds_u32(lds);
    const uint32_t p_step = stage_step<P_KC>(a.p_sx), q_step = stage_step<Q_KC>(a.q_sx);

    // load cursor: the stage issued next = (tile ld_T, batch ld_f of its group, k-stage ld_kt)
    int ld_s = 0, ld_kt = 0, ld_f = 0, ld_T = base;
    uint32_t vp[PIECES], vq[PIECES];
    i4_t rp, rq, rp_lo, rq_lo;
    auto set_tile = [&](int T, int f) {
        const Tile t = tile_of(a, T);
        const int b = t.b * a.fold + f;
        const int64_t po = batch_off(b, a.nsub, a.p_bs, a.p_bs2), qo = batch_off(b, a.nsub, a.q_bs, a.q_bs2);
        rp = rsrc_from(a.p + po, a.p_ext - po);
        rq = rsrc_from(a.q + qo, a.q_ext - qo);
        if constexpr (SPLIT) {
            rp_lo = rsrc_from(a.p_lo + po, a.p_ext - po);
            rq_lo = rsrc_from(a.q_lo + qo, a.q_ext - qo);
        }
        piece_offsets<P_KC>(vp, t.p0, a.p_sx, a.mp, wave, lane);
        piece_offsets<Q_KC>(vq, t.q0, a.q_sx, a.mq, wave, lane);
    };
    set_tile(base, 0);
    const bool loader = wave < LWAVES;                          // wave-uniform
    auto issue = [&]() {
        if (ld_s >= total) return;
        if (loader) {
            const uint32_t img = lds0 + (ld_s % NBUF) * STAGE;
            if constexpr (SPLIT) {
                const int seg = ld_kt / a.ntb, kin = ld_kt - seg * a.ntb;     // segments: hi hi, hi lo, lo hi
                stage_load<P_KC>(seg == 2 ? rp_lo : rp, img, vp, kin * p_step, wave);
                stage_load<Q_KC>(seg == 1 ? rq_lo : rq, img + IMG, vq, kin * q_step, wave);
            } else {
                stage_load<P_KC>(rp, img, vp, ld_kt * p_step, wave);
                stage_load<Q_KC>(rq, img + IMG, vq, ld_kt * q_step, wave);
            }
        }
        ++ld_s;
        if (++ld_kt == NSEG * a.ntb) {
            ld_kt = 0;
            if (++ld_f == a.fold) {
                ld_f = 0;
                ld_T += G;
            }
            if (ld_s < total) set_tile(ld_T, ld_f);
        }
    };
    // stage s's position in its tile: partial (masked) stage?  (k-stage index = s % ntb)
    auto masked = [&](int st) { return a.kv_last < BK && (st % a.ntb) == a.ntb - 1; };
    auto wait_landed = [&](int st) {   // stage st's DMAs done: only the stages issued after it may still fly
        if (!loader) return;
        const int after = ld_s - st - 1;
        if (AHEAD >= 4 && after >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * LOADS) : "memory");
        else if (AHEAD >= 3 && after >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LOADS) : "memory");
        else if (AHEAD >= 2 && after >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LOADS) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    auto barrier = [&]() {
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    auto zero_stage = [&](int st) {    // after the barrier that certified stage st; ends with a barrier
        uint8_t* img = lds + (st % NBUF) * STAGE;
        zero_tail<P_KC>(img, a.kv_last, threadIdx.x);
        zero_tail<Q_KC>(img + IMG, a.kv_last, threadIdx.x);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        barrier();
    };

#pragma unroll
    for (int i = 0; i < AHEAD; ++i) issue();
    wait_landed(0);
    barrier();
    if (masked(0)) zero_stage(0);

    floatx16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    float alpha_eff = a.alpha;
    if constexpr (SPLIT) alpha_eff = __builtin_ldexpf(a.alpha, -(split_exp_pg(*a.p_max) + split_exp_pg(*a.q_max)));

    Frags f0, f1;
    read_frags<P_KC, Q_KC>(f0, lds, 0, wr, wq, lane);

    int kt = 0, f = 0, T = base;
    for (int s = 0; s < total; ++s) {
        const bool more = s + 1 < total;
        if (more) wait_landed(s + 1);
        barrier();                                              // stage s + 1 readable; stage s - 1 released
        issue();                                                // stage s + AHEAD into stage s - 1's buffer
        if (more && masked(s + 1)) zero_stage(s + 1);
        const uint8_t* img = lds + (s % NBUF) * STAGE;
#pragma unroll
        for (int ks = 1; ks < BK / 16; ++ks) {
            Frags& cur = (ks & 1) ? f0 : f1;
            Frags& nxt = (ks & 1) ? f1 : f0;
            read_frags<P_KC, Q_KC>(nxt, img, ks, wr, wq, lane);
            mma<SPLIT>(acc, cur);
            // keep these MFMAs ahead of the wait below: the compiler would otherwise sink them past it (they touch
            // no memory) and the wave would stall on the reads with the MFMA pipe idle
            __builtin_amdgcn_sched_barrier(0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");       // stage s's reads done before its buffer leaves
        Frags& last = ((BK / 16) & 1) ? f0 : f1;                // the final substep's fragments
        Frags& pre = ((BK / 16) & 1) ? f1 : f0;                 // BK / 16 even: f0 again holds substep 0
        if (more) read_frags<P_KC, Q_KC>(pre, lds + ((s + 1) % NBUF) * STAGE, 0, wr, wq, lane);
        mma<SPLIT>(acc, last);
        if (++kt < NSEG * a.ntb) continue;
        kt = 0;
        if (++f < a.fold) continue;
        f = 0;
        // epilogue of tile T.  acc[i][j]: rows p = p0 + 32 (2 i + wr) + 8 g + 4 (lane >> 5) + 0..3 (register 4 g + 0..3),
        // column q = q0 + wq + 32 j + (lane & 31)
        const Tile t = tile_of(a, T);
        T += G;
        if constexpr (EPI == 2) {
            // fp32 out through stage s's buffer in 8 rounds of 32 p x 256 q (32 KB): the waves of wave row wr stage the
            // accumulator block i, the store waves write each q row's 32 p as one 128-B line, non-temporal
            uint8_t* stg = lds + (s % NBUF) * STAGE;               // [256 q][128 B], 16-B chunk c of row q at c ^ (q & 7)
            float* cf = reinterpret_cast<float*>(a.c) + (int64_t)t.b * a.c_bs;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    barrier();                                  // the stage's / previous round's readers are done
                    if (wr == h) {
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            const int q = wq + 32 * j + (lane & 31);
#pragma unroll
                            for (int g = 0; g < 4; ++g) {
                                const int pl = 8 * g + 4 * (lane >> 5);        // p within the round's 32
                                const float4 v = {alpha_eff * acc[i][j][4 * g], alpha_eff * acc[i][j][4 * g + 1],
                                                  alpha_eff * acc[i][j][4 * g + 2], alpha_eff * acc[i][j][4 * g + 3]};
                                *reinterpret_cast<float4*>(stg + q * 128 + 16 * ((pl >> 2) ^ (q & 7))) = v;
                            }
                        }
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    barrier();
                    if (!loader) {
#pragma unroll
                        for (int r = 0; r < 256 / 8 / (WAVES - LWAVES); ++r) {   // 8 rows per wave-instruction
                            const int ql = (r * (WAVES - LWAVES) + (wave - LWAVES)) * 8 + (lane >> 3), c = lane & 7;
                            const float4 v = *reinterpret_cast<const float4*>(stg + ql * 128 + 16 * (c ^ (ql & 7)));
                            const int q = t.q0 + ql, p = t.p0 + 32 * (2 * i + h) + 4 * c;
                            if (q < a.mq) {
                                float* dst = cf + (int64_t)q * a.c_sq + p;
                                if (p + 3 < a.mp && a.c_vec16) {
                                    typedef float f4v_t __attribute__((ext_vector_type(4)));
                                    __builtin_nontemporal_store(f4v_t{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v_t*>(dst));
                                } else {
                                    const float w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                                    for (int e = 0; e < 4; ++e)
                                        if (p + e < a.mp) dst[e] = w[e];
                                }
                            }
                        }
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    }
                }
        } else if constexpr (OUT_F32) {
            // the weight gradients: small outputs, written straight from the accumulators (16 B per lane)
            float* cf = reinterpret_cast<float*>(a.c) + (int64_t)t.b * a.c_bs;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int q = t.q0 + wq + 32 * j + (lane & 31);
                float* crow = cf + (int64_t)min(q, a.mq - 1) * a.c_sq;
                const bool qok = q < a.mq;
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int p = t.p0 + 32 * (2 * i + wr) + 8 * g + 4 * (lane >> 5);
                        const float4 v = {alpha_eff * acc[i][j][4 * g], alpha_eff * acc[i][j][4 * g + 1],
                                          alpha_eff * acc[i][j][4 * g + 2], alpha_eff * acc[i][j][4 * g + 3]};
                        if (qok && p + 3 < a.mp) {
                            *reinterpret_cast<float4*>(crow + p) = v;
                        } else if (qok) {
                            const float w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                            for (int e = 0; e < 4; ++e)
                                if (p + e < a.mp) crow[p + e] = w[e];
                        }
                    }
            }
        } else {
            // bf16 out through stage s's buffer (free until iteration s + 1's barrier) in 4 rounds of 64 p x 256 q: all
            // waves stage their accumulators, the store waves write each q row's 64 p as one 128-B line (8 lanes x
            // 16 B), non-temporal (the output is not re-read here; it must not evict the operand tiles the next
            // workgroups re-read from L2).  The loader waves go on as soon as the last round is staged.
            uint8_t* stg = lds + (s % NBUF) * STAGE;              // [256 q][128 B], 16-B chunk c of row q at c ^ (q & 7)
            uint16_t* cb = reinterpret_cast<uint16_t*>(a.c) + (int64_t)t.b * a.c_bs;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                barrier();                                      // the stage's / previous round's readers are done
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int q = wq + 32 * j + (lane & 31);
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int pl = 32 * wr + 8 * g + 4 * (lane >> 5);       // p within the round's 64
                        uint2 w;
                        w.x = pack_bf16x2(alpha_eff * acc[i][j][4 * g], alpha_eff * acc[i][j][4 * g + 1]);
                        w.y = pack_bf16x2(alpha_eff * acc[i][j][4 * g + 2], alpha_eff * acc[i][j][4 * g + 3]);
                        *reinterpret_cast<uint2*>(stg + q * 128 + 16 * ((pl >> 3) ^ (q & 7)) + (pl & 7) * 2) = w;
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                barrier();
                if (!loader) {
#pragma unroll
                    for (int r = 0; r < 256 / 8 / (WAVES - LWAVES); ++r) {   // 8 rows per wave-instruction
                        const int ql = (r * (WAVES - LWAVES) + (wave - LWAVES)) * 8 + (lane >> 3), c = lane & 7;
                        const uint4 v = *reinterpret_cast<const uint4*>(stg + ql * 128 + 16 * (c ^ (ql & 7)));
                        const int q = t.q0 + ql, p = t.p0 + 64 * i + 8 * c;
                        if (q < a.mq) {
                            uint16_t* dst = cb + (int64_t)q * a.c_sq + p;
                            if (p + 7 < a.mp && a.c_vec16) {
                                typedef unsigned int u4v_t __attribute__((ext_vector_type(4)));
                                __builtin_nontemporal_store(u4v_t{v.x, v.y, v.z, v.w}, reinterpret_cast<u4v_t*>(dst));
                            } else if (p + 7 < a.mp) {
                                reinterpret_cast<uint2*>(dst)[0] = uint2{v.x, v.y};
                                reinterpret_cast<uint2*>(dst)[1] = uint2{v.z, v.w};
                            } else {
                                const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                                for (int e = 0; e < 8; ++e)
                                    if (p + e < a.mp) dst[e] = (uint16_t)(u[e >> 1] >> (16 * (e & 1)));
                            }
                        }
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    }
}

}  // namespace pg
}  // namespace avse

using namespace avse::pg;

// ------------------------------------------------------------------------------------------------ split planes
// x (b, r, c) fp32, c contiguous -> hi / lo fp16 planes (rows hrs, batches hbs apart: x's strides, or a padded layout
// whose rows are 16-B aligned for the GEMM's DMA): hi = fp16(x 2^e), lo = fp16(x 2^e - hi) with max |x| 2^e in
// [2^14, 2^15) (dconv.hip's split, the same 22 significant bits); the planes' padding is not written.
// Two streaming passes (max, then split): a workgroup takes rpb consecutive rows, float4 accesses when the rows are
// 16-B aligned (VEC), the row's last c % 4 elements one by one; 4 accesses in flight per thread either way.
struct PlanesArgs {
    const float* x;
    int64_t rows, r, c, bs, rs, hbs, hrs;
    int rpb;
    uint32_t* maxbits;
    _Float16* hi;
    _Float16* lo;
};

__device__ inline int64_t planes_row_off(const PlanesArgs& a, int64_t row) { return (row / a.r) * a.bs + (row % a.r) * a.rs; }
__device__ inline int64_t planes_out_off(const PlanesArgs& a, int64_t row) {
    return (row / a.r) * a.hbs + (row % a.r) * a.hrs;
}

// grid-stride over the row blocks with a bounded grid of 1024-thread workgroups and one atomicMax per workgroup: the
// max word is shared by every XCD, so its atomics serialise far from the CUs (~17 ns each: one per wave over 10^5 row
// blocks cost 6.8 ms for a C3 activation, profiles/r05i_gemm_f32s_probe.jsonl; 2048 per call cost ~30 us of a 65 MB
// pass), while 16 waves per CU keep enough loads in flight
constexpr int AM_NT = 1024, AM_GRID = 256;
template <bool VEC>
__global__ __launch_bounds__(AM_NT) void planes_absmax_kernel(PlanesArgs a, int64_t nrb) {
    __shared__ uint32_t red[AM_NT / 64];
    float m = 0.f;
    const int64_t c4 = VEC ? a.c / 4 : 0;
    for (int64_t rb = blockIdx.x; rb < nrb; rb += gridDim.x)
    for (int rr = 0; rr < a.rpb; ++rr) {
        const int64_t row = rb * a.rpb + rr;
        if (row >= a.rows) break;
        const float* xr = a.x + planes_row_off(a, row);
        if constexpr (VEC) {
            for (int64_t j0 = threadIdx.x; j0 < c4; j0 += 4 * AM_NT) {
                float4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    v[u] = j0 + u * AM_NT < c4 ? reinterpret_cast<const float4*>(xr)[j0 + u * AM_NT] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
            }
        }
        for (int64_t i0 = 4 * c4 + threadIdx.x; i0 < a.c; i0 += 4 * AM_NT) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = i0 + u * AM_NT < a.c ? xr[i0 + u * AM_NT] : 0.f;
#pragma unroll
            for (int u = 0; u < 4; ++u) m = fmaxf(m, fabsf(v[u]));
        }
    }
    uint32_t v = __float_as_uint(m);
    for (int o = 32; o >= 1; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < AM_NT / 64; ++k) v = max(v, red[k]);
        v = max(v, red[0]);
        if (v) atomicMax(a.maxbits, v);
    }
}

__device__ inline uint32_t split_pair(float x0, float x1, float sc, uint32_t& lo) {
    const float s0 = x0 * sc, s1 = x1 * sc;
    const _Float16 h0 = (_Float16)s0, h1 = (_Float16)s1;
    const _Float16 l0 = (_Float16)(s0 - (float)h0), l1 = (_Float16)(s1 - (float)h1);
    lo = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
    return (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
}

template <bool VEC>
__global__ __launch_bounds__(256) void planes_split_kernel(PlanesArgs a) {
    const float sc = __builtin_ldexpf(1.f, split_exp_pg(*a.maxbits));
    const int64_t c4 = VEC ? a.c / 4 : 0;
    for (int rr = 0; rr < a.rpb; ++rr) {
        const int64_t row = (int64_t)blockIdx.x * a.rpb + rr;
        if (row >= a.rows) break;
        const int64_t off = planes_out_off(a, row);
        const float* xr = a.x + planes_row_off(a, row);
        if constexpr (VEC) {
            uint2* hr = reinterpret_cast<uint2*>(a.hi + off);
            uint2* lr = reinterpret_cast<uint2*>(a.lo + off);
            for (int64_t j0 = threadIdx.x; j0 < c4; j0 += 4 * 256) {
                float4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (j0 + u * 256 < c4) v[u] = reinterpret_cast<const float4*>(xr)[j0 + u * 256];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (j0 + u * 256 >= c4) break;
                    uint2 h, l;
                    h.x = split_pair(v[u].x, v[u].y, sc, l.x);
                    h.y = split_pair(v[u].z, v[u].w, sc, l.y);
                    hr[j0 + u * 256] = h;
                    lr[j0 + u * 256] = l;
                }
            }
        }
        for (int64_t i0 = 4 * c4 + threadIdx.x; i0 < a.c; i0 += 4 * 256) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i0 + u * 256 < a.c) v[u] = xr[i0 + u * 256];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t i = i0 + u * 256;
                if (i >= a.c) break;
                const float w = v[u] * sc;
                const _Float16 h = (_Float16)w;
                a.hi[off + i] = h;
                a.lo[off + i] = (_Float16)(w - (float)h);
            }
        }
    }
}

// x rows of any alignment -> planes with 8-B aligned rows of hrs elements (the padded-row layout, hrs >= c): each thread
// writes 4 consecutive elements of a row as one 8-B store per plane, loading them element by element (lanes read
// consecutive addresses), 4 quadruples in flight; the pad columns c .. hrs - 1 are written as 0, so a GEMM may sum
// over them (the time chunks of a weight gradient).
__global__ __launch_bounds__(256) void planes_split_pad_kernel(PlanesArgs a) {
    const float sc = __builtin_ldexpf(1.f, split_exp_pg(*a.maxbits));
    const int64_t q4 = a.hrs / 4;                                  // quadruples per output row
    for (int rr = 0; rr < a.rpb; ++rr) {
        const int64_t row = (int64_t)blockIdx.x * a.rpb + rr;
        if (row >= a.rows) break;
        const float* xr = a.x + planes_row_off(a, row);
        uint2* hr = reinterpret_cast<uint2*>(a.hi + planes_out_off(a, row));
        uint2* lr = reinterpret_cast<uint2*>(a.lo + planes_out_off(a, row));
        for (int64_t j0 = threadIdx.x; j0 < q4; j0 += 4 * 256) {
            float v[4][4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int64_t i = 4 * (j0 + u * 256) + e;
                    v[u][e] = (j0 + u * 256 < q4 && i < a.c) ? xr[i] : 0.f;
                }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (j0 + u * 256 >= q4) break;
                uint2 h, l;
                h.x = split_pair(v[u][0], v[u][1], sc, l.x);
                h.y = split_pair(v[u][2], v[u][3], sc, l.y);
                hr[j0 + u * 256] = h;
                lr[j0 + u * 256] = l;
            }
        }
    }
}

// y = a + b over the padded (rows, lp) storage of two (b, c, l) operands (one vectorised pass; the pad columns hold
// don't-care values) and max |y| over the logical columns c < l: the C3 out_proj input with its producer-side max
// (the BiMamba direction sum, bimamba.py:253), so the projection's split skips its absmax pass
// MASK (padded rows): row-major walk, rows grid-strided over the workgroups and each row's float4 columns over the
// threads (4 in flight per thread), so the logical-column test needs no division (round 5's flat index took a modulo
// per float4: 0.98 ms per C3 call, 3.2 TB/s, r06j profile)
template <bool MASK>
__global__ __launch_bounds__(256) void add_max_kernel(int n4, int lp4, int l, const float4* __restrict__ a,
                                                      const float4* __restrict__ b, float4* __restrict__ y,
                                                      uint32_t* __restrict__ maxbits) {
    __shared__ uint32_t red[4];
    float m = 0.f;
    if constexpr (MASK) {
        const int rows = n4 / lp4, lfull = l / 4;                 // float4 columns wholly inside the logical row
        for (int row = blockIdx.x; row < rows; row += gridDim.x) {
            const int64_t base = (int64_t)row * lp4;
            for (int c0 = threadIdx.x; c0 < lp4; c0 += 4 * 256) {
                float4 u[4], v[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int c = c0 + k * 256;
                    if (c < lp4) {
                        u[k] = a[base + c];
                        v[k] = b[base + c];
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int c = c0 + k * 256;
                    if (c >= lp4) break;
                    const float4 s = make_float4(u[k].x + v[k].x, u[k].y + v[k].y, u[k].z + v[k].z, u[k].w + v[k].w);
                    y[base + c] = s;
                    if (c < lfull) {
                        m = fmaxf(m, fmaxf(fmaxf(fabsf(s.x), fabsf(s.y)), fmaxf(fabsf(s.z), fabsf(s.w))));
                    } else {
                        const int e = 4 * c;
                        m = fmaxf(m, e < l ? fabsf(s.x) : 0.f);
                        m = fmaxf(m, e + 1 < l ? fabsf(s.y) : 0.f);
                        m = fmaxf(m, e + 2 < l ? fabsf(s.z) : 0.f);
                        m = fmaxf(m, e + 3 < l ? fabsf(s.w) : 0.f);
                    }
                }
            }
        }
    } else {
        const int stride = gridDim.x * 256;
        for (int i0 = blockIdx.x * 256 + threadIdx.x; i0 < n4; i0 += 4 * stride) {    // 4 float4 pairs in flight
            float4 u[4], v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int i = i0 + k * stride;
                if (i < n4) {
                    u[k] = a[i];
                    v[k] = b[i];
                }
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int i = i0 + k * stride;
                if (i >= n4) break;
                const float4 s = make_float4(u[k].x + v[k].x, u[k].y + v[k].y, u[k].z + v[k].z, u[k].w + v[k].w);
                y[i] = s;
                m = fmaxf(m, fmaxf(fmaxf(fabsf(s.x), fabsf(s.y)), fmaxf(fabsf(s.z), fabsf(s.w))));
            }
        }
    }
    uint32_t v = __float_as_uint(m);
    for (int o = 32; o >= 1; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        v = max(max(red[0], red[1]), max(red[2], red[3]));
        if (v) atomicMax(maxbits, v);
    }
}

static int cu_count_cached() {
    static int cu_count[64];
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
        if (cu_count[dev] <= 0 &&
            hipDeviceGetAttribute(&cu_count[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cu_count[dev] = 256;
        cus = cu_count[dev];
    }
    return cus;
}

// shared host path of avse_gemm_bf16 / avse_gemm_f32s: operand checks, Args, persistent grid, instantiation
template <bool SPLIT>
static int launch_gemm(int64_t batch, int64_t mp, int64_t mq, int64_t k, int64_t fold_in, const void* p, const void* p_lo,
                       int64_t p_bs, int64_t p_sx, int64_t p_sk, int64_t p_extent, const uint32_t* p_max, const void* q,
                       const void* q_lo, int64_t q_bs, int64_t q_sx, int64_t q_sk, int64_t q_extent,
                       const uint32_t* q_max, void* c, int64_t c_bs, int64_t c_sq, float alpha, int32_t c_dtype,
                       avse_stream_t stream, int64_t nsub = 1, int64_t p_bs2 = 0, int64_t q_bs2 = 0) {
    if (!p || !q || !c || (SPLIT && (!p_lo || !q_lo || !p_max || !q_max))) return AVSE_EINVAL;
    if (c_dtype != AVSE_BF16 && c_dtype != AVSE_F32) return AVSE_EDTYPE;
    if (SPLIT && c_dtype != AVSE_F32) return AVSE_EDTYPE;
    const int64_t fold = fold_in > 0 ? fold_in : 1;
    if (batch <= 0 || mp <= 0 || mq <= 0 || k <= 0 || batch % fold || nsub >= (1 << 30)) return AVSE_ESHAPE;
    const bool p_kc = p_sk == 1, q_kc = q_sk == 1;
    if (!p_kc && p_sx != 1) return AVSE_ESHAPE;
    if (!q_kc && q_sx != 1) return AVSE_ESHAPE;
    const int64_t p_s = p_kc ? p_sx : p_sk, q_s = q_kc ? q_sx : q_sk;
    const int c_align = c_dtype == AVSE_F32 ? 15 : 7;
    // fp32 out, no folding (the LDS-staged epilogue 2): any row stride (rows not 16-B aligned are stored per element)
    const bool c_any = SPLIT && fold == 1;
    if (p_s % 8 || q_s % 8 || ((uintptr_t)p & 15) || ((uintptr_t)q & 15) || ((uintptr_t)c & c_align) ||
        (!c_any && c_sq % 4) ||
        (SPLIT && (((uintptr_t)p_lo & 15) || ((uintptr_t)q_lo & 15))))
        return AVSE_EALIGN;
    const int64_t tp = (mp + BT - 1) / BT, tq = (mq + BT - 1) / BT, ntb = (k + BK - 1) / BK;
    // 32-bit per-batch byte offsets: the farthest element a stage reads
    const int64_t p_far = p_kc ? (tp * BT) * p_s + ntb * BK : ntb * BK * p_s + tp * BT;
    const int64_t q_far = q_kc ? (tq * BT) * q_s + ntb * BK : ntb * BK * q_s + tq * BT;
    if (p_far * 2 >= (1LL << 31) || q_far * 2 >= (1LL << 31)) return AVSE_ESHAPE;
    const int64_t ntiles = batch / fold * tp * tq;
    if (mp >= (1 << 30) || mq >= (1 << 30) || ntiles * ntb * fold * (SPLIT ? 3 : 1) >= (1LL << 31)) return AVSE_ESHAPE;
    Args a;
    a.p = (const uint16_t*)p;
    a.q = (const uint16_t*)q;
    a.p_lo = (const uint16_t*)p_lo;
    a.q_lo = (const uint16_t*)q_lo;
    a.p_max = p_max;
    a.q_max = q_max;
    a.c = c;
    a.p_bs = p_bs;
    a.q_bs = q_bs;
    a.c_bs = c_bs;
    a.p_ext = p_extent;
    a.q_ext = q_extent;
    a.p_sx = (int32_t)p_s;
    a.q_sx = (int32_t)q_s;
    a.c_sq = (int32_t)c_sq;
    a.mp = (int32_t)mp;
    a.mq = (int32_t)mq;
    a.k = (int32_t)k;
    a.batch = (int32_t)batch;
    a.tp = (int32_t)tp;
    a.tq = (int32_t)tq;
    a.ntiles = (int32_t)ntiles;
    a.ntb = (int32_t)ntb;
    a.fold = (int32_t)fold;
    a.kv_last = (int32_t)(k - (ntb - 1) * BK);
    // the shared weight's tiles vary fastest; otherwise the operand with fewer tiles
    a.q_fast = (q_bs == 0) ? 1 : (p_bs == 0) ? 0 : (tq <= tp);
    a.alpha = alpha;
    a.nsub = nsub > 1 ? (int32_t)nsub : 1;
    a.p_bs2 = p_bs2;
    a.q_bs2 = q_bs2;
    a.c_vec16 = ((uintptr_t)c % 16 == 0) && (c_sq % (c_dtype == AVSE_F32 ? 4 : 8) == 0) &&
                (c_bs % (c_dtype == AVSE_F32 ? 4 : 8) == 0);
    // persistent: one workgroup per CU (128 KB of LDS each), a multiple of 8 (the XCD tile split)
    int64_t G = ((int64_t)cu_count_cached() + 7) / 8 * 8;
    const int64_t need = (ntiles + 7) / 8 * 8;
    if (G > need) G = need;
    const dim3 grid((unsigned)G), block(THREADS);
    hipStream_t st = (hipStream_t)stream;
    // fp32 out: straight from the accumulators for the folded weight gradients (small), LDS-staged lines otherwise
    const int epi = c_dtype == AVSE_BF16 ? 0 : (fold > 1 || !SPLIT) ? 1 : 2;
#define AVSE_PG_LAUNCH(PK, QK, E) hipLaunchKernelGGL((gemm_kernel<PK, QK, E, SPLIT>), grid, block, 0, st, a)
#define AVSE_PG_EPI(PK, QK)                                \
    do {                                                   \
        if (epi == 0) AVSE_PG_LAUNCH(PK, QK, 0);           \
        else if (epi == 1) AVSE_PG_LAUNCH(PK, QK, 1);      \
        else AVSE_PG_LAUNCH(PK, QK, 2);                    \
    } while (0)
    if (p_kc && q_kc) AVSE_PG_EPI(true, true);
    else if (p_kc) AVSE_PG_EPI(true, false);
    else if (q_kc) AVSE_PG_EPI(false, true);
    else AVSE_PG_EPI(false, false);
#undef AVSE_PG_EPI
#undef AVSE_PG_LAUNCH
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

extern "C" {

int avse_gemm_bf16(const avse_gemm_bf16_args* g, avse_stream_t stream) {
    if (!g) return AVSE_EINVAL;
    return launch_gemm<false>(g->batch, g->mp, g->mq, g->k, g->fold, g->p, nullptr, g->p_bs, g->p_sx, g->p_sk,
                              g->p_extent, nullptr, g->q, nullptr, g->q_bs, g->q_sx, g->q_sk, g->q_extent, nullptr, g->c,
                              g->c_bs, g->c_sq, g->alpha, g->c_dtype, stream);
}

int avse_gemm_f32s(const avse_gemm_f32s_args* g, avse_stream_t stream) {
    if (!g) return AVSE_EINVAL;
    return launch_gemm<true>(g->batch, g->mp, g->mq, g->k, g->fold, g->p_hi, g->p_lo, g->p_bs, g->p_sx, g->p_sk,
                             g->p_extent, g->p_max, g->q_hi, g->q_lo, g->q_bs, g->q_sx, g->q_sk, g->q_extent, g->q_max,
                             g->c, g->c_bs, g->c_sq, g->alpha, AVSE_F32, stream, g->nsub, g->p_bs2, g->q_bs2);
}

static int split16_planes_impl(int64_t b, int64_t r, int64_t c, const float* x, int64_t x_bs, int64_t x_rs, void* hi,
                               void* lo, int64_t h_bs, int64_t h_rs, uint32_t* maxbits, bool known,
                               avse_stream_t stream, bool zero_pad = false) {
    if (!x || !hi || !lo || !maxbits) return AVSE_EINVAL;
    if (b <= 0 || r <= 0 || c <= 0 || x_rs < c || (b > 1 && x_bs < (r - 1) * x_rs + c)) return AVSE_ESHAPE;
    if (h_rs < c || (b > 1 && h_bs < (r - 1) * h_rs + c)) return AVSE_ESHAPE;
    hipStream_t st = (hipStream_t)stream;
    if (!known && hipMemsetAsync(maxbits, 0, 4, st) != hipSuccess) return AVSE_ELAUNCH;
    PlanesArgs a;
    a.x = x;
    a.rows = b * r;
    a.r = r;
    a.c = c;
    a.bs = x_bs;
    a.rs = x_rs;
    a.hbs = h_bs;
    a.hrs = h_rs;
    a.maxbits = maxbits;
    a.hi = (_Float16*)hi;
    a.lo = (_Float16*)lo;
    // rows per workgroup: ~1024 float4 of work each
    const int64_t c4 = (c + 3) / 4;
    a.rpb = (int)std::max<int64_t>(1, std::min<int64_t>(1024 / std::max<int64_t>(c4, 1), 64));
    const int64_t blocks = (a.rows + a.rpb - 1) / a.rpb;
    if (blocks >= (1LL << 31)) return AVSE_ESHAPE;
    const bool xvec = ((uintptr_t)x % 16 == 0) && (x_rs % 4 == 0) && (b == 1 || x_bs % 4 == 0);
    const bool hvec = ((uintptr_t)hi % 8 == 0) && ((uintptr_t)lo % 8 == 0) && (h_rs % 4 == 0) && (b == 1 || h_bs % 4 == 0);
    // padded output rows (8-B aligned) differing from x's, or zero_pad with pad columns: the quadruple kernel, which
    // writes the pads as 0
    const bool pad = hvec && (h_rs != x_rs || (b > 1 && h_bs != x_bs) || (zero_pad && h_rs > c));
    if (!known) {
        const int64_t n = b * r * c;
        if (xvec) {
            hipLaunchKernelGGL(planes_absmax_kernel<true>, dim3((unsigned)std::min<int64_t>(blocks, AM_GRID)), dim3(AM_NT), 0,
                               st, a, blocks);
            AVSE_CHECK_LAUNCH();
        } else if (x_rs == c && (b == 1 || x_bs == r * c) && ((uintptr_t)x % 16 == 0) && n >= 4096) {
            // contiguous x whose rows are not 16-B aligned: the flat array in 4096-element rows (float4), the tail as
            // one more row
            PlanesArgs f = a;
            f.rows = f.r = n / 4096;
            f.c = f.rs = 4096;
            f.bs = 0;
            f.rpb = 1;
            hipLaunchKernelGGL(planes_absmax_kernel<true>, dim3((unsigned)std::min<int64_t>(f.rows, AM_GRID)), dim3(AM_NT), 0,
                               st, f, f.rows);
            AVSE_CHECK_LAUNCH();
            if (n % 4096) {
                f.x = x + f.rows * 4096;
                f.rows = f.r = 1;
                f.c = f.rs = n % 4096;
                hipLaunchKernelGGL(planes_absmax_kernel<false>, dim3(1), dim3(AM_NT), 0, st, f, (int64_t)1);
                AVSE_CHECK_LAUNCH();
            }
        } else {
            hipLaunchKernelGGL(planes_absmax_kernel<false>, dim3((unsigned)std::min<int64_t>(blocks, AM_GRID)), dim3(AM_NT), 0,
                               st, a, blocks);
            AVSE_CHECK_LAUNCH();
        }
    }
    if (pad) {
        PlanesArgs p2 = a;
        p2.rpb = (int)std::max<int64_t>(1, std::min<int64_t>(1024 / std::max<int64_t>(h_rs / 4, 1), 64));
        const int64_t pblocks = (a.rows + p2.rpb - 1) / p2.rpb;
        if (pblocks >= (1LL << 31)) return AVSE_ESHAPE;
        hipLaunchKernelGGL(planes_split_pad_kernel, dim3((unsigned)pblocks), dim3(256), 0, st, p2);
    } else if (xvec && hvec) {
        const int64_t n = b * r * c;
        const bool flat = x_rs == c && h_rs == c && (b == 1 || (x_bs == r * c && h_bs == r * c));
        if (flat && c < 1024 && n >= 4096) {
            // contiguous rows shorter than the workgroup's 1024-float4 pass (the (b, l, d_model = 512) projection
            // operands): the flat array as 4096-element rows, every thread busy (512-element rows left half of the
            // threads idle, one row at a time), the tail as one more row
            PlanesArgs f = a;
            f.rows = f.r = n / 4096;
            f.c = f.rs = f.hrs = 4096;
            f.bs = f.hbs = 0;
            f.rpb = 1;
            hipLaunchKernelGGL(planes_split_kernel<true>, dim3((unsigned)f.rows), dim3(256), 0, st, f);
            if (n % 4096) {
                AVSE_CHECK_LAUNCH();
                f.x = x + f.rows * 4096;
                f.hi = a.hi + f.rows * 4096;
                f.lo = a.lo + f.rows * 4096;
                f.rows = f.r = 1;
                f.c = f.rs = f.hrs = n % 4096;
                hipLaunchKernelGGL(planes_split_kernel<true>, dim3(1), dim3(256), 0, st, f);
            }
        } else {
            hipLaunchKernelGGL(planes_split_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, a);
        }
    } else {
        hipLaunchKernelGGL(planes_split_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, a);
    }
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_add_max(int64_t rows, int64_t lp, int64_t l, const float* a, const float* b, float* y, uint32_t* maxbits,
                 avse_stream_t stream) {
    if (!a || !b || !y || !maxbits) return AVSE_EINVAL;
    if (rows <= 0 || l <= 0 || lp < l || lp % 4 || rows * lp / 4 >= (1LL << 31)) return AVSE_ESHAPE;
    if (((uintptr_t)a | (uintptr_t)b | (uintptr_t)y) % 16) return AVSE_EALIGN;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(maxbits, 0, 4, st) != hipSuccess) return AVSE_ELAUNCH;
    const int n4 = (int)(rows * lp / 4);
    const unsigned grid = lp == l
        ? (unsigned)std::max<int64_t>(1, std::min<int64_t>((n4 + 1023) / 1024, 4 * cu_count_cached()))
        : (unsigned)std::max<int64_t>(1, std::min<int64_t>(rows, 8 * cu_count_cached()));
    if (lp == l)
        hipLaunchKernelGGL(add_max_kernel<false>, dim3(grid), dim3(256), 0, st, n4, (int)(lp / 4), (int)l,
                           reinterpret_cast<const float4*>(a), reinterpret_cast<const float4*>(b),
                           reinterpret_cast<float4*>(y), maxbits);
    else
        hipLaunchKernelGGL(add_max_kernel<true>, dim3(grid), dim3(256), 0, st, n4, (int)(lp / 4), (int)l,
                           reinterpret_cast<const float4*>(a), reinterpret_cast<const float4*>(b),
                           reinterpret_cast<float4*>(y), maxbits);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_split16_planes(int64_t b, int64_t r, int64_t c, const float* x, int64_t x_bs, int64_t x_rs, void* hi, void* lo,
                        uint32_t* maxbits, avse_stream_t stream) {
    return split16_planes_impl(b, r, c, x, x_bs, x_rs, hi, lo, x_bs, x_rs, maxbits, false, stream);
}

int avse_split16_planes_known(int64_t b, int64_t r, int64_t c, const float* x, int64_t x_bs, int64_t x_rs, void* hi,
                              void* lo, const uint32_t* maxbits, avse_stream_t stream) {
    return split16_planes_impl(b, r, c, x, x_bs, x_rs, hi, lo, x_bs, x_rs, const_cast<uint32_t*>(maxbits), true, stream);
}

int avse_split16_planes_to(int64_t b, int64_t r, int64_t c, const float* x, int64_t x_bs, int64_t x_rs, void* hi,
                           void* lo, int64_t h_bs, int64_t h_rs, uint32_t* maxbits, int32_t known, avse_stream_t stream) {
    return split16_planes_impl(b, r, c, x, x_bs, x_rs, hi, lo, h_bs, h_rs, maxbits, known != 0, stream, true);
}

}  // extern "C"
