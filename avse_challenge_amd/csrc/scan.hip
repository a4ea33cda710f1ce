// Selective-scan forward / backward for gfx950 (MI355X).
//
// Replaces selective_scan_cuda.fwd/bwd (mamba-ssm 1.1.3.post1, un-vendored) as called at
// /root/reference/Mamba-TasNet/modules/mamba/selective_scan_interface.py:42,67,218,252.
// Semantics: selective_scan_ref (:91-157) with real A, n_groups == 1, dstate 16.
//
// Decomposition (channel-parallel, sequential in time — no inter-chunk scan needed):
//   * workgroup = 256 threads = 4 waves; one batch row b and CPB = 64 channels d.
//   * a channel's 16 states are split over G = 4 ADJACENT lanes (4 states each), so the
//     per-step reduction y = sum_n C_n h_n is two DPP quad_perm adds (no LDS);
//   * time is processed in chunks of TC = 64 steps staged in LDS: u and dt (softplus
//     applied once per element at load time) interleaved as float2 rows (one ds_read_b64
//     per step), B and C transposed to [t][B0..15 C0..15] rows (two ds_read_b128 per step,
//     broadcast to the 16 channels of a wave), all HBM traffic lane-contiguous;
//   * the forward stores the state at every chunk end into the x intermediates, which is
//     what lets the backward restart every chunk without a second recompute pass.
// Backward per chunk (reverse order): recompute the chunk forward keeping the state at
// each 16-step sub-chunk start, then per sub-chunk (reverse) recompute 16 steps into
// registers and run the adjoint (lambda) recurrence backwards.  dB/dC (sums over d) are
// reduced across the wave's 16 channels with permlane swaps and DPP rotations (no selects, no LDS
// swizzles), across the 4 waves in LDS, and written as per-workgroup partial slabs summed by a
// second kernel — deterministic, no float atomics.
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace avse {
namespace scan {

constexpr int NSTATE = 16;
constexpr int NS = 4;            // states per lane
constexpr int G = NSTATE / NS;   // lanes per channel
constexpr int THREADS = 256;
constexpr int CPW = 64 / G;      // channels per wave
constexpr int CPB = 4 * CPW;     // channels per block (64)
constexpr int TC = 64;           // chunk (checkpoint) length
constexpr int TS = 16;           // backward sub-chunk
constexpr int UD_STRIDE = 2 * TC + 2;   // float2 rows, 16 channels of a wave -> distinct banks
constexpr int Z_STRIDE = 2 * TC + 2;
constexpr int BC_STRIDE = 2 * NSTATE + 4;  // 36 floats: 16-B aligned rows, 4-way write conflicts

struct Lane {
    int wave, lane, c, g;
};
__device__ inline Lane lane_ids() {
    Lane L;
    L.wave = threadIdx.x >> 6;
    L.lane = threadIdx.x & 63;
    L.c = L.wave * CPW + (L.lane >> 2);
    L.g = L.lane & 3;
    return L;
}

// ------------------------------------------------------------------------------- loaders
// Every thread owns tile column t = lane (one time step) and rows wave + 4*i; all the chunk's
// global loads are issued into registers first (several KB in flight per wave) and written to
// LDS afterwards, so a chunk load costs ~one HBM round trip instead of one per element.  The
// logical step t of chunk k lives at memory position pos = t0 + t, or L-1-(t0+t) when reversed.
constexpr int RPT = CPB * TC / THREADS;        // 16 rows per thread
constexpr int BPT = NSTATE * TC / THREADS;     // 4 B (and C) rows per thread

__device__ inline int tpos(int t, int L, bool rev) { return rev ? L - 1 - t : t; }

// Loaded values stay in the load's destination register until first use: for bf16 the raw 16-bit
// pattern (zero-extended by buffer_load_u16) is widened to fp32 only where it is consumed, so the
// prefetch of chunk k + 1 is not waited for right after it is issued (decoding at load time forced
// s_waitcnt vmcnt(0) there: the bf16 forward ran 1.7x slower than fp32, profiles/r01_scan_study.txt).
template <typename Tin> struct rawv;
template <> struct rawv<float> {
    using R = float;
    __device__ static inline R ld(__amdgpu_buffer_rsrc_t r, int v, int s) { return bufld<float>::ld(r, v, s); }
    __device__ static inline float f(R x) { return x; }
};
template <> struct rawv<bf16_t> {
    using R = uint32_t;
    __device__ static inline R ld(__amdgpu_buffer_rsrc_t r, int v, int s) {
        return (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, v * 2, s * 2, 0);
    }
    __device__ static inline float f(R x) { return __uint_as_float(x << 16); }
};

template <typename Tin>
struct RowRegs {
    typename rawv<Tin>::R v[RPT];
    __device__ inline void load(const Tin* p, int64_t bs, int64_t ds, int b, int d0, int D, int t0, int tn, int L,
                                bool rev) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        const int nrow = min(CPB, D - d0);
        const auto rs = make_rsrc(p + b * bs + (int64_t)d0 * ds, (int64_t)(nrow - 1) * ds + L);
        const int voff = wave * (int)ds + tpos(t0 + lane, L, rev);
#pragma unroll
        for (int i = 0; i < RPT; ++i) v[i] = rawv<Tin>::ld(rs, voff, 4 * i * (int)ds);   // raw: masked at use
    }
    __device__ inline float at(int i) const { return rawv<Tin>::f(v[i]); }
    // element i is real data iff the lane's step is inside the chunk and the row exists; the
    // select happens when the registers are consumed, so no wait is forced at load time
    __device__ inline float get(int i, int tn, int nrow) const {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        return (lane < tn && wave + 4 * i < nrow) ? at(i) : 0.f;
    }
};

template <typename Tin>
struct BCRegs {
    typename rawv<Tin>::R bv[BPT], cv[BPT];
    __device__ inline void load(const Tin* B, int64_t B_bs, int64_t B_ns, const Tin* C, int64_t C_bs, int64_t C_ns,
                                int b, int t0, int tn, int L, bool rev) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        const int pos = tpos(t0 + lane, L, rev);
        const auto rb = make_rsrc(B + b * B_bs, (int64_t)(NSTATE - 1) * B_ns + L);
        const auto rc = make_rsrc(C + b * C_bs, (int64_t)(NSTATE - 1) * C_ns + L);
        const int vb = wave * (int)B_ns + pos, vc = wave * (int)C_ns + pos;
#pragma unroll
        for (int i = 0; i < BPT; ++i) {
            bv[i] = rawv<Tin>::ld(rb, vb, 4 * i * (int)B_ns);
            cv[i] = rawv<Tin>::ld(rc, vc, 4 * i * (int)C_ns);
        }
    }
    __device__ inline void store(float* s_bc, int tn) const {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        const bool tv = lane < tn;
#pragma unroll
        for (int i = 0; i < BPT; ++i) {
            s_bc[lane * BC_STRIDE + wave + 4 * i] = tv ? rawv<Tin>::f(bv[i]) : 0.f;
            s_bc[lane * BC_STRIDE + NSTATE + wave + 4 * i] = tv ? rawv<Tin>::f(cv[i]) : 0.f;
        }
    }
};

// (u, dt) rows: dt = softplus(delta + bias) applied once per element here; bias_r holds the
// thread's 16 row biases (loaded once per kernel, so no global load sits in the chunk loop)
template <typename Tin, bool SOFTPLUS, bool HAS_BIAS, bool FULL>
__device__ inline void store_ud(float* s_ud, const RowRegs<Tin>& ru, const RowRegs<Tin>& rd, const float* bias_r,
                                int tn, int nrow) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        float dt = rd.at(i);
        if (HAS_BIAS) dt += bias_r[i];
        if (SOFTPLUS) dt = softplus2(dt);     // the forward's dt bit for bit (its replay restarts from the forward's states)
        float uv = ru.at(i);
        if (!FULL) {
            const bool ok = lane < tn && wave + 4 * i < nrow;
            dt = ok ? dt : 0.f;
            uv = ok ? uv : 0.f;
        }
        *reinterpret_cast<float2*>(&s_ud[(wave + 4 * i) * UD_STRIDE + 2 * lane]) = make_float2(uv, dt);
    }
}

// Forward staging: (dt u, dt) rows with dt = softplus(delta + bias), and D u kept in the thread's registers for
// the flush (the flush thread owns the same (row, step) elements), so the recurrence does neither the dt u
// product nor the D u skip term per lane and step.  FULL: every step and row of the chunk is real data, no
// selects (all chunks but the row's last one).
template <typename Tin, bool SOFTPLUS, bool HAS_BIAS, bool HAS_D, bool FULL>
__device__ inline void store_fwd(float* s_ud, const RowRegs<Tin>& ru, const RowRegs<Tin>& rd, const float2* s_par,
                                 float* du_keep, int tn, int nrow) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        const float2 par = s_par[wave + 4 * i];         // (bias, D) of the row: one broadcast LDS read
        float dt = rd.at(i);
        if (HAS_BIAS) dt += par.x;
        if (SOFTPLUS) dt = softplus2(dt);
        float uv = ru.at(i);
        if (!FULL) {
            const bool ok = lane < tn && wave + 4 * i < nrow;
            dt = ok ? dt : 0.f;
            uv = ok ? uv : 0.f;
        }
        du_keep[i] = HAS_D ? par.y * uv : 0.f;
        *reinterpret_cast<float2*>(&s_ud[(wave + 4 * i) * UD_STRIDE + 2 * lane]) = make_float2(dt * uv, dt);
    }
}

// the wave index as a wave-uniform value: row biases (and row offsets) then live in SGPRs
__device__ inline int wave_u() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

template <bool HAS_BIAS>
__device__ inline void load_bias_rows(float* bias_r, const float* bias, int d0, int D) {
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < RPT; ++i) bias_r[i] = (HAS_BIAS && d0 + wave + 4 * i < D) ? bias[d0 + wave + 4 * i] : 0.f;
}

// max |.| over the workgroup's 4 waves into *p as float bits (one vector atomic per workgroup -- same-word atomics
// serialise far from the CUs; non-negative floats order as their bits): the producer-side max of an accumulated
// output, for the split-fp16 GEMM that consumes it (round 6).  Every thread of the workgroup calls it.
__device__ inline void block_absmax_to(float m, uint32_t* p) {
    __shared__ uint32_t s_mx[THREADS / 64];
    uint32_t bits = __float_as_uint(m);
    for (int o = 32; o >= 1; o >>= 1) bits = max(bits, (uint32_t)__shfl_xor((int)bits, o, 64));
    if ((threadIdx.x & 63) == 0) s_mx[threadIdx.x >> 6] = bits;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < THREADS / 64; ++w) bits = max(bits, s_mx[w]);
        atomicMax(p, bits);
    }
}

// ------------------------------------------------------------------------------- forward
template <typename Tin, bool HAS_Z, bool HAS_D, bool HAS_BIAS, bool SOFTPLUS>
__global__ __launch_bounds__(THREADS) void fwd_kernel(avse_scan_fwd_args a, int nblk_d) {
    // z is not staged in LDS: the flush re-reads the chunk's z (L2 / Infinity-Cache resident: it was
    // read one chunk earlier by a neighbouring workgroup or is still in flight) and applies silu
    // there.  That keeps LDS at 42 KB and VGPRs under 168, i.e. 3 workgroups (12 waves) per CU.
    __shared__ __attribute__((aligned(16))) float s_ud[CPB * UD_STRIDE];
    __shared__ __attribute__((aligned(16))) float s_bc[TC * BC_STRIDE];
    __shared__ float2 s_par[CPB];                      // (delta_bias, D) per row of the block

    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int b = bid / nblk_d, d0 = (bid % nblk_d) * CPB;
    const int D = (int)a.dim, L = (int)a.seqlen;
    const bool rev = a.reverse != 0;
    const Lane id = lane_ids();
    const int d = d0 + id.c;
    const bool dvalid = d < D;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x < CPB) {
        const int r = d0 + (int)threadIdx.x;
        s_par[threadIdx.x] = make_float2((HAS_BIAS && r < D) ? a.delta_bias[r] : 0.f, (HAS_D && r < D) ? a.D[r] : 0.f);
    }

    // the lane's 4 states as 2 packed pairs: every state update is v_pk_mul / v_pk_fma on pairs
    f2_t A2v[NS / 2], h2[NS / 2];
#pragma unroll
    for (int p = 0; p < NS / 2; ++p) {
        const int j = id.g * NS + 2 * p;
        A2v[p] = dvalid ? f2_t{a.A[(int64_t)d * NSTATE + j], a.A[(int64_t)d * NSTATE + j + 1]} * AVSE_LOG2E : f2_t{0.f, 0.f};
        h2[p] = f2_t{0.f, 0.f};
    }

    const Tin* u = (const Tin*)a.u;
    const Tin* dl = (const Tin*)a.delta;
    const Tin* z = (const Tin*)a.z;
    const int nck = (L + TC - 1) / TC;
    const int nck32 = (L + 31) / 32;
    float* xrow = a.x + ((int64_t)b * D + (dvalid ? d : 0)) * nck32 * (2 * NSTATE) + 2 * id.g * NS;

    const int nrow = min(CPB, D - d0);
    RowRegs<Tin> ru, rd;
    BCRegs<Tin> rbc;
    ru.load(u, a.u_bs, a.u_ds, b, d0, D, 0, min(TC, L), L, rev);
    rd.load(dl, a.delta_bs, a.delta_ds, b, d0, D, 0, min(TC, L), L, rev);
    rbc.load((const Tin*)a.B, a.B_bs, a.B_ns, (const Tin*)a.C, a.C_bs, a.C_ns, b, 0, min(TC, L), L, rev);
    __syncthreads();                                   // s_par
    float du_keep[RPT];                                // D u of the thread's staged elements, added at the flush
    float zmax = 0.f;                                  // out_z_max: running max |out_z| of the thread's elements

    for (int k = 0; k < nck; ++k) {
        const int t0 = k * TC, tn = min(TC, L - t0);
        // registers -> LDS (chunk k)
        if (tn == TC && nrow == CPB)
            store_fwd<Tin, SOFTPLUS, HAS_BIAS, HAS_D, true>(s_ud, ru, rd, s_par, du_keep, tn, nrow);
        else
            store_fwd<Tin, SOFTPLUS, HAS_BIAS, HAS_D, false>(s_ud, ru, rd, s_par, du_keep, tn, nrow);
        rbc.store(s_bc, tn);
        __syncthreads();
        // prefetch chunk k + 1 while chunk k computes
        if (k + 1 < nck) {
            const int t1 = t0 + TC, tn1 = min(TC, L - t1);
            ru.load(u, a.u_bs, a.u_ds, b, d0, D, t1, tn1, L, rev);
            rd.load(dl, a.delta_bs, a.delta_ds, b, d0, D, t1, tn1, L, rev);
            rbc.load((const Tin*)a.B, a.B_bs, a.B_ns, (const Tin*)a.C, a.C_bs, a.C_ns, b, t1, tn1, L, rev);
        }

        float* my_ud = &s_ud[id.c * UD_STRIDE];
        // 8 steps per iteration: the LDS reads of all 8 issue together and the 8 cross-lane
        // y reductions (DPP) are independent, so one wave per SIMD still keeps its pipes busy.
        constexpr int U = 8;
        auto steps = [&](int t, auto UNR) {
            constexpr int NU = decltype(UNR)::value;
            float yv[NU];
#pragma unroll
            for (int q = 0; q < NU; ++q) {
                const float2 ud = *reinterpret_cast<const float2*>(&my_ud[2 * (t + q)]);   // (dt u, dt)
                const float4 bq = *reinterpret_cast<const float4*>(&s_bc[(t + q) * BC_STRIDE + id.g * NS]);
                const float4 cq = *reinterpret_cast<const float4*>(&s_bc[(t + q) * BC_STRIDE + NSTATE + id.g * NS]);
                const f2_t bp[2] = {f2_t{bq.x, bq.y}, f2_t{bq.z, bq.w}};
                const f2_t cp[2] = {f2_t{cq.x, cq.y}, f2_t{cq.z, cq.w}};
                const f2_t dt2 = f2_t{ud.y, ud.y}, dtu2 = f2_t{ud.x, ud.x};
                f2_t y2 = f2_t{0.f, 0.f};
#pragma unroll
                for (int p = 0; p < NS / 2; ++p) {
                    h2[p] = exp2_2(dt2 * A2v[p]) * h2[p] + dtu2 * bp[p];
                    y2 += h2[p] * cp[p];
                }
                yv[q] = y2.x + y2.y;
            }
#pragma unroll
            for (int q = 0; q < NU; ++q) yv[q] = group_sum<G>(yv[q]);
            // every lane of the channel's quad holds the same sum and writes it to the same LDS word:
            // no exec-mask branch per step, so the NU reductions and stores schedule together
#pragma unroll
            for (int q = 0; q < NU; ++q) my_ud[2 * (t + q)] = yv[q];   // dt u slot <- y (D u added at the flush)
        };
        // always the full 64 steps: the staged tail of the last chunk is zero (dt = 0, u = 0, B = C = 0), which
        // leaves h unchanged, so no step needs a bounds test; the state is checkpointed every 16 steps
        // (x slot j = state after logical step 16 j + 15, clamped to the last step)
#pragma unroll 1
        for (int q32 = 0; q32 < TC / 32; ++q32) {
            steps(q32 * 32, std::integral_constant<int, U>());
            steps(q32 * 32 + U, std::integral_constant<int, U>());
            const f2_t ha0 = h2[0], ha1 = h2[1];               // state after step 16 of the 32
            steps(q32 * 32 + 2 * U, std::integral_constant<int, U>());
            steps(q32 * 32 + 3 * U, std::integral_constant<int, U>());
            const int r = k * (TC / 32) + q32;                  // x row: (after step 32r + 15, after 32r + 31)
            if (dvalid && r < nck32) {
                float4* xp = reinterpret_cast<float4*>(xrow + (int64_t)r * (2 * NSTATE));
                xp[0] = make_float4(ha0.x, h2[0].x, ha0.y, h2[0].y);
                xp[1] = make_float4(ha1.x, h2[1].x, ha1.y, h2[1].y);
            }
        }
        RowRegs<Tin> rz;       // this chunk's z for the gate, issued before the barrier wait (issuing it with the
        if (HAS_Z) rz.load(z, a.z_bs, a.z_ds, b, d0, D, t0, tn, L, rev);   // prefetch measured the same, round 3)
        RowRegs<Tin> racc;     // out_z_accumulate: the other direction's gated output, added at the flush
        if (HAS_Z && a.out_z_accumulate)
            racc.load((const Tin*)a.out_z, a.out_z_bs, a.out_z_ds, b, d0, D, t0, tn, L, rev);
        __syncthreads();
        // flush chunk k outputs (lane = time column, rows wave + 4i): buffer stores, row step in soffset
        {
            const int nrow = min(CPB, D - d0);
            const auto ro = make_rsrc((Tin*)a.out + b * a.out_bs + (int64_t)d0 * a.out_ds,
                                      (int64_t)(nrow - 1) * a.out_ds + L);
            const int vo = wave * (int)a.out_ds + tpos(t0 + lane, L, rev);
            // rows past D need no test: their offsets lie beyond the resource's range, whose stores the hardware
            // drops; steps past L do (inside the range they would land in the row padding), one exec mask for all
            float outv[RPT];
#pragma unroll
            for (int i = 0; i < RPT; ++i) outv[i] = s_ud[(wave + 4 * i) * UD_STRIDE + 2 * lane] + du_keep[i];
            if (a.out && lane < tn) {      // out is optional when z is given (training fwd: the bwd recomputes it)
#pragma unroll
                for (int i = 0; i < RPT; ++i) bufst<Tin>::st(ro, vo, 4 * i * (int)a.out_ds, outv[i]);
            }
            if (HAS_Z) {
                const auto rz_ = make_rsrc((Tin*)a.out_z + b * a.out_z_bs + (int64_t)d0 * a.out_z_ds,
                                           (int64_t)(nrow - 1) * a.out_z_ds + L);
                const int vz = wave * (int)a.out_z_ds + tpos(t0 + lane, L, rev);
#pragma unroll
                for (int i = 0; i < RPT; ++i) outv[i] *= siluf_(rz.at(i));   // 16 independent gates (ILP)
                if (a.out_z_accumulate) {
#pragma unroll
                    for (int i = 0; i < RPT; ++i) outv[i] += racc.at(i);
                }
                if (lane < tn) {
#pragma unroll
                    for (int i = 0; i < RPT; ++i) bufst<Tin>::st(rz_, vz, 4 * i * (int)a.out_z_ds, outv[i]);
                    if (a.out_z_max) {
#pragma unroll
                        for (int i = 0; i < RPT; ++i)
                            if (wave + 4 * i < nrow) zmax = fmaxf(zmax, fabsf(outv[i]));
                    }
                }
            }
        }
        __syncthreads();
    }
    if (HAS_Z && a.out_z_max) block_absmax_to(zmax, a.out_z_max);     // a.out_z_max: uniform over the grid
}

// ------------------------------------------------------------------------------- backward
// Sum of 8 values over the 16 channel lanes (lane bits 2..5) of a wave without selects: a
// permlane32_swap + add per pair halves 8 -> 4 values (bit 5), permlane16_swap + add halves 4 -> 2
// (bit 4), two DPP row rotations (ror 8, ror 4) finish bits 3 and 2.  Lane (b2, b3, b4, b5) then holds
// the full sums of value indices vi = 4 b5 + 2 b4 + j in r[j], j = 0, 1, for its own state group
// (bits 0-1); lanes with b2 = b3 = 0 carry the unique copy.  16 VALU, no LDS swizzles.
__device__ inline void rs8_swap(const float v[8], float r[2]) {
    // the swapped pairs of two adjacent value indices are added as one v_pk_add_f32 (3 packed adds for the 6
    // scalar ones of the two swap stages)
    f2_t w[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[2 * i]), __float_as_uint(v[2 * i + 4]), false, false);
        auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[2 * i + 1]), __float_as_uint(v[2 * i + 5]), false, false);
        w[i] = f2_t{__uint_as_float(p[0]), __uint_as_float(q[0])} + f2_t{__uint_as_float(p[1]), __uint_as_float(q[1])};
    }
    // w[0] = (w_0, w_1), w[1] = (w_2, w_3) in the notation of the scalar form
    auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(w[0].x), __float_as_uint(w[1].x), false, false);
    auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(w[0].y), __float_as_uint(w[1].y), false, false);
    const f2_t xy = f2_t{__uint_as_float(p[0]), __uint_as_float(q[0])} + f2_t{__uint_as_float(p[1]), __uint_as_float(q[1])};
    float xs[2] = {xy.x, xy.y};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        float x = xs[j];
        x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x128, 0xF, 0xF, true));   // row_ror:8
        x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x124, 0xF, 0xF, true));   // row_ror:4
        r[j] = x;
    }
}

// Reduce-scatter over a channel's quad (lanes g = 0..3): lane g returns the quad's sum of v[g].  Two DPP stages
// (xor 2, then xor 1), each lane keeping the half its partner does not: 9 VALU for 4 sums (4 group_sums: 8)
__device__ inline float quad_rs4(const float v[4], int g) {
    const bool b1 = (g & 2) != 0, b0 = (g & 1) != 0;
    float k[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) k[j] = (b1 ? v[j + 2] : v[j]) + dpp_xor2(b1 ? v[j] : v[j + 2]);
    return (b0 ? k[1] : k[0]) + dpp_xor1(b0 ? k[0] : k[1]);
}

constexpr int RED = 8;   // adjoint steps buffered per cross-wave dB/dC flush

// keeps the scheduler from hoisting the LDS reads of all 16 unrolled steps (which needs ~10 VGPRs per step
// on top of the 64 of the state history and spills); the other wave of the SIMD covers the LDS latency
// (session-3 A/B, tools/gpu_round2z2.sh: masks letting VALU / SALU / transcendentals cross the fence moved the
// C3 and C5 backward by -0.7 .. +1.8 %: the kernel is VALU-throughput bound, not latency bound)
#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

// PRE (delta_softplus == 2): delta already holds softplus(delta_raw + bias) (avse_dtproj's epilogue), so staging applies
// neither; the epilogue still returns ddelta w.r.t. delta_raw (x sigma = 1 - exp(-dt)) and accumulates ddelta_bias.
template <typename Tin, bool HAS_Z, bool HAS_D, bool HAS_BIAS, bool SOFTPLUS, bool FOLD, bool PRE = false>
__global__ __launch_bounds__(THREADS, 2) void bwd_kernel(avse_scan_bwd_args a, int nblk_d) {
    __shared__ __attribute__((aligned(16))) float s_ud[CPB * UD_STRIDE];   // (u, dt) -> (du, ddelta)
    __shared__ __attribute__((aligned(16))) float s_zg[CPB * Z_STRIDE];    // (F, g) -> (dz, g)  [(z, dout) unfolded]
    __shared__ __attribute__((aligned(16))) float s_bc[TC * BC_STRIDE];
    __shared__ __attribute__((aligned(16))) float s_red[4 * RED * 2 * NSTATE];
    __shared__ float s_bias[CPB];              // delta_bias of the block's rows (LDS, not 16 VGPRs per thread)

    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int b = bid / nblk_d, cb = bid % nblk_d, d0 = cb * CPB;
    const int D = (int)a.dim, L = (int)a.seqlen;
    const Lane id = lane_ids();
    const int d = d0 + id.c;
    const bool dvalid = d < D;
    const int nck = (L + TC - 1) / TC;
    const int nck32 = (L + 31) / 32;

    // the lane's 4 states as 2 packed pairs (v_pk_mul / v_pk_fma), as in the forward
    constexpr int NP = NS / 2;
    f2_t A2v[NP];                              // A log2(e); dL/d(dt) sums A2v terms and is scaled by ln 2 once
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const int j = id.g * NS + 2 * p;
        A2v[p] = dvalid ? f2_t{a.A[(int64_t)d * NSTATE + j], a.A[(int64_t)d * NSTATE + j + 1]} * AVSE_LOG2E
                        : f2_t{0.f, 0.f};
    }
    const float Dv = (HAS_D && dvalid) ? a.D[d] : 0.f;

    // lam = dL/dh carried backwards over the whole row; dAn = lam dA of the step after the current one, so
    // lam(t) = g(t) C(t) + dAn is one packed FMA (the product is shared with that step's lhp)
    f2_t lam[NP], dAn[NP], dA_acc[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) { lam[p] = f2_t{0.f, 0.f}; dAn[p] = f2_t{0.f, 0.f}; dA_acc[p] = f2_t{0.f, 0.f}; }
    float dD_acc = 0.f, dbias_acc = 0.f;

    const Tin* u = (const Tin*)a.u;
    const Tin* dl = (const Tin*)a.delta;
    const Tin* z = (const Tin*)a.z;
    const Tin* dout = (const Tin*)a.dout;
    float* ws_bc = a.workspace;                                    // (b, nblk_d, 32, L)
    const int64_t slab = (int64_t)2 * NSTATE * L;
    const float* xrow = a.x + ((int64_t)b * D + (dvalid ? d : 0)) * nck32 * (2 * NSTATE) + 2 * id.g * NS;

    const bool rev = a.reverse != 0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nrow_b = min(CPB, D - d0);
    if (threadIdx.x < CPB) s_bias[threadIdx.x] = (HAS_BIAS && d0 + (int)threadIdx.x < D) ? a.delta_bias[d0 + threadIdx.x] : 0.f;
    __syncthreads();
    constexpr bool fold_gate = FOLD;        // = !recompute_out_z (the drop-in's reference call recomputes out_z)
    // the 16-step checkpoint (state after step ts - 1) of the sub-chunk starting at logical step ts, into ck_nx; slot
    // j < 0 (the row's first sub-chunk) restarts from zero.  Clamped address, select at use: no branch, no wait here
    f2_t ck_nx[NP];
    bool ck_ok = false;
    // (the prefetch also runs for sub-chunks past the row's end, which are skipped: the slot is clamped to the row's
    // 2 nck32 checkpoints, whose last one is the last element of the tensor for the last (b, d))
    auto ck_load = [&](int ts_abs) {
        const int j = ts_abs / TS - 1;
        ck_ok = ts_abs >= 0 && j >= 0 && j < 2 * nck32 && dvalid;
        const int jc = min(max(j, 0), 2 * nck32 - 1);
        const float* xp = xrow + (int64_t)(jc >> 1) * (2 * NSTATE) + (jc & 1);
#pragma unroll
        for (int p = 0; p < NP; ++p) ck_nx[p] = f2_t{xp[4 * p], xp[4 * p + 2]};
    };
    ck_load((nck - 1) * TC + (TC / TS - 1) * TS);

    float dzmax = 0.f;                                 // dz_max: running max |dz| of the thread's elements
    for (int k = nck - 1; k >= 0; --k) {
        const int t0 = k * TC, tn = min(TC, L - t0);
        {
            // all global loads of the chunk in flight before any LDS store; steps past the row's end stage
            // as zeros (dt = u = B = C = g = 0): the recurrences then pass through them unchanged
            RowRegs<Tin> ru, rd, rz, rg;
            BCRegs<Tin> rbc;
            ru.load(u, a.u_bs, a.u_ds, b, d0, D, t0, tn, L, rev);
            rd.load(dl, a.delta_bs, a.delta_ds, b, d0, D, t0, tn, L, rev);
            if (HAS_Z) rz.load(z, a.z_bs, a.z_ds, b, d0, D, t0, tn, L, rev);
            rg.load(dout, a.dout_bs, a.dout_ds, b, d0, D, t0, tn, L, rev);
            rbc.load((const Tin*)a.B, a.B_bs, a.B_ns, (const Tin*)a.C, a.C_bs, a.C_ns, b, t0, tn, L, rev);
            __builtin_amdgcn_sched_barrier(0);   // no bf16 decode scheduled between the loads (each would wait for its load)
            __syncthreads();
            // with z (and no out_z recompute) the gate is folded here, once per element instead of once
            // per lane per step: s_zg = (F, g) with g = dout silu(z) and F = dout sg (1 + z (1 - sg)),
            // so dz = out F in the replay; otherwise s_zg = (z, dout)
            {
                float bias_r[RPT];
#pragma unroll
                for (int i = 0; i < RPT; ++i) bias_r[i] = s_bias[wave + 4 * i];
                store_ud<Tin, SOFTPLUS, HAS_BIAS, false>(s_ud, ru, rd, bias_r, tn, nrow_b);
            }
#pragma unroll
            for (int i = 0; i < RPT; ++i) {
                const float zv = HAS_Z ? rz.get(i, tn, nrow_b) : 0.f, gd = rg.get(i, tn, nrow_b);
                float2 v = make_float2(zv, gd);
                if (HAS_Z && fold_gate) {
                    const float sg = sigmoidf_(zv);
                    v = make_float2(gd * sg * (1.f + zv * (1.f - sg)), gd * zv * sg);
                }
                *reinterpret_cast<float2*>(&s_zg[(wave + 4 * i) * Z_STRIDE + 2 * lane]) = v;
            }
            rbc.store(s_bc, tn);
        }
        __syncthreads();

        // 16-step sub-chunks in reverse; each restarts from the forward's 16-step checkpoint (no recompute pass
        // over the chunk), replays its steps into registers, then runs the adjoint
#pragma unroll 1
        for (int s = TC / TS - 1; s >= 0; --s) {
            const int ts = s * TS;
            // this sub-chunk's checkpoint was loaded one sub-chunk ago; issue the next one's now, so its global-memory
            // latency overlaps this sub-chunk's replay and adjoint (waited on where it was used: ~1-2 us per 16 steps)
            f2_t h0[NP];
            {
                const bool ok = ck_ok;
#pragma unroll
                for (int p = 0; p < NP; ++p) h0[p] = ok ? ck_nx[p] : f2_t{0.f, 0.f};
                ck_load(s > 0 ? t0 + ts - TS : t0 - TS);
            }
            if (ts >= tn) continue;                 // wholly past the row's end: lam stays 0, nothing to add
            // the replay keeps each step's dA = exp(dt A) (the adjoint re-evaluates no exponential) and the state after
            // every odd step; the adjoint gets h(t-1) dA(t) at odd steps as h(t) - dt u B(t), and at even steps
            // recomputes h(t) = dA(t) h(t-1) + dt u B(t) from the stored odd state (96 VGPRs instead of 64 for h alone)
            f2_t dAs[TS][NP], hodd[TS / 2][NP];
            {
                f2_t h[NP];
#pragma unroll
                for (int p = 0; p < NP; ++p) h[p] = h0[p];
                // the LDS operands of step i + 1 are read while step i computes (one step of software
                // pipelining: with two waves per SIMD the LDS latency is otherwise exposed every step)
                float2 ud_n = *reinterpret_cast<const float2*>(&s_ud[id.c * UD_STRIDE + 2 * ts]);
                float4 bq_n = *reinterpret_cast<const float4*>(&s_bc[ts * BC_STRIDE + id.g * NS]);
                float4 cq_n = *reinterpret_cast<const float4*>(&s_bc[ts * BC_STRIDE + NSTATE + id.g * NS]);
                float y_q[4];          // the quad partials of y = sum_n C h of the group's 4 steps
#pragma unroll
                for (int i = 0; i < TS; ++i) {
                    const int t = ts + i;
                    const float2 ud = ud_n;
                    const float4 bq = bq_n, cq = cq_n;
                    if (i + 1 < TS) {
                        ud_n = *reinterpret_cast<const float2*>(&s_ud[id.c * UD_STRIDE + 2 * (t + 1)]);
                        bq_n = *reinterpret_cast<const float4*>(&s_bc[(t + 1) * BC_STRIDE + id.g * NS]);
                        cq_n = *reinterpret_cast<const float4*>(&s_bc[(t + 1) * BC_STRIDE + NSTATE + id.g * NS]);
                    }
                    const f2_t bp[2] = {f2_t{bq.x, bq.y}, f2_t{bq.z, bq.w}};
                    const f2_t cp[2] = {f2_t{cq.x, cq.y}, f2_t{cq.z, cq.w}};
                    const f2_t dt2 = f2_t{ud.y, ud.y}, dtu2 = f2_t{ud.y * ud.x, ud.y * ud.x};
                    f2_t y2 = f2_t{0.f, 0.f};
#pragma unroll
                    for (int p = 0; p < NP; ++p) {
                        const f2_t dA = exp2_2(dt2 * A2v[p]);
                        dAs[i][p] = dA;
                        h[p] = pkfma(dA, h[p], dtu2 * bp[p]);
                        if (i & 1) hodd[i >> 1][p] = h[p];
                        y2 = pkfma(h[p], cp[p], y2);
                    }
                    y_q[i & 3] = y2.x + y2.y;
                    if ((i & 3) == 3 && HAS_Z) {
                        // the gate of steps i-3 .. i, one step per lane of the quad: lane g reduce-scatters y of step
                        // i - 3 + g, forms out = y + D u and dz = out F (folded) or the full silu gate (s_zg = (z, dout))
                        const float y = quad_rs4(y_q, id.g);
                        const int tg = t - 3 + id.g;
                        const float out = y + Dv * s_ud[id.c * UD_STRIDE + 2 * tg];
                        float* zg_p = &s_zg[id.c * Z_STRIDE + 2 * tg];
                        if (fold_gate) {
                            zg_p[0] = out * zg_p[0];                      // (F, g) -> (dz, g)
                        } else {
                            const float2 zg = *reinterpret_cast<const float2*>(zg_p);
                            const float sg = sigmoidf_(zg.x);
                            const float sl = zg.x * sg;
                            *reinterpret_cast<float2*>(zg_p) =
                                make_float2(zg.y * out * sg * (1.f + zg.x * (1.f - sg)), zg.y * sl);   // (dz, g)
                            if (!FOLD && a.recompute_out_z && dvalid && tg < tn)   // direct (uncoalesced) store
                                io<Tin>::st((Tin*)a.out_z + b * a.out_z_bs + (int64_t)d * a.out_z_ds + tpos(t0 + tg, L, rev),
                                            out * sl);
                        }
                    }
                    SCHED_FENCE();
                }
            }
            // adjoint sweep (the LDS operands of step i - 1 are read while step i computes)
            float2 ud_n = *reinterpret_cast<const float2*>(&s_ud[id.c * UD_STRIDE + 2 * (ts + TS - 1)]);
            float gv_n = s_zg[id.c * Z_STRIDE + 2 * (ts + TS - 1) + 1];
            float4 bq_n = *reinterpret_cast<const float4*>(&s_bc[(ts + TS - 1) * BC_STRIDE + id.g * NS]);
            float4 cq_n = *reinterpret_cast<const float4*>(&s_bc[(ts + TS - 1) * BC_STRIDE + NSTATE + id.g * NS]);
            float dus_q[4], ddt_q[4];     // quad partials of sum_n lam B and sum_n A lam dA h of the group's 4 steps
#pragma unroll
            for (int i = TS - 1; i >= 0; --i) {
                const int t = ts + i;
                float part[8];
                {
                    const float2 ud = ud_n;
                    const float gv = gv_n;
                    const float4 bq = bq_n, cq = cq_n;
                    if (i > 0) {
                        ud_n = *reinterpret_cast<const float2*>(&s_ud[id.c * UD_STRIDE + 2 * (t - 1)]);
                        gv_n = s_zg[id.c * Z_STRIDE + 2 * (t - 1) + 1];
                        bq_n = *reinterpret_cast<const float4*>(&s_bc[(t - 1) * BC_STRIDE + id.g * NS]);
                        cq_n = *reinterpret_cast<const float4*>(&s_bc[(t - 1) * BC_STRIDE + NSTATE + id.g * NS]);
                    }
                    const f2_t bp[2] = {f2_t{bq.x, bq.y}, f2_t{bq.z, bq.w}};
                    const f2_t cp[2] = {f2_t{cq.x, cq.y}, f2_t{cq.z, cq.w}};
                    const float dt = ud.y, uu = ud.x;
                    const f2_t dt2 = f2_t{dt, dt}, gv2 = f2_t{gv, gv};
                    const f2_t dtu2 = f2_t{dt * uu, dt * uu};
                    f2_t ddt2 = f2_t{0.f, 0.f}, dus2 = f2_t{0.f, 0.f};
#pragma unroll
                    for (int p = 0; p < NP; ++p) {
                        // dAn holds lam(t + 1) dA(t + 1): the product the previous step formed for its lhp
                        lam[p] = pkfma(gv2, cp[p], dAn[p]);
                        const f2_t dA = dAs[i][p];
                        const f2_t ldA = lam[p] * dA;
                        f2_t ht, lhp;                              // h(t) and lam dA h(t - 1)
                        if (i & 1) {
                            ht = hodd[i >> 1][p];
                            lhp = lam[p] * pkfma(-dtu2, bp[p], ht);
                        } else {
                            const f2_t hp = (i == 0) ? h0[p] : hodd[i > 0 ? (i - 1) >> 1 : 0][p];
                            ht = pkfma(dA, hp, dtu2 * bp[p]);
                            lhp = ldA * hp;
                        }
                        ddt2 = pkfma(A2v[p], lhp, ddt2);           // x ln 2 and + u * sum(lam B) once per lane, below
                        dus2 = pkfma(lam[p], bp[p], dus2);
                        dA_acc[p] = pkfma(dt2, lhp, dA_acc[p]);
                        const f2_t pb = lam[p] * dtu2, pc = gv2 * ht;
                        part[2 * p] = pb.x;
                        part[2 * p + 1] = pb.y;
                        part[4 + 2 * p] = pc.x;
                        part[4 + 2 * p + 1] = pc.y;
                        dAn[p] = ldA;
                    }
                    dus_q[i & 3] = dus2.x + dus2.y;               // lane partials; summed over the quad below
                    ddt_q[i & 3] = ddt2.x + ddt2.y;
                }
                SCHED_FENCE();
                float r2[2];
                rs8_swap(part, r2);
                {
                    // vi = 4 b5 + 2 b4 + j: slot = (b5 ? C : B) + g * 4 + 2 b4 + j.  The slot does not depend on lane
                    // bits 2-3 and those four lanes hold the same sums, so all of them store (same word, same value):
                    // no exec-mask branch, and the reduction stays in the step's basic block for the scheduler
                    const int slot = ((id.lane >> 5) & 1) * NSTATE + id.g * NS + ((id.lane >> 4) & 1) * 2;
                    float* dst = &s_red[(id.wave * RED + (i & (RED - 1))) * 2 * NSTATE + slot];
                    *reinterpret_cast<float2*>(dst) = make_float2(r2[0], r2[1]);
                }
                if ((i & 3) == 0) {
                    // per-channel epilogue of steps i .. i+3, one step per lane of the quad (not 4 copies of each):
                    // lane g reduce-scatters the quad's partials to the sums of step i + g and finishes that step's
                    // du, ddelta (the softplus derivative included) and its dD / ddelta_bias terms
                    const float dus = quad_rs4(dus_q, id.g), ddt_s = quad_rs4(ddt_q, id.g);
                    const int tg = ts + i + id.g;
                    float* ud_p = &s_ud[id.c * UD_STRIDE + 2 * tg];
                    const float2 ud = *reinterpret_cast<const float2*>(ud_p);
                    const float gv = s_zg[id.c * Z_STRIDE + 2 * tg + 1];
                    const float ddt = ddt_s * AVSE_LN2 + ud.x * dus;
                    const float du = dus * ud.y + gv * Dv;
                    const float sig = (SOFTPLUS || PRE) ? (1.f - fast_exp(-ud.y)) : 1.f;
                    const float ddr = ddt * sig;
                    dD_acc += gv * ud.x;
                    dbias_acc += ddr;
                    *reinterpret_cast<float2*>(ud_p) = make_float2(du, ddr);
                }
                if ((i & (RED - 1)) == 0) {
                    // cross-wave sum of steps ts+i .. ts+i+RED-1 -> partial slab
                    __syncthreads();
                    for (int idx = threadIdx.x; idx < RED * 2 * NSTATE; idx += THREADS) {
                        const int slot = idx / RED, ii = idx % RED, tt = ts + i + ii;
                        if (tt < tn) {
                            float v = 0.f;
#pragma unroll
                            for (int w = 0; w < 4; ++w) v += s_red[(w * RED + ii) * 2 * NSTATE + slot];
                            ws_bc[((int64_t)b * nblk_d + cb) * slab + (int64_t)slot * L + tpos(t0 + tt, L, rev)] = v;
                        }
                    }
                    __syncthreads();
                }
            }
        }
        RowRegs<Tin> rdz;      // dz_accumulate: the other direction's dz, loaded across the barrier (its latency was
        if (HAS_Z && a.dz_accumulate)   // exposed per chunk when loaded at the store: +0.35 ms per C5 launch)
            rdz.load((const Tin*)a.dz, a.dz_bs, a.dz_ds, b, d0, D, t0, tn, L, rev);
        __syncthreads();
        // write du, ddelta, dz (+ out_z) tiles (lane = time column): buffer stores, row step in soffset
        {
            const int nrow = min(CPB, D - d0);
            const int pos = tpos(t0 + lane, L, rev);
            const auto r_du = make_rsrc((Tin*)a.du + b * a.du_bs + (int64_t)d0 * a.du_ds, (int64_t)(nrow - 1) * a.du_ds + L);
            const auto r_dd = make_rsrc((Tin*)a.ddelta + b * a.ddelta_bs + (int64_t)d0 * a.ddelta_ds,
                                        (int64_t)(nrow - 1) * a.ddelta_ds + L);
            const int v_du = wave * (int)a.du_ds + pos, v_dd = wave * (int)a.ddelta_ds + pos;
            // rows past D: beyond the resources' ranges (stores dropped by the hardware); steps past L: exec mask
            float2 v[RPT];
#pragma unroll
            for (int i = 0; i < RPT; ++i) v[i] = *reinterpret_cast<const float2*>(&s_ud[(wave + 4 * i) * UD_STRIDE + 2 * lane]);
            if (lane < tn) {
#pragma unroll
                for (int i = 0; i < RPT; ++i) {
                    bufst<Tin>::st(r_du, v_du, 4 * i * (int)a.du_ds, v[i].x);
                    bufst<Tin>::st(r_dd, v_dd, 4 * i * (int)a.ddelta_ds, v[i].y);
                }
            }
            if (HAS_Z) {
                const auto r_dz = make_rsrc((Tin*)a.dz + b * a.dz_bs + (int64_t)d0 * a.dz_ds, (int64_t)(nrow - 1) * a.dz_ds + L);
                const int v_dz = wave * (int)a.dz_ds + pos;
                float dzv[RPT];
#pragma unroll
                for (int i = 0; i < RPT; ++i) dzv[i] = s_zg[(wave + 4 * i) * Z_STRIDE + 2 * lane];
                if (a.dz_accumulate) {             // the other BiMamba direction's dz, summed in place (round 6)
#pragma unroll
                    for (int i = 0; i < RPT; ++i) dzv[i] += rdz.at(i);
                }
                if (lane < tn) {
#pragma unroll
                    for (int i = 0; i < RPT; ++i) bufst<Tin>::st(r_dz, v_dz, 4 * i * (int)a.dz_ds, dzv[i]);
                    if (a.dz_max) {
#pragma unroll
                        for (int i = 0; i < RPT; ++i)
                            if (wave + 4 * i < nrow) dzmax = fmaxf(dzmax, fabsf(dzv[i]));
                    }
                }
            }
        }
        __syncthreads();
    }
    if (HAS_Z && a.dz_max) block_absmax_to(dzmax, a.dz_max);
    // per-(b, d) partials of dA, dD, ddelta_bias
    float* ws_d = ws_bc + (int64_t)a.batch * nblk_d * slab;       // (b, D, 18)
    if (dvalid) {
        float* p = ws_d + ((int64_t)b * D + d) * (NSTATE + 2);
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            p[id.g * NS + 2 * q] = dA_acc[q].x;
            p[id.g * NS + 2 * q + 1] = dA_acc[q].y;
        }
        dD_acc = group_sum<G>(dD_acc);                  // each lane of the quad finished a quarter of the steps
        dbias_acc = group_sum<G>(dbias_acc);
        if (id.g == 0) {
            p[NSTATE] = dD_acc;
            p[NSTATE + 1] = dbias_acc;
        }
    }
}

// dB/dC: sum partial slabs over channel blocks
__global__ void reduce_bc_kernel(const float* ws, int nblk_d, int L, int batch, float* dB, int64_t dB_bs,
                                 int64_t dB_ns, float* dC, int64_t dC_bs, int64_t dC_ns) {
    const int64_t slab = (int64_t)2 * NSTATE * L;
    const int64_t total = (int64_t)batch * 2 * NSTATE * L;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int t = (int)(i % L);
        const int slot = (int)((i / L) % (2 * NSTATE));
        const int b = (int)(i / ((int64_t)L * 2 * NSTATE));
        float v = 0.f;
        for (int cb = 0; cb < nblk_d; ++cb) v += ws[((int64_t)b * nblk_d + cb) * slab + (int64_t)slot * L + t];
        if (slot < NSTATE) dB[b * dB_bs + slot * dB_ns + t] = v;
        else dC[b * dC_bs + (slot - NSTATE) * dC_ns + t] = v;
    }
}

// dA (d, n), dD (d), ddelta_bias (d): sum over batch — one workgroup per channel d, threads striding
// over the batch (DPMamba's inter pass runs thousands of sequences), then a fixed tree (deterministic)
__global__ __launch_bounds__(THREADS) void reduce_d_kernel(const float* ws_d, int batch, int D, float* dA, float* dD,
                                                           float* dbias) {
    constexpr int NV = NSTATE + 2;
    __shared__ float red[THREADS / 64][NV];
    const int d = blockIdx.x;
    float v[NV];
#pragma unroll
    for (int c = 0; c < NV; ++c) v[c] = 0.f;
    for (int b = threadIdx.x; b < batch; b += THREADS) {
        const float* p = ws_d + ((int64_t)b * D + d) * NV;
#pragma unroll
        for (int c = 0; c < NV; ++c) v[c] += p[c];
    }
#pragma unroll
    for (int c = 0; c < NV; ++c) {
        float t = v[c];
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) t += __shfl_xor(t, m, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][c] = t;
    }
    __syncthreads();
    if (threadIdx.x < NV) {
        const int c = threadIdx.x;
        const float t = red[0][c] + red[1][c] + red[2][c] + red[3][c];
        if (c < NSTATE) dA[(int64_t)d * NSTATE + c] = t;
        else if (c == NSTATE) { if (dD) dD[d] = t; }
        else if (dbias) dbias[d] = t;
    }
}

template <typename Tin, bool HAS_Z, bool HAS_D, bool HAS_BIAS>
static void launch_fwd(const avse_scan_fwd_args& a, int nblk_d, int nblocks, hipStream_t st) {
    if (a.delta_softplus == 1)          // 2: delta holds the final step sizes (avse_dtproj), nothing to apply
        hipLaunchKernelGGL((fwd_kernel<Tin, HAS_Z, HAS_D, HAS_BIAS, true>), dim3(nblocks), dim3(THREADS), 0, st, a, nblk_d);
    else
        hipLaunchKernelGGL((fwd_kernel<Tin, HAS_Z, HAS_D, HAS_BIAS, false>), dim3(nblocks), dim3(THREADS), 0, st, a, nblk_d);
}

template <typename Tin, bool HAS_Z, bool HAS_D, bool HAS_BIAS>
static void launch_bwd(const avse_scan_bwd_args& a, int nblk_d, int nblocks, hipStream_t st) {
    const bool fold = !(HAS_Z && a.recompute_out_z);
    if constexpr (!HAS_BIAS) {
        if (a.delta_softplus == 2) {
            if (fold)
                hipLaunchKernelGGL((bwd_kernel<Tin, HAS_Z, HAS_D, false, false, true, true>), dim3(nblocks), dim3(THREADS), 0,
                                   st, a, nblk_d);
            else
                hipLaunchKernelGGL((bwd_kernel<Tin, HAS_Z, HAS_D, false, false, false, true>), dim3(nblocks), dim3(THREADS),
                                   0, st, a, nblk_d);
            return;
        }
    }
    if (a.delta_softplus && fold)
        hipLaunchKernelGGL((bwd_kernel<Tin, HAS_Z, HAS_D, HAS_BIAS, true, true>), dim3(nblocks), dim3(THREADS), 0, st, a, nblk_d);
    else if (a.delta_softplus)
        hipLaunchKernelGGL((bwd_kernel<Tin, HAS_Z, HAS_D, HAS_BIAS, true, false>), dim3(nblocks), dim3(THREADS), 0, st, a, nblk_d);
    else if (fold)
        hipLaunchKernelGGL((bwd_kernel<Tin, HAS_Z, HAS_D, HAS_BIAS, false, true>), dim3(nblocks), dim3(THREADS), 0, st, a, nblk_d);
    else
        hipLaunchKernelGGL((bwd_kernel<Tin, HAS_Z, HAS_D, HAS_BIAS, false, false>), dim3(nblocks), dim3(THREADS), 0, st, a, nblk_d);
}

}  // namespace scan
}  // namespace avse

using namespace avse;
using namespace avse::scan;

#define AVSE_DISPATCH_FLAGS(LAUNCH, T, ARGS, ...)                                                   \
    do {                                                                                           \
        const bool hz = ARGS.z != nullptr, hd = ARGS.D != nullptr, hb = ARGS.delta_bias != nullptr; \
        if (hz && hd && hb) LAUNCH<T, true, true, true>(ARGS, __VA_ARGS__);                        \
        else if (hz && hd) LAUNCH<T, true, true, false>(ARGS, __VA_ARGS__);                        \
        else if (hz && hb) LAUNCH<T, true, false, true>(ARGS, __VA_ARGS__);                        \
        else if (hz) LAUNCH<T, true, false, false>(ARGS, __VA_ARGS__);                             \
        else if (hd && hb) LAUNCH<T, false, true, true>(ARGS, __VA_ARGS__);                        \
        else if (hd) LAUNCH<T, false, true, false>(ARGS, __VA_ARGS__);                             \
        else if (hb) LAUNCH<T, false, false, true>(ARGS, __VA_ARGS__);                             \
        else LAUNCH<T, false, false, false>(ARGS, __VA_ARGS__);                                    \
    } while (0)

extern "C" {

int64_t avse_scan_n_chunks(int64_t seqlen) { return (seqlen + 31) / 32; }   // rows of two 16-step checkpoints

int64_t avse_scan_bwd_workspace_bytes(int64_t batch, int64_t dim, int64_t seqlen, int64_t dstate) {
    (void)dstate;
    const int64_t nblk_d = (dim + CPB - 1) / CPB;
    return 4 * (batch * nblk_d * 2 * NSTATE * seqlen + batch * dim * (NSTATE + 2));
}

static int check_mode(int32_t delta_softplus, const float* delta_bias) {
    if (delta_softplus < 0 || delta_softplus > 2) return AVSE_EINVAL;
    if (delta_softplus == 2 && delta_bias) return AVSE_EINVAL;     // the bias is already inside delta
    return AVSE_OK;
}

static int check_common(int64_t batch, int64_t dim, int64_t seqlen, int64_t dstate, int32_t dtype) {
    if (batch <= 0 || dim <= 0 || seqlen <= 0) return AVSE_ESHAPE;
    if (dstate != NSTATE) return AVSE_ESHAPE;
    if (dtype != AVSE_F32 && dtype != AVSE_BF16) return AVSE_EDTYPE;
    if (batch * ((dim + CPB - 1) / CPB) > (1LL << 30)) return AVSE_ESHAPE;
    return AVSE_OK;
}

int avse_scan_fwd(const avse_scan_fwd_args* a, avse_stream_t stream) {
    if (!a || !a->u || !a->delta || !a->A || !a->B || !a->C || !a->x) return AVSE_EINVAL;
    if (a->z ? !a->out_z : !a->out) return AVSE_EINVAL;
    int rc = check_mode(a->delta_softplus, a->delta_bias);
    if (rc) return rc;
    rc = check_common(a->batch, a->dim, a->seqlen, a->dstate, a->in_dtype);
    if (rc) return rc;
    const int nblk_d = (int)((a->dim + CPB - 1) / CPB);
    const int nblocks = (int)(a->batch * nblk_d);
    hipStream_t st = (hipStream_t)stream;
    if (a->in_dtype == AVSE_F32) AVSE_DISPATCH_FLAGS(launch_fwd, float, (*a), nblk_d, nblocks, st);
    else AVSE_DISPATCH_FLAGS(launch_fwd, bf16_t, (*a), nblk_d, nblocks, st);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_scan_bwd(const avse_scan_bwd_args* a, avse_stream_t stream) {
    if (!a || !a->u || !a->delta || !a->A || !a->B || !a->C || !a->dout || !a->x || !a->du || !a->ddelta ||
        !a->dA || !a->dB || !a->dC || !a->workspace)
        return AVSE_EINVAL;
    if (a->z && !a->dz) return AVSE_EINVAL;
    if (a->recompute_out_z && (!a->z || !a->out_z)) return AVSE_EINVAL;
    if (a->D && !a->dD) return AVSE_EINVAL;
    if (a->delta_bias && !a->ddelta_bias) return AVSE_EINVAL;
    int rc = check_mode(a->delta_softplus, a->delta_bias);
    if (rc) return rc;
    rc = check_common(a->batch, a->dim, a->seqlen, a->dstate, a->in_dtype);
    if (rc) return rc;
    const int nblk_d = (int)((a->dim + CPB - 1) / CPB);
    const int nblocks = (int)(a->batch * nblk_d);
    hipStream_t st = (hipStream_t)stream;
    if (a->in_dtype == AVSE_F32) AVSE_DISPATCH_FLAGS(launch_bwd, float, (*a), nblk_d, nblocks, st);
    else AVSE_DISPATCH_FLAGS(launch_bwd, bf16_t, (*a), nblk_d, nblocks, st);
    AVSE_CHECK_LAUNCH();
    const int64_t slab = 2 * NSTATE * a->seqlen;
    const float* ws_d = a->workspace + a->batch * nblk_d * slab;
    const int64_t tot = a->batch * 2 * NSTATE * a->seqlen;
    const int rb = (int)std::min<int64_t>((tot + 255) / 256, 4096);
    hipLaunchKernelGGL(reduce_bc_kernel, dim3(rb), dim3(256), 0, st, a->workspace, nblk_d, (int)a->seqlen,
                       (int)a->batch, (float*)a->dB, a->dB_bs, a->dB_ns, (float*)a->dC, a->dC_bs, a->dC_ns);
    AVSE_CHECK_LAUNCH();
    hipLaunchKernelGGL(reduce_d_kernel, dim3((unsigned)a->dim), dim3(THREADS), 0, st, ws_d, (int)a->batch,
                       (int)a->dim, a->dA, a->dD, a->ddelta_bias);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
