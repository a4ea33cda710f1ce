// LSTM recurrence with each sequence spread over G workgroups (one per CU), W_hh resident in LDS.
//
// Same contract as lstm.hip (avse1 FusionNet nn.LSTM(1540, 257), /root/reference/baseline/avse1/model.py:88): the
// caller forms gx = X W_ih^T + b for all steps and the weight gradients as GEMMs; this file runs the time loop.
// lstm.hip runs one workgroup per sequence and streams W_hh (4H x H fp32, 1.06 MB at H = 257) from L2 every step:
// ~9.6 us per step, bound by one CU's L2 bandwidth, with 32 of 256 CUs busy (profiles/r03_avse1_default_bench_*).
// Here workgroup g of a sequence owns hidden units [u0, u1) (H / G each) and keeps the 4 gate rows of those units
// (forward) or their transpose (backward) in LDS for the whole launch, so a step reads no weights from HBM / L2:
//
//   forward step:  gate rows of the own units = gx + W_rows h_{t-1} (two lanes per gate row, four fma chains each),
//                  cell update of the own units, then h_t of the own units is
//                  handed to the sequence's G workgroups as data-tagged 8-byte granules {tag = step + 1, h} and every
//                  workgroup sweeps all H granules back into LDS (cdna_hip_programming.md §6 Guideline 16, form R2:
//                  the data is the flag, no fence).
//   backward step: the own units' pre-activation gate gradients, then the partial dh_{t-1} = W_own^T dg_own over ALL
//                  H units (two lanes per unit), published as H granules; each workgroup sums the G partials of its own
//                  units in a fixed order (deterministic).
//
// Granule slots alternate by step parity, so a producer one step ahead never overwrites a slot a slower consumer of
// the previous step still has to read.  Every slot is zeroed by the launch function (a memset node under graph
// capture).  Residency: a sequence's G workgroups must run concurrently.  They are consecutive block ids, and the
// launch refuses (AVSE_ENORESIDENT, nothing enqueued) a grid larger than the workgroups of that kernel the device can
// hold at once (occupancy x CUs), so with in-order dispatch every sequence's group eventually runs together even
// when other work holds CUs.  Every spin is still bounded (a CU mask, or persistent kernels of another process that
// never yield): on timeout the workgroup writes a code into the launch's status word (every later wait of the launch
// then gives up at once) AND into the caller's sticky error flag, which the host checks (kernels.lstm_group_status /
// raise_if_kernel_error; ddp.Trainer after every step), so a timed-out launch raises instead of training on garbage.
#include <algorithm>

#include "common.h"

namespace avse {
namespace lstmg {

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

constexpr int MAXG = 16, MAXU = 64, MAXH = 512;
// a hand-off wait gives up after 1 s of the 100 MHz realtime counter (a legitimate wait is one step, microseconds, or
// at most the time other work holds CUs the group still needs)
constexpr uint64_t WAIT_TICKS = 100000000ull;

// hardware exp / rcp (a few ulp; the step's dot products carry more rounding than that)
__device__ inline float sigm(float x) { return fast_rcp(1.f + fast_exp(-x)); }
__device__ inline float tanh_(float x) { return fmaf(2.f, sigm(2.f * x), -1.f); }

__device__ inline unsigned long long granule(unsigned tag, float v) {
    return ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(v);
}

// one wave: re-read the granules g[idx(lane, k)] (k < NK; idx < 0: none) until every tag == tag, then hand each value
// to out(lane, k, v) in ascending k.  Returns false on timeout or once another workgroup has timed out (status set).
template <int NK, typename Idx, typename Out>
__device__ inline bool sweep(const gu64* g, unsigned tag, gu32* status, gu32* errflag, Idx idx, Out out) {
    const int lane = threadIdx.x & 63;
    unsigned long long v[NK];
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    for (unsigned spins = 0;; ++spins) {
        bool ok = true;
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int64_t i = idx(lane, k);
            if (i >= 0) {
                v[k] = __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok &= (unsigned)(v[k] >> 32) == tag;
            }
        }
        if (__all(ok)) break;
        if ((spins & 63) == 63) {
            const unsigned st = __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (st != 0u || __builtin_amdgcn_s_memrealtime() - t_start > WAIT_TICKS) {
                if (st == 0u && lane == 0) {
                    __hip_atomic_store(status, 0x71000000u + tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(errflag, 0x71000000u + tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                return false;
            }
        }
        __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int k = 0; k < NK; ++k)
        if (idx(lane, k) >= 0) out(lane, k, __uint_as_float((unsigned)v[k]));
    return true;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, NOT for its global loads and
// stores (__syncthreads() drains vmcnt, which put the HBM latency of the step's output stores and of the next
// step's prefetched inputs on the critical path of every step: ~2 us).
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct Geo {
    int G, U, u0, nu, RS, R;        // groups, max units per group, own first unit / count, W row stride, gate rows
};

__device__ inline Geo geo(int H, int G, int g) {
    Geo q;
    q.G = G;
    q.U = (H + G - 1) / G;
    q.u0 = g * q.U;
    q.nu = max(0, min(H, q.u0 + q.U) - q.u0);
    q.RS = (H + 3) & ~3;
    q.R = 4 * q.nu;
    return q;
}

// hbuf: [2][B][H] granules.  LDS: W rows [4U][RS] (row rr = gate q * nu + unit), h [RS], gate pre-activations [4U]
__global__ __launch_bounds__(512) void fwd_kernel(int T, int H, int G, int reverse, const float* __restrict__ gx,
                                                  const float* __restrict__ whh, float* __restrict__ hout,
                                                  int64_t hout_bs, int64_t hout_ts, float* __restrict__ c_all,
                                                  float* __restrict__ gates, unsigned long long* hbuf_, unsigned* status_,
                                                  unsigned* errflag_) {
    gu64* hbuf = (gu64*)hbuf_;                        // global address space: agent-scope atomics
    gu32* status = (gu32*)status_;
    gu32* errflag = (gu32*)errflag_;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int b = blockIdx.x / G, g = blockIdx.x % G, tid = threadIdx.x;
    const int B = gridDim.x / G;
    const Geo q = geo(H, G, g);
    float* s_w = sm;                                  // [4U][RS]
    float* s_h = s_w + 4 * q.U * q.RS;                // [RS]
    float* s_gp = s_h + q.RS;                         // [4U]
    const int H4 = 4 * H;
    // stage the own gate rows (zero-padded to RS columns) and h_{-1} = 0
    for (int e = tid; e < q.R * q.RS; e += blockDim.x) {
        const int rr = e / q.RS, k = e % q.RS;
        const int gq = rr / q.nu, j = q.u0 + rr % q.nu;
        s_w[e] = k < H ? whh[(int64_t)(gq * H + j) * H + k] : 0.f;
    }
    for (int k = tid; k < q.RS; k += blockDim.x) s_h[k] = 0.f;
    // gate row rr = 32 * wave + lane % 32; lanes 32..63 of the wave take the upper half of k (two partial sums,
    // each over 4 independent fma chains: a short dependency chain per step)
    const int lane = tid & 63, rr = (tid >> 6) * 32 + (lane & 31), hk = lane >> 5;
    const bool rowok = rr < q.R;
    const int gq = rowok ? rr / q.nu : 0, jr = rowok ? q.u0 + rr % q.nu : 0;
    const int NK4 = q.RS / 4, KH4 = (NK4 + 1) / 2;
    const int k4lo = hk ? KH4 : 0, k4hi = hk ? NK4 : KH4;
    float c = 0.f;
    bool alive = true;
    __syncthreads();
    const float4* w4 = reinterpret_cast<const float4*>(s_w + (rowok ? rr : 0) * q.RS);
    const float4* h4 = reinterpret_cast<const float4*>(s_h);
    auto gx_at = [&](int s) {                         // this thread's gx entry of step s (its HBM latency is hidden
        const int t = reverse ? T - 1 - s : s;        // behind the previous step's hand-off)
        return (rowok && hk == 0) ? gx[((int64_t)b * T + t) * H4 + gq * H + jr] : 0.f;
    };
    float gx_next = gx_at(0);
    for (int s = 0; s < T; ++s) {
        const int t = reverse ? T - 1 - s : s;
        const int64_t bt = (int64_t)b * T + t;
        const float gx_cur = gx_next;
        if (s + 1 < T) gx_next = gx_at(s + 1);
        {
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
            for (int k4 = k4lo; k4 < k4hi; ++k4) {       // padding columns add w = 0 times h = 0
                const float4 w = w4[k4], hv = h4[k4];
                a.x = fmaf(w.x, hv.x, a.x);
                a.y = fmaf(w.y, hv.y, a.y);
                a.z = fmaf(w.z, hv.z, a.z);
                a.w = fmaf(w.w, hv.w, a.w);
            }
            float acc = (a.x + a.y) + (a.z + a.w);
            acc += __shfl_xor(acc, 32, 64);               // both k halves (commutative: same value in both lanes)
            if (rowok && hk == 0) s_gp[rr] = gx_cur + acc;
        }
        lds_barrier();
        gu64* slot = hbuf + ((int64_t)(s & 1) * B + b) * H;
        if (tid < q.nu) {
            const int j = q.u0 + tid;
            const float ig = sigm(s_gp[tid]), fg = sigm(s_gp[q.nu + tid]), gg = tanh_(s_gp[2 * q.nu + tid]),
                        og = sigm(s_gp[3 * q.nu + tid]);
            c = fmaf(fg, c, ig * gg);
            const float h = og * tanh_(c);
            __hip_atomic_store(slot + j, granule((unsigned)s + 1u, h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            hout[(int64_t)b * hout_bs + (int64_t)t * hout_ts + j] = h;
            c_all[bt * H + j] = c;
            float* gt = gates + bt * H4;
            gt[j] = ig;
            gt[H + j] = fg;
            gt[2 * H + j] = gg;
            gt[3 * H + j] = og;
        }
        if (tid < 64 && alive) {                          // wave 0 gathers h_t of all units (own ones included)
            alive = sweep<MAXH / 64>(slot, (unsigned)s + 1u, status, errflag,
                                     [&](int l, int k) -> int64_t { return l + 64 * k < H ? l + 64 * k : -1; },
                                     [&](int l, int k, float v) { s_h[l + 64 * k] = v; });
        }
        lds_barrier();
    }
}

// pbuf: [2][B][G][H] granules.  LDS: W^T of the own rows [H][RS4] (column rr = gate q * nu + unit, RS4 = 4U
// rounded to 4), dg [RS4], dh of the own units from the next step [U]
__global__ __launch_bounds__(768) void bwd_kernel(int T, int H, int G, int reverse, const float* __restrict__ dh_out,
                                                  int64_t dh_bs, int64_t dh_ts, const float* __restrict__ gates,
                                                  const float* __restrict__ c_all, const float* __restrict__ whh,
                                                  float* __restrict__ dgp, unsigned long long* pbuf_, unsigned* status_,
                                                  unsigned* errflag_) {
    gu64* pbuf = (gu64*)pbuf_;
    gu32* status = (gu32*)status_;
    gu32* errflag = (gu32*)errflag_;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int b = blockIdx.x / G, g = blockIdx.x % G, tid = threadIdx.x;
    const int B = gridDim.x / G;
    const Geo q = geo(H, G, g);
    const int RS4 = (4 * q.U + 3) & ~3;
    float* s_wt = sm;                                 // [H][RS4]
    float* s_dg = s_wt + H * RS4;                     // [RS4]
    float* s_dh = s_dg + RS4;                         // [U]
    const int H4 = 4 * H;
    for (int e = tid; e < H * RS4; e += blockDim.x) {
        const int k = e / RS4, rr = e % RS4;
        float v = 0.f;
        if (rr < q.R) {
            const int gq = rr / q.nu, j = q.u0 + rr % q.nu;
            v = whh[(int64_t)(gq * H + j) * H + k];
        }
        s_wt[e] = v;
    }
    for (int i = tid; i < RS4; i += blockDim.x) s_dg[i] = 0.f;
    if (tid < q.U) s_dh[tid] = 0.f;
    float dc_carry = 0.f;
    bool alive = true;
    // the own unit's step inputs (gates, c, c_prev, dh_out), loaded one step ahead: their HBM latency is hidden
    // behind the previous step's hand-off
    struct In { float ig, fg, gg, og, c, cp, dho; };
    auto load_in = [&](int s) {
        In v = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (tid < q.nu) {
            const int t = reverse ? s : T - 1 - s, tp = reverse ? t + 1 : t - 1, j = q.u0 + tid;
            const int64_t bt = (int64_t)b * T + t;
            const float* gt = gates + bt * H4;
            v.ig = gt[j]; v.fg = gt[H + j]; v.gg = gt[2 * H + j]; v.og = gt[3 * H + j];
            v.c = c_all[bt * H + j];
            v.cp = (tp >= 0 && tp < T) ? c_all[((int64_t)b * T + tp) * H + j] : 0.f;
            v.dho = dh_out[(int64_t)b * dh_bs + (int64_t)t * dh_ts + j];
        }
        return v;
    };
    const int col = (tid >> 6) * 32 + (tid & 31), hr = (tid & 63) >> 5;   // column, row half
    const bool colok = col < H;
    const int NR4 = RS4 / 4, RH4 = (NR4 + 1) / 2, r4lo = hr ? RH4 : 0, r4hi = hr ? NR4 : RH4;
    In nxt = load_in(0);
    __syncthreads();
    for (int s = 0; s < T; ++s) {
        const int t = reverse ? s : T - 1 - s;          // reverse order of the forward
        const int64_t bt = (int64_t)b * T + t;
        const In cur = nxt;
        if (s + 1 < T) nxt = load_in(s + 1);
        if (tid < q.nu) {
            const int j = q.u0 + tid;
            const float ig = cur.ig, fg = cur.fg, gg = cur.gg, og = cur.og, c = cur.c, cp = cur.cp;
            const float dh = cur.dho + s_dh[tid];
            const float tc = tanh_(c);
            const float dc = fmaf(dh * og, 1.f - tc * tc, dc_carry);
            const float di = dc * gg * ig * (1.f - ig);
            const float df = dc * cp * fg * (1.f - fg);
            const float dgv = dc * ig * (1.f - gg * gg);
            const float dO = dh * tc * og * (1.f - og);
            dc_carry = dc * fg;
            s_dg[tid] = di;
            s_dg[q.nu + tid] = df;
            s_dg[2 * q.nu + tid] = dgv;
            s_dg[3 * q.nu + tid] = dO;
            float* o = dgp + bt * H4;
            o[j] = di;
            o[H + j] = df;
            o[2 * H + j] = dgv;
            o[3 * H + j] = dO;
        }
        lds_barrier();
        gu64* slot = pbuf + ((int64_t)(s & 1) * B + b) * G * H;
        {                                                 // partial dh_{t-1}[col] over the own gate rows:
            const float4* w4 = reinterpret_cast<const float4*>(s_wt + (colok ? col : 0) * RS4);
            const float4* d4 = reinterpret_cast<const float4*>(s_dg);
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f);    // 2 lanes per column, 4 fma chains each
#pragma unroll 9
            for (int r4 = r4lo; r4 < r4hi; ++r4) {
                const float4 w = w4[r4], d = d4[r4];
                a.x = fmaf(w.x, d.x, a.x);
                a.y = fmaf(w.y, d.y, a.y);
                a.z = fmaf(w.z, d.z, a.z);
                a.w = fmaf(w.w, d.w, a.w);
            }
            float acc = (a.x + a.y) + (a.z + a.w);
            acc += __shfl_xor(acc, 32, 64);
            if (colok && hr == 0)
                __hip_atomic_store(slot + (int64_t)g * H + col, granule((unsigned)s + 1u, acc), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (tid < 64 && alive) {                          // wave 0, lane = own unit: dh = sum of the G partials
            float acc = 0.f;                               // in group order (deterministic)
            alive = sweep<MAXG>(slot, (unsigned)s + 1u, status, errflag,
                                [&](int l, int k) -> int64_t {
                                    return (l < q.nu && k < G) ? (int64_t)k * H + q.u0 + l : -1;
                                },
                                [&](int l, int k, float v) { acc += v; });
            if (tid < q.nu) s_dh[tid] = acc;
        }
        lds_barrier();
    }
}

}  // namespace lstmg
}  // namespace avse

using namespace avse;

namespace {

// smallest G in {1, 2, 4, 8, 16} whose forward and backward LDS fit 160 KiB with H / G <= 64 units per workgroup
// (H <= 384)
int group_size(int64_t H) {
    if (H <= 0 || H > 384) return 0;                  // backward: 2 lanes per unit column in <= 768 threads
    for (int G = 1; G <= lstmg::MAXG; G *= 2) {
        const int64_t U = (H + G - 1) / G, RS = (H + 3) & ~3LL, RS4 = (4 * U + 3) & ~3LL;
        const int64_t fwd = 4 * (4 * U * RS + RS + 4 * U), bwd = 4 * (H * RS4 + RS4 + U);
        if (U <= lstmg::MAXU && fwd <= 160 * 1024 && bwd <= 160 * 1024) return G;
    }
    return 0;
}

size_t fwd_lds(int64_t H, int G) {
    const int64_t U = (H + G - 1) / G, RS = (H + 3) & ~3LL;
    return 4 * (size_t)(4 * U * RS + RS + 4 * U);
}
size_t bwd_lds(int64_t H, int G) {
    const int64_t U = (H + G - 1) / G, RS4 = (4 * U + 3) & ~3LL;
    return 4 * (size_t)(H * RS4 + RS4 + U);
}
int fwd_threads(int64_t H, int G) {
    const int64_t U = (H + G - 1) / G;
    return (int)std::max<int64_t>(64, (4 * U + 31) / 32 * 64);          // 32 gate rows per wave
}
int bwd_threads(int64_t H) { return (int)((H + 31) / 32 * 64); }        // 32 columns per wave

// the kernels take up to 160 KiB of dynamic LDS (set once per process; thread-safe static init)
bool lds_attr_set() {
    static const bool ok =
        hipFuncSetAttribute(reinterpret_cast<const void*>(&lstmg::fwd_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess &&
        hipFuncSetAttribute(reinterpret_cast<const void*>(&lstmg::bwd_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    return ok;
}

// workgroups of the forward (backward) kernel the current device holds at once at hidden size H: occupancy per CU
// x CUs; 0 when it cannot be determined
int64_t capacity(int64_t H, bool backward) {
    const int G = group_size(H);
    if (G == 0 || !lds_attr_set()) return 0;
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    const hipError_t e = backward
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstmg::bwd_kernel, bwd_threads(H), bwd_lds(H, G))
        : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstmg::fwd_kernel, fwd_threads(H, G), fwd_lds(H, G));
    if (e != hipSuccess) return 0;
    return (int64_t)per_cu * cus;
}

}  // namespace

extern "C" {

int64_t avse_lstm_group_size(int64_t B, int64_t H) {
    const int G = group_size(H);
    return (G > 0 && B > 0 && B * G <= 256) ? G : 0;
}

int64_t avse_lstm_group_workspace_bytes(int64_t B, int64_t H) {
    const int64_t G = avse_lstm_group_size(B, H);
    if (G == 0) return 0;
    return 16 + 2 * B * G * H * 8;                    // status block + the backward's granules (>= the forward's)
}

int64_t avse_lstm_group_capacity(int64_t H, int32_t backward) { return capacity(H, backward != 0); }

int avse_lstm_fwd_group(int64_t B, int64_t T, int64_t H, int32_t reverse, const float* gx, const float* whh,
                        float* hout, int64_t hout_bs, int64_t hout_ts, float* c_all, float* gates, void* workspace,
                        uint32_t* error_flag, avse_stream_t stream) {
    if (!gx || !whh || !hout || !c_all || !gates || !workspace || !error_flag) return AVSE_EINVAL;
    const int G = (int)avse_lstm_group_size(B, H);
    if (G == 0 || T <= 0 || T >= (1LL << 31)) return AVSE_ESHAPE;
    if (B * G > capacity(H, false)) return AVSE_ENORESIDENT;
    hipStream_t st = (hipStream_t)stream;
    const int64_t used = 16 + 2 * B * H * 8;
    if (hipMemsetAsync(workspace, 0, (size_t)((used + 15) & ~15LL), st) != hipSuccess) return AVSE_ELAUNCH;
    auto* status = reinterpret_cast<unsigned*>(workspace);
    auto* hbuf = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(workspace) + 16);
    hipLaunchKernelGGL(lstmg::fwd_kernel, dim3((unsigned)(B * G)), dim3(fwd_threads(H, G)), fwd_lds(H, G), st, (int)T,
                       (int)H, G, (int)reverse, gx, whh, hout, hout_bs, hout_ts, c_all, gates, hbuf, status,
                       reinterpret_cast<unsigned*>(error_flag));
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_lstm_bwd_group(int64_t B, int64_t T, int64_t H, int32_t reverse, const float* dh_out, int64_t dh_bs,
                        int64_t dh_ts, const float* gates, const float* c_all, const float* whh, float* dgates,
                        void* workspace, uint32_t* error_flag, avse_stream_t stream) {
    if (!dh_out || !gates || !c_all || !whh || !dgates || !workspace || !error_flag) return AVSE_EINVAL;
    const int G = (int)avse_lstm_group_size(B, H);
    if (G == 0 || T <= 0 || T >= (1LL << 31)) return AVSE_ESHAPE;
    if (bwd_threads(H) > 768) return AVSE_ESHAPE;
    if (B * G > capacity(H, true)) return AVSE_ENORESIDENT;
    hipStream_t st = (hipStream_t)stream;
    const int64_t used = 16 + 2 * B * G * H * 8;
    if (hipMemsetAsync(workspace, 0, (size_t)((used + 15) & ~15LL), st) != hipSuccess) return AVSE_ELAUNCH;
    auto* status = reinterpret_cast<unsigned*>(workspace);
    auto* pbuf = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(workspace) + 16);
    hipLaunchKernelGGL(lstmg::bwd_kernel, dim3((unsigned)(B * G)), dim3(bwd_threads(H)), bwd_lds(H, G), st, (int)T,
                       (int)H, G, (int)reverse, dh_out, dh_bs, dh_ts, gates, c_all, whh, dgates, pbuf, status,
                       reinterpret_cast<unsigned*>(error_flag));
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
