// STFT magnitude (framing + real FFT-512) and iSTFT (inverse real FFT + overlap-add) for gfx950.
//
// Replaces the CPU librosa 0.8.1 calls of the avse1 path (/root/reference/baseline/avse1):
//   dataset.py:112-118  |stft(y, n_fft=512, hop=128, win=512, 'hann', center=True)|.T
//   test.py:85-88       istft(mag * exp(i*angle(noisy_stft)), hop 128, win 512, length=len(clean))
// librosa 0.8.1 semantics: periodic Hann, reflect padding of n_fft/2 on both sides, no scaling;
// istft divides the overlap-added windowed frames by the window sum-square (where > tiny).
//
// One wave per frame.  The 512 real samples are packed as 256 complex values
// z[m] = x[2m] + i x[2m+1], transformed by a radix-4 Stockham FFT (4 stages, one radix-4
// butterfly per lane per stage, ping-pong through LDS, no bit reversal), then split into the
// 257 real-input bins X[k] = E[k] + W512^k O[k].  Window and twiddles are computed once per
// workgroup with sincospi (accurate), so the arithmetic is fp32 FFT (rel. err ~1e-6).
// HBM traffic: 4 B read per sample per frame (L2 absorbs the 4x frame overlap) + 4 B per bin.
#include "common.h"

namespace avse {
namespace stft {

constexpr int NFFT = 512, HOP = 128, NB = NFFT / 2 + 1, NC = 256;
constexpr int WAVES = 4, THREADS = 64 * WAVES;

struct Tables {
    float win[NFFT];
    float2 tw256[NC];       // exp(-2 pi i q / 256)
    float2 tw512[NC + 1];   // exp(-2 pi i k / 512)
};

__device__ inline float2 cmul(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
__device__ inline float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ inline float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ inline float2 cconj(float2 a) { return make_float2(a.x, -a.y); }

__device__ inline void init_tables(Tables& T) {
    for (int i = threadIdx.x; i < NFFT; i += THREADS) {
        // periodic Hann: 0.5 - 0.5 cos(2 pi n / 512)
        T.win[i] = 0.5f - 0.5f * cospif((float)i / 256.f);
    }
    for (int i = threadIdx.x; i < NC; i += THREADS) {
        float s, c;
        sincospif(-(float)i / 128.f, &s, &c);
        T.tw256[i] = make_float2(c, s);
    }
    for (int i = threadIdx.x; i <= NC; i += THREADS) {
        float s, c;
        sincospif(-(float)i / 256.f, &s, &c);
        T.tw512[i] = make_float2(c, s);
    }
}

// forward complex FFT-256 of buf (natural order in, natural order out); returns the buffer
// holding the result (a or b).  Called by one full wave.
__device__ inline float2* fft256(float2* a, float2* b, const Tables& T, int lane) {
    float2* src = a;
    float2* dst = b;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
        const int Ns = 1 << (2 * st);
        float2 v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = src[lane + 64 * r];
        const int m = lane & (Ns - 1);
        if (st > 0) {
#pragma unroll
            for (int r = 1; r < 4; ++r) v[r] = cmul(v[r], T.tw256[(m * r * (64 / Ns)) & 255]);
        }
        const float2 a0 = cadd(v[0], v[2]), a1 = csub(v[0], v[2]), a2 = cadd(v[1], v[3]);
        const float2 d13 = csub(v[1], v[3]);
        const float2 a3 = make_float2(d13.y, -d13.x);  // (v1 - v3) * (-i)
        const int base = (lane / Ns) * Ns * 4 + m;
        dst[base] = cadd(a0, a2);
        dst[base + Ns] = cadd(a1, a3);
        dst[base + 2 * Ns] = csub(a0, a2);
        dst[base + 3 * Ns] = csub(a1, a3);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        float2* t = src;
        src = dst;
        dst = t;
    }
    return src;
}

__global__ __launch_bounds__(THREADS) void stft_kernel(int batch, int T, int frames, const float* __restrict__ wave,
                                                       float* __restrict__ mag, float* __restrict__ spec) {
    __shared__ Tables tab;
    __shared__ float2 bufA[WAVES][NC], bufB[WAVES][NC];
    init_tables(tab);
    __syncthreads();
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int fid = blockIdx.x * WAVES + wid;
    if (fid >= batch * frames) return;
    const int b = fid / frames, f = fid % frames;
    const float* wr = wave + (int64_t)b * T;
    // load 8 consecutive padded samples per lane: n = 8*lane + e
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
        float xs[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int n = 8 * lane + e + q;
            int i = f * HOP + n - NFFT / 2;
            i = i < 0 ? -i : i;
            i = i >= T ? 2 * (T - 1) - i : i;
            xs[q] = wr[i] * tab.win[n];
        }
        bufA[wid][4 * lane + e / 2] = make_float2(xs[0], xs[1]);
    }
    __builtin_amdgcn_wave_barrier();
    float2* Z = fft256(bufA[wid], bufB[wid], tab, lane);
    float* mrow = mag + (int64_t)fid * NB;
    float* srow = spec ? spec + (int64_t)fid * NB * 2 : nullptr;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        const int k = lane + 64 * q;
        if (k <= NC && (q < 4 || lane == 0)) {
            const float2 zk = Z[k & 255];
            const float2 zr = cconj(Z[(NC - k) & 255]);
            const float2 E = make_float2(0.5f * (zk.x + zr.x), 0.5f * (zk.y + zr.y));
            const float2 dd = csub(zk, zr);
            const float2 O = make_float2(0.5f * dd.y, -0.5f * dd.x);   // -0.5i * (zk - conj(zr))
            const float2 X = cadd(E, cmul(tab.tw512[k], O));
            mrow[k] = sqrtf(X.x * X.x + X.y * X.y);
            if (srow) *reinterpret_cast<float2*>(&srow[2 * k]) = X;
        }
    }
}

// per frame: X = mag * unit(phase) -> windowed time frame (512) into frames_buf
__global__ __launch_bounds__(THREADS) void istft_frames_kernel(int batch, int frames, const float* __restrict__ mag,
                                                               const float* __restrict__ phase,
                                                               float* __restrict__ out) {
    __shared__ Tables tab;
    __shared__ float2 bufA[WAVES][NC], bufB[WAVES][NC];
    __shared__ float2 X[WAVES][NB];
    init_tables(tab);
    __syncthreads();
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int fid = blockIdx.x * WAVES + wid;
    if (fid >= batch * frames) return;
    const float* mrow = mag + (int64_t)fid * NB;
    const float* prow = phase + (int64_t)fid * NB * 2;
    for (int k = lane; k < NB; k += 64) {
        const float2 p = *reinterpret_cast<const float2*>(&prow[2 * k]);
        const float r = sqrtf(p.x * p.x + p.y * p.y);
        // np.angle(0) = 0 -> unit phase (1, 0)
        const float2 u = r > 0.f ? make_float2(p.x / r, p.y / r) : make_float2(1.f, 0.f);
        float2 v = make_float2(mrow[k] * u.x, mrow[k] * u.y);
        if (k == 0 || k == NC) v.y = 0.f;   // irfft ignores the imaginary DC / Nyquist parts
        X[wid][k] = v;
    }
    __builtin_amdgcn_wave_barrier();
    // Z[k] = E[k] + i O[k]; E = (X[k] + conj X[256-k]) / 2 ; O = (X[k] - conj X[256-k]) W^-k / 2
    // inverse FFT via conj(FFT(conj(Z))) / 256
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int k = lane + 64 * q;
        const float2 xk = X[wid][k];
        const float2 xr = cconj(X[wid][NC - k]);
        const float2 E = make_float2(0.5f * (xk.x + xr.x), 0.5f * (xk.y + xr.y));
        const float2 Od = make_float2(0.5f * (xk.x - xr.x), 0.5f * (xk.y - xr.y));
        const float2 O = cmul(Od, cconj(tab.tw512[k]));
        const float2 Z = make_float2(E.x - O.y, E.y + O.x);   // E + i O
        bufA[wid][k] = cconj(Z);
    }
    __builtin_amdgcn_wave_barrier();
    float2* z = fft256(bufA[wid], bufB[wid], tab, lane);
    float* orow = out + (int64_t)fid * NFFT;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int m = lane + 64 * q;
        const float2 v = z[m];
        // conj and scale: x[2m] = Re, x[2m+1] = -Im(FFT(conj Z)) / 256
        const float xe = v.x * (1.f / 256.f), xo = -v.y * (1.f / 256.f);
        *reinterpret_cast<float2*>(&orow[2 * m]) = make_float2(xe * tab.win[2 * m], xo * tab.win[2 * m + 1]);
    }
}

__global__ __launch_bounds__(256) void istft_ola_kernel(int batch, int fstride, int frames, int length,
                                                        const float* __restrict__ fb, float* __restrict__ out) {
    const int64_t total = (int64_t)batch * length;
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int b = (int)(i / length), t = (int)(i % length);
    const int p = t + NFFT / 2;                       // position in the centred (padded) signal
    const int ylen = NFFT + HOP * (frames - 1);
    float y = 0.f, wss = 0.f;
    if (p < ylen) {
        int f0 = (p - NFFT + HOP) / HOP;              // ceil((p - 511) / 128) for p >= 511
        if (p < NFFT - 1) f0 = 0;
        const int f1 = min(frames - 1, p / HOP);
        for (int f = f0; f <= f1; ++f) {
            const int n = p - f * HOP;
            y += fb[((int64_t)b * fstride + f) * NFFT + n];
            const float w = 0.5f - 0.5f * cospif((float)n / 256.f);
            wss += w * w;
        }
        if (wss > 1.17549435e-38f) y /= wss;
    }
    out[i] = y;
}

}  // namespace stft
}  // namespace avse

using namespace avse::stft;

extern "C" {

int64_t avse_stft_frames(int64_t T) { return 1 + T / HOP; }

int avse_stft_fwd(int64_t batch, int64_t T, const float* wave, float* mag, float* spec, avse_stream_t stream) {
    if (!wave || !mag) return AVSE_EINVAL;
    if (batch <= 0 || T <= NFFT / 2 || batch * T > (1LL << 31) - 1) return AVSE_ESHAPE;
    const int frames = (int)avse_stft_frames(T);
    const int64_t nf = batch * frames;
    hipLaunchKernelGGL(stft_kernel, dim3((unsigned)((nf + WAVES - 1) / WAVES)), dim3(THREADS), 0, (hipStream_t)stream,
                       (int)batch, (int)T, frames, wave, mag, spec);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

int avse_istft(int64_t batch, int64_t frames, int64_t length, const float* mag, const float* phase, float* frames_buf,
               float* wave_out, avse_stream_t stream) {
    if (!mag || !phase || !frames_buf || !wave_out) return AVSE_EINVAL;
    if (batch <= 0 || frames <= 0 || length <= 0) return AVSE_ESHAPE;
    // librosa 0.8.1: with length given, only ceil((length + n_fft) / hop) frames are used
    int64_t used = (length + NFFT + HOP - 1) / HOP;
    if (used > frames) used = frames;
    hipStream_t st = (hipStream_t)stream;
    // frames_buf and the inputs keep the full frame stride; only `used` frames are transformed
    // (process all frames: rows are independent and the OLA only reads the first `used`)
    const int64_t nf = batch * frames;
    hipLaunchKernelGGL(istft_frames_kernel, dim3((unsigned)((nf + WAVES - 1) / WAVES)), dim3(THREADS), 0, st,
                       (int)batch, (int)frames, mag, phase, frames_buf);
    AVSE_CHECK_LAUNCH();
    const int64_t tot = batch * length;
    hipLaunchKernelGGL(istft_ola_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (int)batch,
                       (int)frames, (int)used, (int)length, frames_buf, wave_out);
    AVSE_CHECK_LAUNCH();
    return AVSE_OK;
}

}  // extern "C"
