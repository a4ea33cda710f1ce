// VALU throughput micro-benchmark for gfx950: issue rate of v_fma_f32, v_pk_fma_f32, v_exp_f32 and
// mixes, at a chosen number of waves per SIMD.  Prints ns per wave-instruction per SIMD -> cycles.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
#define N_ITER 4096

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, float s) {
    f2 a[8];
    float e[8];
    for (int i = 0; i < 8; ++i) { a[i] = f2{threadIdx.x * 1e-3f + i, s * i}; e[i] = -threadIdx.x * 1e-4f - i * 1e-2f; }
    const f2 m = f2{0.999f, 0.998f}, c = f2{1e-3f, 2e-3f};
    for (int it = 0; it < N_ITER; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (MODE == 0) { a[i].x = __builtin_fmaf(a[i].x, m.x, c.x); }                  // v_fma_f32
            if (MODE == 1) { a[i] = a[i] * m + c; }                                         // v_pk_fma_f32
            if (MODE == 2) { e[i] = __builtin_amdgcn_exp2f(e[i]) - 1.5f; }                 // v_exp + v_sub
            if (MODE == 3) { a[i] = a[i] * m + c; e[i] = __builtin_amdgcn_exp2f(e[i]) - 1.5f; }  // pk_fma + exp + sub
            if (MODE == 4) { e[i] = __builtin_amdgcn_exp2f(e[i]); }                        // v_exp chain
            if (MODE == 5) { a[i].x = __builtin_fmaf(a[i].x, m.x, c.x); a[i].y = __builtin_fmaf(a[i].y, m.y, c.y); }  // 2 fma
        }
    }
    float r = 0.f;
    for (int i = 0; i < 8; ++i) r += a[i].x + a[i].y + e[i];
    if (r == 12345.f) out[threadIdx.x] = r;
}

template <int MODE>
float run(int blocks) {
    float* o;
    hipMalloc(&o, 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, o, 1.f);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, o, 1.f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipFree(o);
    return ms / 5;
}

int main() {
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_exp_f32+v_sub", "pk_fma+exp+sub", "v_exp chain", "2x v_fma_f32"};
    for (int wps = 1; wps <= 4; wps *= 2) {
        const int blocks = 256 * wps;      // 4 waves per block -> wps waves per SIMD
        float ms[6] = {run<0>(blocks), run<1>(blocks), run<2>(blocks), run<3>(blocks), run<4>(blocks), run<5>(blocks)};
        for (int m = 0; m < 6; ++m) {
            // wave-instructions per SIMD (body = 8 ops of the mode per iteration)
            double winst = (double)wps * N_ITER * 8;
            printf("waves/SIMD %d  %-18s %.3f ms  %.2f ns per 8-op group per wave  (%.2f cyc@2.1GHz per group-op)\n", wps,
                   names[m], ms[m], ms[m] * 1e6 / winst, ms[m] * 1e6 / winst * 2.1);
        }
    }
    return 0;
}
