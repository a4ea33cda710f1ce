// HBM access-pattern micro-benchmark for the scan's data movement (tools/ubench, not product code).
// Every workgroup (256 threads) walks 64 rows of a (B*D, L) fp32 matrix in time chunks of TC steps,
// the way the selective scan streams u / delta / z in and out_z back: per chunk it reads TC steps of
// each of its rows from 3 input tensors and writes them (summed) to 1 output tensor.
// Compares run lengths per row (TC * 4 bytes) and access widths against a flat streaming copy.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int TC, int ROWS, int VEC>
__global__ __launch_bounds__(256) void rowwalk(const float* __restrict__ a, const float* __restrict__ b,
                                               const float* __restrict__ c, float* __restrict__ o, int L, int nrows) {
    const int r0 = blockIdx.x * ROWS;
    constexpr int LPR = TC / VEC;                // lanes per row
    constexpr int RPI = 256 / LPR;               // rows per block-instruction
    const int sub = threadIdx.x / LPR, col = (threadIdx.x % LPR) * VEC;
    for (int t0 = 0; t0 + TC <= L; t0 += TC) {
#pragma unroll
        for (int i = 0; i < ROWS / RPI; ++i) {
            const int r = r0 + i * RPI + sub;
            const size_t off = (size_t)r * L + t0 + col;
            if constexpr (VEC == 4) {
                const float4 x = *reinterpret_cast<const float4*>(a + off);
                const float4 y = *reinterpret_cast<const float4*>(b + off);
                const float4 z = *reinterpret_cast<const float4*>(c + off);
                *reinterpret_cast<float4*>(o + off) = make_float4(x.x + y.x + z.x, x.y + y.y + z.y, x.z + y.z + z.z,
                                                                  x.w + y.w + z.w);
            } else {
                o[off] = a[off] + b[off] + c[off];
            }
        }
    }
}

__global__ void flatcopy(const float4* __restrict__ a, const float4* __restrict__ b, const float4* __restrict__ c,
                         float4* __restrict__ o, size_t n4) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const float4 x = a[i], y = b[i], z = c[i];
        o[i] = make_float4(x.x + y.x + z.x, x.y + y.y + z.y, x.z + y.z + z.z, x.w + y.w + z.w);
    }
}

template <typename F>
float timeit(F f) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    f();
    hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) f();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    const int B = 64, D = 1024, L = 4096;          // L a multiple of every TC (aligned rows)
    const size_t n = (size_t)B * D * L;
    float *a, *b, *c, *o;
    if (hipMalloc(&a, n * 4) || hipMalloc(&b, n * 4) || hipMalloc(&c, n * 4) || hipMalloc(&o, n * 4)) return 1;
    if (hipMemset(a, 0, n * 4) || hipMemset(b, 0, n * 4) || hipMemset(c, 0, n * 4)) return 1;
    const double gb = 4.0 * n * 4 / 1e9;
    const int nrows = B * D;
    float ms = timeit([&] { hipLaunchKernelGGL(flatcopy, dim3(4096), dim3(256), 0, 0, (const float4*)a, (const float4*)b,
                                               (const float4*)c, (float4*)o, n / 4); });
    printf("flat streaming x4            %.3f ms  %.0f GB/s\n", ms, gb / ms * 1e3);
#define RUN(TC, VEC)                                                                                         \
    ms = timeit([&] { hipLaunchKernelGGL((rowwalk<TC, 64, VEC>), dim3(nrows / 64), dim3(256), 0, 0, a, b, c, o, L, nrows); }); \
    printf("rowwalk 64 rows TC=%-4d vec=%d  %.3f ms  %.0f GB/s\n", TC, VEC, ms, gb / ms * 1e3);
    RUN(64, 1) RUN(64, 4) RUN(128, 1) RUN(128, 4) RUN(256, 4) RUN(512, 4) RUN(1024, 4)
    return 0;
}
